// Implicit-GEMM convolution on CDNA4 MFMA (gfx950).
//
// Replaces the nn.Conv2d / nn.Conv3d forward and backward the reference runs on
// every train step (edsr_net.py:28-64, duf_net.py:35-49,116-214,
// drf_net.py:55-147; backward via loss.backward(), base_trainer.py:128).
//
// Layout: activations channels-last (N,D,H,W,C) in bf16 or fp32; weights
// pre-packed [kd][kh][kw][cout_pad][cin_pad].  One workgroup (4 waves) owns an
// output tile of 8 rows x 32 columns of one (n, d) slice and NT output
// channels.  Per (kd, 32-channel chunk) stage it copies the input tile plus its
// (kh-1, kw-1) halo and the stage's weights into LDS (80-byte rows: 64 data +
// 16 pad, conflict-free for ds_read_b128 column slices), then runs all kh*kw
// taps out of LDS.  MFMA orientation is "weights x voxels" so that each lane's
// accumulator column is one voxel and its registers hold 4 consecutive output
// channels -> 8/16-byte channels-last stores.
//   bf16: v_mfma_f32_32x32x16_bf16, one per 16 channels.
//   fp32: v_mfma_f32_32x32x2_f32, four per 8 channels (exact fp32, parity path).
#include "vsrk_common.h"
#include "vsrk_internal.h"

namespace {

constexpr int TH = 8;
constexpr int TW = 32;
constexpr int ROWB = 80;  // LDS bytes per staged voxel/weight row

struct ConvArgs {
  View x, y, res, msk;
  const char* w;
  const float* bias;
  const float* pro_scale;
  const float* pro_shift;
  int cin, cout, cin_pad, cout_pad;
  int kd, kh, kw, pd, ph, pw;
  int prologue, act, accumulate, has_res, has_mask, xvec, bias_r;
  float out_scale;
  int tiles_h, tiles_w;
};

// Load the 16-byte chunk of channels [c, c+E) of voxel `off` (element offset of
// channel c).  Vector load when the view allows it, else element loads with
// zero fill past `cin` (1-channel head/tail convs).  The prologue is applied
// to real channels only: zero padding stays zero.
template <typename T>
__device__ __forceinline__ uint4 load_chunk(const char* base, int64_t off, int c, int cin, bool vec, int mode,
                                            const float* sc, const float* sh);

template <typename T>
__device__ __forceinline__ uint4 apply_prologue(uint4 v, int c, int mode, const float* sc,
                                                const float* sh) {
  constexpr int E = Chunk<T>::E;
  float f[E];
  Chunk<T>::unpack(v, f);
  if (mode & VSRK_PRO_AFFINE) {
#pragma unroll
    for (int e = 0; e < E; ++e) f[e] = fmaf(f[e], sc[c + e], sh[c + e]);
  }
  if (mode & VSRK_PRO_RELU) {
#pragma unroll
    for (int e = 0; e < E; ++e) f[e] = fmaxf(f[e], 0.f);
  }
  return Chunk<T>::pack(f);
}

template <typename T>
__device__ __forceinline__ uint4 load_chunk(const char* base, int64_t off, int c, int cin, bool vec, int mode,
                                            const float* sc, const float* sh) {
  constexpr int E = Chunk<T>::E;
  const T* p = reinterpret_cast<const T*>(base) + off;
  if (vec && c + E <= cin) {
    uint4 v = *reinterpret_cast<const uint4*>(p);
    return mode ? apply_prologue<T>(v, c, mode, sc, sh) : v;
  }
  float f[E];
#pragma unroll
  for (int e = 0; e < E; ++e) {
    float t = 0.f;
    if (c + e < cin) {
      t = to_f32<T>(p[e]);
      if (mode & VSRK_PRO_AFFINE) t = fmaf(t, sc[c + e], sh[c + e]);
      if (mode & VSRK_PRO_RELU) t = fmaxf(t, 0.f);
    }
    f[e] = t;
  }
  return Chunk<T>::pack(f);
}

// acc += W(32 rows of co, 16-byte k slice) x X(16-byte k slice, 32 voxels)
template <typename T>
__device__ __forceinline__ void mma(f32x16& acc, uint4 a, uint4 b);
template <>
__device__ __forceinline__ void mma<bf16>(f32x16& acc, uint4 a, uint4 b) {
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a),
                                                __builtin_bit_cast(bf16x8, b), acc, 0, 0, 0);
}
template <>
__device__ __forceinline__ void mma<float>(f32x16& acc, uint4 a, uint4 b) {
  // lane half hf supplies k = 4*hf + j for MFMA j on both operands, so the
  // four k=2 products cover the 8 channels of the slice exactly once.
  acc = __builtin_amdgcn_mfma_f32_32x32x2f32(__builtin_bit_cast(float, a.x), __builtin_bit_cast(float, b.x), acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x2f32(__builtin_bit_cast(float, a.y), __builtin_bit_cast(float, b.y), acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x2f32(__builtin_bit_cast(float, a.z), __builtin_bit_cast(float, b.z), acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x2f32(__builtin_bit_cast(float, a.w), __builtin_bit_cast(float, b.w), acc, 0, 0, 0);
}

template <typename YT>
__device__ __forceinline__ void load4(const char* base, int64_t off, bool vec, int valid, float* v) {
  const YT* p = reinterpret_cast<const YT*>(base) + off;
  if (vec) {
    if constexpr (sizeof(YT) == 4) {
      float4 t = *reinterpret_cast<const float4*>(p);
      v[0] = t.x; v[1] = t.y; v[2] = t.z; v[3] = t.w;
    } else {
      uint2 t = *reinterpret_cast<const uint2*>(p);
      const bf16* b = reinterpret_cast<const bf16*>(&t);
      for (int e = 0; e < 4; ++e) v[e] = (float)b[e];
    }
  } else {
    for (int e = 0; e < 4; ++e) v[e] = e < valid ? to_f32<YT>(p[e]) : 0.f;
  }
}

template <typename T, int NT, typename YT>
__global__ __launch_bounds__(256) void conv_fwd_kernel(ConvArgs a) {
  constexpr int NS = NT / 32;
  constexpr int E = Chunk<T>::E;
  constexpr int CK = 4 * E;  // channels per stage: 64 bytes
  extern __shared__ __attribute__((aligned(16))) char lds[];

  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, r = lane & 31, hf = lane >> 5;
  int bid = blockIdx.x;
  const int tw_i = bid % a.tiles_w;
  bid /= a.tiles_w;
  const int th_i = bid % a.tiles_h;
  bid /= a.tiles_h;
  const int dz = bid % a.y.d;
  const int nb = bid / a.y.d;
  const int h0 = th_i * TH, w0 = tw_i * TW;
  const int n0 = blockIdx.y * NT;
  const int HWd = TW + a.kw - 1;
  const int HHd = TH + a.kh - 1;
  const int slots = HHd * HWd;
  const int taps2 = a.kh * a.kw;
  char* ldsA = lds;
  char* ldsB = lds + slots * ROWB;

  f32x16 acc[2][NS];
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int n = 0; n < NS; ++n)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[m][n][i] = 0.f;

  for (int kdi = 0; kdi < a.kd; ++kdi) {
    const int di = dz + kdi - a.pd;
    if (di < 0 || di >= a.x.d) continue;  // block-uniform
    for (int c0 = 0; c0 < a.cin; c0 += CK) {
      __syncthreads();
      for (int q = tid; q < slots * 4; q += 256) {
        const int slot = q >> 2, part = q & 3;
        const int hh = slot / HWd, ww = slot - hh * HWd;
        const int hi = h0 + hh - a.ph, wi = w0 + ww - a.pw;
        const int c = c0 + part * E;
        uint4 v = make_uint4(0, 0, 0, 0);
        if (hi >= 0 && hi < a.x.h && wi >= 0 && wi < a.x.w && c < a.cin)
          v = load_chunk<T>(a.x.ptr, view_off(a.x, nb, di, hi, wi, c), c, a.cin, a.xvec, a.prologue, a.pro_scale,
                            a.pro_shift);
        *reinterpret_cast<uint4*>(ldsA + slot * ROWB + part * 16) = v;
      }
      const int brows = taps2 * NT;
      for (int q = tid; q < brows * 4; q += 256) {
        const int row = q >> 2, part = q & 3;
        const int tap = row / NT, nn = row - tap * NT;
        const int co = n0 + nn;
        uint4 v = make_uint4(0, 0, 0, 0);
        if (co < a.cout_pad) {
          const int64_t idx = ((int64_t)(kdi * taps2 + tap) * a.cout_pad + co) * a.cin_pad + c0 + part * E;
          v = *reinterpret_cast<const uint4*>(a.w + idx * sizeof(T));
        }
        *reinterpret_cast<uint4*>(ldsB + row * ROWB + part * 16) = v;
      }
      __syncthreads();
      for (int tap = 0; tap < taps2; ++tap) {
        const int khi = tap / a.kw, kwi = tap - khi * a.kw;
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          uint4 bx[2], aw[NS];
#pragma unroll
          for (int ms = 0; ms < 2; ++ms) {
            const int slot = (wave * 2 + ms + khi) * HWd + r + kwi;
            bx[ms] = *reinterpret_cast<const uint4*>(ldsA + slot * ROWB + ks * 32 + hf * 16);
          }
#pragma unroll
          for (int ns = 0; ns < NS; ++ns)
            aw[ns] = *reinterpret_cast<const uint4*>(ldsB + (tap * NT + ns * 32 + r) * ROWB + ks * 32 + hf * 16);
#pragma unroll
          for (int ms = 0; ms < 2; ++ms)
#pragma unroll
            for (int ns = 0; ns < NS; ++ns) mma<T>(acc[ms][ns], aw[ns], bx[ms]);
        }
      }
    }
  }

  // epilogue: acc[ms][ns][4g+e] = (co = n0 + ns*32 + 8g + 4hf + e, voxel column r)
#pragma unroll
  for (int ms = 0; ms < 2; ++ms) {
    const int ho = h0 + wave * 2 + ms, wo = w0 + r;
    if (ho >= a.y.h || wo >= a.y.w) continue;
#pragma unroll
    for (int ns = 0; ns < NS; ++ns) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int co = n0 + ns * 32 + 8 * g + 4 * hf;
        if (co >= a.cout) continue;
        const int valid = min(4, a.cout - co);
        float v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float t = acc[ms][ns][4 * g + e];
          if (a.bias && e < valid) {
            int cb = co + e;
            if (a.bias_r > 1) {  // view order (sub, c') -> torch order c'*r*r + sub
              const int rr = a.bias_r * a.bias_r, cp = a.cout / rr;
              const int sub = cb / cp;
              cb = (cb - sub * cp) * rr + sub;
            }
            t += a.bias[cb];
          }
          t *= a.out_scale;
          if (a.act == VSRK_ACT_RELU) t = fmaxf(t, 0.f);
          v[e] = t;
        }
        const int64_t yo = view_off(a.y, nb, dz, ho, wo, co);
        const bool vec = (valid == 4) && ((yo & 3) == 0) &&
                         ((((uintptr_t)a.y.ptr) & (4 * sizeof(YT) - 1)) == 0);
        if (a.has_mask) {
          float m[4];
          load4<YT>(a.msk.ptr, view_off(a.msk, nb, dz, ho, wo, co), vec, valid, m);
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = m[e] > 0.f ? v[e] : 0.f;
        }
        if (a.has_res) {
          float rr[4];
          load4<YT>(a.res.ptr, view_off(a.res, nb, dz, ho, wo, co), vec, valid, rr);
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] += rr[e];
        }
        if (a.accumulate) {
          float o[4];
          load4<YT>(a.y.ptr, yo, vec, valid, o);
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] += o[e];
        }
        YT* yp = reinterpret_cast<YT*>(a.y.ptr) + yo;
        if (vec) {
          if constexpr (sizeof(YT) == 4) {
            *reinterpret_cast<float4*>(yp) = make_float4(v[0], v[1], v[2], v[3]);
          } else {
            uint2 t;
            bf16* b = reinterpret_cast<bf16*>(&t);
            for (int e = 0; e < 4; ++e) b[e] = (bf16)v[e];
            *reinterpret_cast<uint2*>(yp) = t;
          }
        } else {
          for (int e = 0; e < valid; ++e) yp[e] = from_f32<YT>(v[e]);
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------
// weight packing
// ---------------------------------------------------------------------------
template <typename T>
__global__ void pack_weight_kernel(const float* __restrict__ w, T* __restrict__ out, int cout, int cin,
                                   int kd, int kh, int kw, int mode, int perm_r, int co_pad,
                                   int ci_pad, int64_t total) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= total) return;
  // out index = ((tap * co_pad + o) * ci_pad + i) in the packed (primed) roles
  const int i = idx % ci_pad;
  const int64_t t1 = idx / ci_pad;
  const int o = t1 % co_pad;
  const int tap = t1 / co_pad;
  const int kwi = tap % kw, khi = (tap / kw) % kh, kdi = tap / (kw * kh);
  int co, ci, sd, sh, sw;
  if (mode == 0) {
    co = o; ci = i; sd = kdi; sh = khi; sw = kwi;
  } else {
    co = i; ci = o; sd = kd - 1 - kdi; sh = kh - 1 - khi; sw = kw - 1 - kwi;
  }
  float v = 0.f;
  if (co < cout && ci < cin) {
    int cot = co;
    if (perm_r > 1) {  // view order (sub, c') -> torch order c'*r*r + sub
      const int rr = perm_r * perm_r, cp = cout / rr;
      const int sub = co / cp, cc = co - sub * cp;
      cot = cc * rr + sub;
    }
    v = w[((((int64_t)cot * cin + ci) * kd + sd) * kh + sh) * kw + sw];
  }
  out[idx] = from_f32<T>(v);
}

// ---------------------------------------------------------------------------
// weight gradient
// ---------------------------------------------------------------------------
// Grid: x = split s (range of output tiles), y = combo (co tile, ci chunk, kd).
// Each workgroup stages a 8x32 dY tile (32 output channels) and the matching
// input halo (32 input channels, prologue applied) and accumulates
// dW[tap][co][ci] over its tiles with the voxel index as the MFMA k dimension
// (transposed LDS reads: ds_read_b64_tr_b16).  Waves split the voxels; the
// four wave partials are summed through LDS and stored as one fp32 slab per
// (split, combo); wgrad_reduce sums slabs in split order -> deterministic.
struct WgradArgs {
  View x, dy;
  const float* pro_scale;
  const float* pro_shift;
  float* ws;
  int cin, cout;
  int kd, kh, kw, pd, ph, pw;
  int prologue, xvec, dyvec;
  int tiles_h, tiles_w, ntiles;
  int tiles_per_split;
  int n_ci_chunks, n_co_tiles;
};

typedef short v4i16 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4i16 lds_v4i16;

__device__ __forceinline__ v4i16 ds_read_tr(const char* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)(p));
}

template <typename T>
__global__ __launch_bounds__(256) void conv_wgrad_kernel(WgradArgs a) {
  constexpr int E = Chunk<T>::E;
  constexpr int RB = 32 * (int)sizeof(T);  // bytes per staged row: 32 channels
  constexpr int CPR = RB / 16;             // 16-byte chunks per row
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int HWd = TW + a.kw - 1, HHd = TH + a.kh - 1, slots = HHd * HWd;
  const int taps2 = a.kh * a.kw;
  char* ldsY = lds;                   // [256 voxels][32 co]
  char* ldsX = lds + TH * TW * RB;    // [slots][32 ci]

  int combo = blockIdx.y;
  const int cot = combo % a.n_co_tiles;
  combo /= a.n_co_tiles;
  const int cic = combo % a.n_ci_chunks;
  const int kdi = combo / a.n_ci_chunks;
  const int co0 = cot * 32, ci0 = cic * 32;

  f32x16 acc[9];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[t][i] = 0.f;

  const int t_begin = blockIdx.x * a.tiles_per_split;
  const int t_end = min(a.ntiles, t_begin + a.tiles_per_split);
  for (int t = t_begin; t < t_end; ++t) {
    int b = t;
    const int tw_i = b % a.tiles_w;
    b /= a.tiles_w;
    const int th_i = b % a.tiles_h;
    b /= a.tiles_h;
    const int dz = b % a.dy.d;
    const int nb = b / a.dy.d;
    const int di = dz + kdi - a.pd;
    if (di < 0 || di >= a.x.d) continue;
    const int h0 = th_i * TH, w0 = tw_i * TW;
    __syncthreads();
    // stage dY tile (zero outside the output / beyond cout)
    for (int q = tid; q < TH * TW * CPR; q += 256) {
      const int vox = q / CPR, part = q - vox * CPR;
      const int ho = h0 + vox / TW, wo = w0 + (vox % TW);
      const int c = co0 + part * E;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (ho < a.dy.h && wo < a.dy.w && c < a.cout)
        v = load_chunk<T>(a.dy.ptr, view_off(a.dy, nb, dz, ho, wo, c), c, a.cout, a.dyvec, 0, nullptr, nullptr);
      *reinterpret_cast<uint4*>(ldsY + vox * RB + part * 16) = v;
    }
    for (int q = tid; q < slots * CPR; q += 256) {
      const int slot = q / CPR, part = q - slot * CPR;
      const int hh = slot / HWd, ww = slot - hh * HWd;
      const int hi = h0 + hh - a.ph, wi = w0 + ww - a.pw;
      const int c = ci0 + part * E;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (hi >= 0 && hi < a.x.h && wi >= 0 && wi < a.x.w && c < a.cin)
        v = load_chunk<T>(a.x.ptr, view_off(a.x, nb, di, hi, wi, c), c, a.cin, a.xvec, a.prologue, a.pro_scale,
                          a.pro_shift);
      *reinterpret_cast<uint4*>(ldsX + slot * RB + part * 16) = v;
    }
    __syncthreads();
    if constexpr (sizeof(T) == 2) {
      // k = voxel.  Group g = lane>>4 reads a 4-row x 16-column block; lane
      // 4q+p addresses row q, columns 4p..4p+3; it receives column (lane&15).
      const int g = lane >> 4, i16 = lane & 15, q = i16 >> 2, p = i16 & 3;
      const int hfk = g >> 1, colb = (g & 1) * 16 + 4 * p;
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        const int vrow = wave * 2 + (ks >> 1);       // tile row of these 16 voxels
        const int vcol0 = (ks & 1) * 16 + 8 * hfk;  // first voxel column of this lane half
        v4i16 y0 = ds_read_tr(ldsY + (vrow * TW + vcol0 + q) * RB + colb * 2);
        v4i16 y1 = ds_read_tr(ldsY + (vrow * TW + vcol0 + 4 + q) * RB + colb * 2);
        bf16x8 af = __builtin_bit_cast(bf16x8, __builtin_shufflevector(y0, y1, 0, 1, 2, 3, 4, 5, 6, 7));
#pragma unroll
        for (int tap = 0; tap < 9; ++tap) {
          if (tap < taps2) {
            const int khi = tap / a.kw, kwi = tap - (tap / a.kw) * a.kw;
            const int s0 = (vrow + khi) * HWd + vcol0 + kwi;
            v4i16 x0 = ds_read_tr(ldsX + (s0 + q) * RB + colb * 2);
            v4i16 x1 = ds_read_tr(ldsX + (s0 + 4 + q) * RB + colb * 2);
            bf16x8 bfr = __builtin_bit_cast(bf16x8, __builtin_shufflevector(x0, x1, 0, 1, 2, 3, 4, 5, 6, 7));
            acc[tap] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af, bfr, acc[tap], 0, 0, 0);
          }
        }
      }
    } else {
      // fp32: 32x32x2, lane l: A[co=l&31][k=l>>5], B[k=l>>5][ci=l&31]
      const int r = lane & 31, hfk = lane >> 5;
      for (int kk = 0; kk < 64; kk += 2) {
        const int vox = wave * 64 + kk + hfk;
        const int vrow = vox / TW, vcol = vox % TW;
        const float av = *reinterpret_cast<const float*>(ldsY + vox * RB + r * 4);
#pragma unroll
        for (int tap = 0; tap < 9; ++tap) {
          if (tap < taps2) {
            const int khi = tap / a.kw, kwi = tap - (tap / a.kw) * a.kw;
            const int s = (vrow + khi) * HWd + vcol + kwi;
            const float bv = *reinterpret_cast<const float*>(ldsX + s * RB + r * 4);
            acc[tap] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bv, acc[tap], 0, 0, 0);
          }
        }
      }
    }
  }
  // sum the four wave partials through LDS (fixed order), store the slab
  __syncthreads();
  float* red = reinterpret_cast<float*>(lds);
  const int r = lane & 31, hfo = lane >> 5;
  for (int w = 0; w < 4; ++w) {
    if (wave == w) {
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) {
        if (tap < taps2) {
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            const int co = (i & 3) + 8 * (i >> 2) + 4 * hfo;
            float* dst = red + (tap * 32 + co) * 32 + r;
            *dst = (w == 0) ? acc[tap][i] : *dst + acc[tap][i];
          }
        }
      }
    }
    __syncthreads();
  }
  const int slab = taps2 * 1024;
  float* out = a.ws + ((int64_t)blockIdx.x * gridDim.y + blockIdx.y) * slab;
  for (int i = tid; i < slab; i += 256) out[i] = red[i];
}

// dw[co][ci][kd][kh][kw] (torch, fp32) = scale * sum_s slab[s][combo][tap][co%32][ci%32]
__global__ void wgrad_reduce_kernel(const float* __restrict__ ws, float* __restrict__ dw, int splits,
                                    int ncombos, int cout, int cin, int kd, int kh, int kw,
                                    int n_co_tiles, int n_ci_chunks, int perm_r, float scale,
                                    int accumulate) {
  const int64_t total = (int64_t)cout * cin * kd * kh * kw;
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= total) return;
  // enumerate in slab-friendly order: idx -> (kdi, combo-local, tap, co, ci)
  const int taps2 = kh * kw;
  const int ci = idx % cin;
  int64_t t = idx / cin;
  const int co = t % cout;
  t /= cout;
  const int tap = t % taps2;
  const int kdi = t / taps2;
  const int combo = (kdi * n_ci_chunks + ci / 32) * n_co_tiles + co / 32;
  const int slab = taps2 * 1024;
  const float* p = ws + (int64_t)combo * slab + (tap * 32 + (co % 32)) * 32 + (ci % 32);
  float s = 0.f;
  for (int k = 0; k < splits; ++k) s += p[(int64_t)k * ncombos * slab];
  int cot = co;
  if (perm_r > 1) {
    const int rr = perm_r * perm_r, cp = cout / rr;
    const int sub = co / cp, cc = co - sub * cp;
    cot = cc * rr + sub;
  }
  const int khi = tap / kw, kwi = tap % kw;
  float* d = dw + ((((int64_t)cot * cin + ci) * kd + kdi) * kh + khi) * kw + kwi;
  s *= scale;
  *d = accumulate ? *d + s : s;
}

}  // namespace

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
// Can the kernels read this view in 16-byte chunks?  (aligned base, strides
// and channel count multiples of one chunk; sub-pixel blocks chunk-aligned)
static bool chunk_ok(const vsrk_tensor5* t, int esize) {
  const int epc = 16 / esize;
  const int r = t->shuffle > 1 ? t->shuffle : 1;
  return ((uintptr_t)t->ptr) % 16 == 0 && t->sn % epc == 0 && t->sd % epc == 0 && t->sh % epc == 0 &&
         t->sw % epc == 0 && (t->c / (r * r)) % epc == 0;
}

static bool view_ok(const vsrk_tensor5* t, const char* what) {
  if (!t || !t->ptr) {
    vsrk_set_error("%s: null view", what);
    return false;
  }
  const int r = t->shuffle > 1 ? t->shuffle : 1;
  if (t->c % (r * r) != 0 || (r > 1 && (t->c / (r * r)) % 8 != 0)) {
    vsrk_set_error("%s: sub-pixel view needs channels divisible by 8*shuffle^2 (c=%d, r=%d)", what, t->c, r);
    return false;
  }
  return true;
}

extern "C" size_t vsrk_conv_packed_elems(int32_t cout, int32_t cin, int32_t kd, int32_t kh, int32_t kw,
                                         int32_t mode) {
  const int co = mode == 0 ? cout : cin, ci = mode == 0 ? cin : cout;
  return (size_t)kd * kh * kw * round_up(co, 32) * round_up(ci, 32);
}

extern "C" int vsrk_conv_pack_weight(int32_t dtype, const float* w, int32_t cout, int32_t cin, int32_t kd,
                                     int32_t kh, int32_t kw, int32_t mode, int32_t perm_r, void* packed,
                                     void* stream) {
  VSRK_CHECK(w && packed, "conv_pack_weight: null pointer");
  VSRK_CHECK(mode == 0 || mode == 1, "conv_pack_weight: mode must be 0 or 1");
  VSRK_CHECK(perm_r <= 1 || cout % (perm_r * perm_r) == 0, "conv_pack_weight: cout %% r^2 != 0");
  const int co = mode == 0 ? cout : cin, ci = mode == 0 ? cin : cout;
  const int co_pad = round_up(co, 32), ci_pad = round_up(ci, 32);
  const int64_t total = (int64_t)kd * kh * kw * co_pad * ci_pad;
  const int blk = 256;
  const int grid = (int)ceil_div64(total, blk);
  hipStream_t s = (hipStream_t)stream;
  if (dtype == VSRK_BF16)
    pack_weight_kernel<bf16><<<grid, blk, 0, s>>>(w, (bf16*)packed, cout, cin, kd, kh, kw, mode, perm_r,
                                                  co_pad, ci_pad, total);
  else
    pack_weight_kernel<float><<<grid, blk, 0, s>>>(w, (float*)packed, cout, cin, kd, kh, kw, mode, perm_r,
                                                   co_pad, ci_pad, total);
  VSRK_LAUNCH_CHECK("conv_pack_weight");
  return VSRK_OK;
}

template <typename T, int NT, typename YT>
static int launch_fwd(const ConvArgs& a, int grid_x, hipStream_t s) {
  const int slots = (TH + a.kh - 1) * (TW + a.kw - 1);
  const size_t lds = (size_t)slots * ROWB + (size_t)a.kh * a.kw * NT * ROWB;
  auto kern = conv_fwd_kernel<T, NT, YT>;
  if (lds > 64 * 1024) (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  dim3 grid(grid_x, ceil_div(a.cout, NT));
  kern<<<grid, 256, lds, s>>>(a);
  VSRK_LAUNCH_CHECK("conv_fwd");
  return VSRK_OK;
}

extern "C" int vsrk_conv_fwd(const vsrk_conv_desc* d, const vsrk_tensor5* x, const void* w_packed,
                             const float* bias, const float* pro_scale, const float* pro_shift,
                             const vsrk_tensor5* residual, const vsrk_tensor5* mask, const vsrk_tensor5* y,
                             void* stream) {
  VSRK_CHECK(d && x && y && w_packed, "conv_fwd: null argument");
  const int xdt = x->dtype, ydt = y->dtype;
  VSRK_CHECK(xdt == VSRK_F32 || xdt == VSRK_BF16, "conv_fwd: bad x dtype");
  VSRK_CHECK(ydt == xdt || ydt == VSRK_F32, "conv_fwd: y dtype must equal x dtype or be f32");
  const int es = xdt == VSRK_BF16 ? 2 : 4;
  if (!view_ok(x, "conv_fwd x") || !view_ok(y, "conv_fwd y")) return VSRK_ERR_INVALID;
  VSRK_CHECK(y->ptr, "conv_fwd: null y");
  VSRK_CHECK(d->kh >= 1 && d->kh <= 3 && d->kw >= 1 && d->kw <= 3 && d->kd >= 1,
             "conv_fwd: kernel %dx%dx%d unsupported (kh,kw <= 3)", d->kd, d->kh, d->kw);
  VSRK_CHECK(x->n == y->n, "conv_fwd: batch mismatch");
  VSRK_CHECK(!(d->prologue & VSRK_PRO_AFFINE) || (pro_scale && pro_shift), "conv_fwd: affine prologue needs scale/shift");
  const int yr = y->shuffle > 1 ? y->shuffle : 1;
  VSRK_CHECK(yr == 1 || (y->c / (yr * yr)) % 4 == 0, "conv_fwd: shuffled output needs c/r^2 %% 4 == 0");
  if (residual) {
    VSRK_CHECK(residual->dtype == ydt && residual->c == y->c && residual->h == y->h && residual->w == y->w,
               "conv_fwd: residual view mismatch");
  }
  if (mask) {
    VSRK_CHECK(mask->dtype == ydt && mask->c == y->c && mask->h == y->h && mask->w == y->w,
               "conv_fwd: mask view mismatch");
  }
  ConvArgs a;
  a.x = make_view(x);
  a.y = make_view(y);
  if (residual) a.res = make_view(residual); else a.res = a.y;
  if (mask) a.msk = make_view(mask); else a.msk = a.y;
  a.w = (const char*)w_packed;
  a.bias = bias;
  a.pro_scale = pro_scale;
  a.pro_shift = pro_shift;
  a.cin = x->c;
  a.cout = y->c;
  a.cin_pad = round_up(x->c, 32);
  a.cout_pad = round_up(y->c, 32);
  a.kd = d->kd; a.kh = d->kh; a.kw = d->kw;
  a.pd = d->pd; a.ph = d->ph; a.pw = d->pw;
  a.prologue = d->prologue;
  a.act = d->act;
  a.accumulate = d->accumulate;
  a.has_res = residual != nullptr;
  a.has_mask = mask != nullptr;
  a.xvec = chunk_ok(x, es);
  a.bias_r = d->bias_perm_r;
  a.out_scale = d->out_scale;
  a.tiles_h = ceil_div(y->h, TH);
  a.tiles_w = ceil_div(y->w, TW);
  const int64_t gx = (int64_t)y->n * y->d * a.tiles_h * a.tiles_w;
  VSRK_CHECK(gx < (1ll << 31), "conv_fwd: grid too large");
  hipStream_t s = (hipStream_t)stream;
  const int NT = y->c <= 32 ? 32 : (y->c <= 64 ? 64 : 128);
  if (xdt == VSRK_BF16) {
    if (ydt == VSRK_BF16) {
      if (NT == 32) return launch_fwd<bf16, 32, bf16>(a, (int)gx, s);
      if (NT == 64) return launch_fwd<bf16, 64, bf16>(a, (int)gx, s);
      return launch_fwd<bf16, 128, bf16>(a, (int)gx, s);
    }
    if (NT == 32) return launch_fwd<bf16, 32, float>(a, (int)gx, s);
    if (NT == 64) return launch_fwd<bf16, 64, float>(a, (int)gx, s);
    return launch_fwd<bf16, 128, float>(a, (int)gx, s);
  }
  if (NT == 32) return launch_fwd<float, 32, float>(a, (int)gx, s);
  if (NT == 64) return launch_fwd<float, 64, float>(a, (int)gx, s);
  return launch_fwd<float, 128, float>(a, (int)gx, s);
}

static void wgrad_plan(const vsrk_conv_desc* d, const vsrk_tensor5* x, const vsrk_tensor5* dy, int* splits,
                       int* tps, int* ncombos, int* ntiles, int* nco, int* nci) {
  const int th = ceil_div(dy->h, TH), tw = ceil_div(dy->w, TW);
  *ntiles = dy->n * dy->d * th * tw;
  *nco = ceil_div(dy->c, 32);
  *nci = ceil_div(x->c, 32);
  *ncombos = *nco * *nci * d->kd;
  // aim for ~2048 workgroups in total
  int want = ceil_div(2048, *ncombos);
  if (want < 1) want = 1;
  if (want > *ntiles) want = *ntiles;
  *tps = ceil_div(*ntiles, want);
  *splits = ceil_div(*ntiles, *tps);
}

extern "C" size_t vsrk_conv_wgrad_workspace_size(const vsrk_conv_desc* d, const vsrk_tensor5* x,
                                                 const vsrk_tensor5* dy) {
  int splits, tps, ncombos, ntiles, nco, nci;
  wgrad_plan(d, x, dy, &splits, &tps, &ncombos, &ntiles, &nco, &nci);
  const size_t slab = (size_t)splits * ncombos * d->kh * d->kw * 1024 * sizeof(float);
  return std::max(slab, vsrk_channel_reduce_ws_bytes(dy->c));
}

extern "C" int vsrk_conv_wgrad(const vsrk_conv_desc* d, const vsrk_tensor5* x, const vsrk_tensor5* dy,
                               const float* pro_scale, const float* pro_shift, float dy_scale, int32_t perm_r,
                               float* dw, float* dbias, int32_t accumulate, void* workspace,
                               size_t workspace_bytes, void* stream) {
  VSRK_CHECK(d && x && dy && dw, "conv_wgrad: null argument");
  VSRK_CHECK(x->dtype == dy->dtype, "conv_wgrad: x/dy dtype mismatch");
  const int es = x->dtype == VSRK_BF16 ? 2 : 4;
  if (!view_ok(x, "conv_wgrad x") || !view_ok(dy, "conv_wgrad dy")) return VSRK_ERR_INVALID;
  VSRK_CHECK(d->kh >= 1 && d->kh <= 3 && d->kw >= 1 && d->kw <= 3, "conv_wgrad: kh,kw <= 3");
  VSRK_CHECK(!(d->prologue & VSRK_PRO_AFFINE) || (pro_scale && pro_shift), "conv_wgrad: affine prologue needs scale/shift");
  int splits, tps, ncombos, ntiles, nco, nci;
  wgrad_plan(d, x, dy, &splits, &tps, &ncombos, &ntiles, &nco, &nci);
  const size_t need = vsrk_conv_wgrad_workspace_size(d, x, dy);
  VSRK_CHECK(workspace && workspace_bytes >= need, "conv_wgrad: workspace %zu < %zu bytes", workspace_bytes, need);
  WgradArgs a;
  a.x = make_view(x);
  a.dy = make_view(dy);
  a.pro_scale = pro_scale;
  a.pro_shift = pro_shift;
  a.ws = (float*)workspace;
  a.cin = x->c;
  a.cout = dy->c;
  a.kd = d->kd; a.kh = d->kh; a.kw = d->kw;
  a.pd = d->pd; a.ph = d->ph; a.pw = d->pw;
  a.prologue = d->prologue;
  a.xvec = chunk_ok(x, es);
  a.dyvec = chunk_ok(dy, es);
  a.tiles_h = ceil_div(dy->h, TH);
  a.tiles_w = ceil_div(dy->w, TW);
  a.ntiles = ntiles;
  a.tiles_per_split = tps;
  a.n_ci_chunks = nci;
  a.n_co_tiles = nco;
  const int slots = (TH + d->kh - 1) * (TW + d->kw - 1);
  const size_t lds = (size_t)(TH * TW + slots) * 32 * es;
  hipStream_t s = (hipStream_t)stream;
  dim3 grid(splits, ncombos);
  if (x->dtype == VSRK_BF16) {
    conv_wgrad_kernel<bf16><<<grid, 256, lds, s>>>(a);
  } else {
    auto kern = conv_wgrad_kernel<float>;
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    kern<<<grid, 256, lds, s>>>(a);
  }
  VSRK_LAUNCH_CHECK("conv_wgrad");
  const int64_t total = (int64_t)dy->c * x->c * d->kd * d->kh * d->kw;
  wgrad_reduce_kernel<<<(int)ceil_div64(total, 256), 256, 0, s>>>(
      (const float*)workspace, dw, splits, ncombos, dy->c, x->c, d->kd, d->kh, d->kw, nco, nci, perm_r, dy_scale,
      accumulate);
  VSRK_LAUNCH_CHECK("conv_wgrad_reduce");
  if (dbias) {
    // the slab has been consumed by the reduce above (stream order): reuse it
    int rc = vsrk_channel_reduce_internal(dy, 0, perm_r, dy_scale, dbias, nullptr, accumulate, workspace,
                                          workspace_bytes, s);
    if (rc) return rc;
  }
  return VSRK_OK;
}
