// Convolutions with a thin channel side, where the implicit-GEMM kernels
// (conv_fwd.hip / conv_fast.hip / conv_wgrad.hip) would pad the thin side to
// a 32-wide MFMA block and do 10-30x the useful work:
//  * thin input (cin <= 4): the 1-channel network head -- nn.Conv2d(in, F, 3)
//    (edsr_net.py:28, drf_net.py:25, duf_net.py:35 as a (1,3,3) Conv3d) --
//    and the data gradient of the 1-channel tail conv (edsr_net.py:32).
//    The MFMA k dimension becomes (tap, channel) instead of channel:
//    K = kd*kh*kw*cin <= 32 is one or two k-steps of v_mfma_f32_32x32x16_bf16
//    on an im2col gather from an LDS patch.
//  * thin output (cout <= 3): the tail conv F -> 1 at HR resolution
//    (edsr_net.py:32, drf_net.py:147) and the data gradient of the head.
//    The MFMA m dimension becomes (tap, output channel):
//    P[(tap, co)][u] = sum_c w[tap][co][c] * x[u][c] for every input voxel u of
//    a halo tile, then y[v][co] = sum_tap P[(tap, co)][v + tap].
//  * thin weight gradient (cout <= 3): dW[tap][co][c] = sum_u x[u][c] *
//    dy[u - tap + pad][co], again with (tap, co) as the MFMA m dimension, into
//    the same per-split slabs as conv_wgrad_kernel (same deterministic reduce).
// All three are HBM-bound (read the wide side once, write the output once);
// the MFMAs only keep the arithmetic off the VALU.  Forward epilogue semantics
// equal conv_fwd's: t = (acc + bias) * out_scale -> act -> mask -> + residual -> + y.
#include "conv_common.h"
#include "vsrk_internal.h"

namespace {
using namespace vsrk_conv;

constexpr int THR = 256;         // 4 waves
constexpr int TH = 8;            // output tile rows
constexpr int TWT = 32;          // output tile columns (one MFMA column block per row)
constexpr int CG = 32;           // output channels per thin-in epilogue pass (one MFMA block)
constexpr int OROW = CG + 4;     // floats per voxel row of the transposed thin-in output (conflict-free)
constexpr int PATCH_MAX = 1024;  // bf16 elements of the thin-in input patch
constexpr int NPF = PATCH_MAX / THR;  // patch elements prefetched per thread
constexpr int XROW = 80;         // thin-out LDS bytes per staged voxel row (32 bf16 + 16 pad)
constexpr int UMAX = 352;        // thin-out halo voxels per tile, padded to 32 (10 x 34 = 340)
constexpr int NLX = UMAX * 4 / THR + 1;  // thin-out 16-byte chunks staged per thread and stage (5.5 -> 6)
constexpr int NPW = 4;           // thin wgrad: dY patch elements per thread (cout * 10 * 34 <= 1024)

struct ThinArgs {
  View x, y, res, msk;
  const void* w;  // packed [kd][kh][kw][cout_pad][cin_pad], the input's 16-bit type
  const float* bias;
  const float* pro_scale;
  const float* pro_shift;
  const float* act_param;
  const float* mask_slope;
  int cin, cout, cin_pad, cout_pad;
  int kd, kh, kw, pd, ph, pw;
  int prologue, act, accumulate, has_res, has_mask, vec;
  float out_scale;
  int tiles_h, tiles_w, ntiles, tiles_per_blk;
};

struct TileIdx {
  int nb, dz, h0, w0;
};
__device__ __forceinline__ TileIdx tile_at(int t, int tiles_w, int tiles_h, int depth) {
  TileIdx ti;
  const int tw_i = t % tiles_w;
  t /= tiles_w;
  const int th_i = t % tiles_h;
  t /= tiles_h;
  ti.dz = t % depth;
  ti.nb = t / depth;
  ti.h0 = th_i * TH;
  ti.w0 = tw_i * TWT;
  return ti;
}

// BN-affine / ReLU input prologue of one element of channel c
__device__ __forceinline__ float pro_el(int prologue, const float* sc, const float* sh, float v, int c) {
  if (prologue & VSRK_PRO_AFFINE) v = fmaf(v, sc[c], sh[c]);
  if (prologue & VSRK_PRO_RELU) v = fmaxf(v, 0.f);
  return v;
}

// Epilogue of E consecutive output channels co..co+E-1 of one voxel; yo / ro /
// mo are the element offsets of channel co in y / residual / mask (views with
// unit channel stride).  Full 16-byte chunks go as one load/store each.
template <typename YT, int E>
__device__ __forceinline__ void epi_chunk(const ThinArgs& a, const float* acc, const float* bias_s, int64_t yo,
                                          int64_t ro, int64_t mo, int co, float aslope, float mslope) {
  constexpr int CE = 16 / (int)sizeof(YT);
  YT* yp = reinterpret_cast<YT*>(a.y.ptr) + yo;
  const YT* rp = reinterpret_cast<const YT*>(a.res.ptr) + ro;
  const YT* mp = reinterpret_cast<const YT*>(a.msk.ptr) + mo;
  const bool full = E == CE && a.vec && co + E <= a.cout;
  float m[E], rr[E], o[E], v[E];
  if (full) {
    if constexpr (E == CE) {
      if (a.has_mask) Chunk<YT>::unpack(*reinterpret_cast<const uint4*>(mp), m);
      if (a.has_res) Chunk<YT>::unpack(*reinterpret_cast<const uint4*>(rp), rr);
      if (a.accumulate) Chunk<YT>::unpack(*reinterpret_cast<const uint4*>(yp), o);
    }
  } else {
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const bool ok = co + e < a.cout;
      m[e] = (ok && a.has_mask) ? to_f32<YT>(mp[e]) : 0.f;
      rr[e] = (ok && a.has_res) ? to_f32<YT>(rp[e]) : 0.f;
      o[e] = (ok && a.accumulate) ? to_f32<YT>(yp[e]) : 0.f;
    }
  }
#pragma unroll
  for (int e = 0; e < E; ++e) {
    float t = fmaf(acc[e], a.out_scale, bias_s[e]);  // (acc + bias) * out_scale
    t = act_apply(a.act, t, aslope);
    if (a.has_mask) t = mask_apply(m[e], t, mslope);
    if (a.has_res) t += rr[e];
    if (a.accumulate) t += o[e];
    v[e] = t;
  }
  if (full) {
    if constexpr (E == CE) *reinterpret_cast<uint4*>(yp) = Chunk<YT>::pack(v);
  } else {
#pragma unroll
    for (int e = 0; e < E; ++e)
      if (co + e < a.cout) yp[e] = from_f32<YT>(v[e]);
  }
}

__device__ __forceinline__ int64_t corner(const View& v, int nb, int d, int h, int w) {
  return nb * v.sn + (int64_t)d * v.sd + (int64_t)h * v.sh + (int64_t)w * v.sw;
}

// ---------------------------------------------------------------------------
// thin input: K = (tap, c) im2col
// ---------------------------------------------------------------------------
// A workgroup walks a contiguous run of 8x32 output tiles.  Per tile the input
// patch (cin x kd x (8+kh-1) x (32+kw-1), prologue applied, zero padded) is
// staged into LDS as bf16; wave w owns output rows w and w+4 and gathers their
// im2col B fragments once; A fragments (weights, every output channel) stay
// in registers for the whole run.  Per 32-channel block the accumulators go
// through LDS transposed to voxel-major rows and all 256 threads store
// 16-byte channel chunks.  Every per-thread index (patch slot, epilogue chunk)
// is fixed for the launch and precomputed as an offset from the tile corner,
// so a tile costs one 64-bit corner per tensor.
template <typename YT, int KS, int NCBM, typename H>
__global__ __launch_bounds__(THR) __attribute__((amdgpu_waves_per_eu(KS * NCBM <= 2 ? 3 : 2))) void conv_thin_in_kernel(
    ThinArgs a) {
  constexpr int E = 16 / (int)sizeof(YT);
  constexpr int NCH = CG / E;         // chunks per voxel and channel block
  constexpr int NIT = 256 * NCH / THR;  // epilogue chunks per thread and block
  extern __shared__ __attribute__((aligned(16))) char lds[];
  float* lout = reinterpret_cast<float*>(lds);                  // [256][OROW]
  H* patch = reinterpret_cast<H*>(lds + 256 * OROW * 4);  // [cin][kd][HH][WW]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, n = lane & 31, hf = lane >> 5;
  const int HH = TH + a.kh - 1, WW = TWT + a.kw - 1;
  const int K = a.kd * a.kh * a.kw * a.cin;
  const int taps2 = a.kh * a.kw;
  const int npatch = a.cin * a.kd * HH * WW;
  const int ncb = ceil_div(a.cout, 32);
  const float aslope = a.act == VSRK_ACT_PRELU ? *a.act_param : 0.f;
  const float mslope = a.mask_slope ? *a.mask_slope : 0.f;

  // im2col offsets of this lane's k values (-1: k >= K, reads zero)
  int boff[KS][8];
#pragma unroll
  for (int s = 0; s < KS; ++s)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int k = 16 * s + 8 * hf + j;
      if (k < K) {
        const int c = k % a.cin, tap = k / a.cin;
        const int dzk = tap / taps2, r2 = tap % taps2, khk = r2 / a.kw, kwk = r2 % a.kw;
        boff[s][j] = ((c * a.kd + dzk) * HH + khk) * WW + kwk;
      } else {
        boff[s][j] = -1;
      }
    }
  // weights: A[co][k] = w[tap][co][c]
  typename V8<H>::type afr[NCBM][KS];
#pragma unroll
  for (int cb = 0; cb < NCBM; ++cb)
#pragma unroll
    for (int s = 0; s < KS; ++s)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int k = 16 * s + 8 * hf + j, co = cb * 32 + n;
        H v = (H)0.f;
        if (cb < ncb && k < K) {
          const int c = k % a.cin, tap = k / a.cin;
          v = reinterpret_cast<const H*>(a.w)[((int64_t)tap * a.cout_pad + co) * a.cin_pad + c];  // zero-padded past cout
        }
        afr[cb][s][j] = v;
      }
  // patch slots: offset from the tile's input corner and (dz, h, w) position
  int p_rel[NPF], p_geo[NPF];
#pragma unroll
  for (int k = 0; k < NPF; ++k) {
    const int i = tid + k * THR;
    const int ww = i % WW;
    int r = i / WW;
    const int hh = r % HH;
    r /= HH;
    const int dzk = r % a.kd, c = r / a.kd;
    p_rel[k] = (int)((int64_t)dzk * a.x.sd + (int64_t)hh * a.x.sh + (int64_t)ww * a.x.sw) + c;
    p_geo[k] = i < npatch ? ((dzk << 20) | (hh << 10) | ww) : -1;
  }
  // epilogue chunks: voxel v = i / NCH (row v/32, column v%32), channel chunk q = i % NCH
  int y_rel[NIT], r_rel[NIT], m_rel[NIT], e_vx[NIT];
#pragma unroll
  for (int k = 0; k < NIT; ++k) {
    const int i = tid + k * THR, v = i / NCH, q = i % NCH;
    const int vr = v / 32, vc = v % 32;
    y_rel[k] = (int)(vr * a.y.sh + vc * a.y.sw) + q * E;
    r_rel[k] = (int)(vr * a.res.sh + vc * a.res.sw) + q * E;
    m_rel[k] = (int)(vr * a.msk.sh + vc * a.msk.sw) + q * E;
    e_vx[k] = (vr << 8) | vc;
  }
  const int qe = (tid % NCH) * E;  // channel offset of every epilogue chunk within a block

  // Patch staging is software-pipelined: the next tile's elements are loaded
  // into registers while this tile computes and stores.
  const H* xb = reinterpret_cast<const H*>(a.x.ptr);
  const int L = xcd_remap(blockIdx.x, gridDim.x);
  const int t0 = L * a.tiles_per_blk, t1 = min(a.ntiles, t0 + a.tiles_per_blk);
  H pv[NPF];
  unsigned pmask = 0;
  auto fetch = [&](int t) __attribute__((always_inline)) {
    const TileIdx ti = tile_at(t, a.tiles_w, a.tiles_h, a.y.d);
    const int d0 = ti.dz - a.pd, hb = ti.h0 - a.ph, wb = ti.w0 - a.pw;
    const H* base = xb + corner(a.x, ti.nb, d0, hb, wb);
    pmask = 0;
#pragma unroll
    for (int k = 0; k < NPF; ++k) {
      const int g = p_geo[k];
      const int di = d0 + (g >> 20), hi = hb + ((g >> 10) & 1023), wi = wb + (g & 1023);
      const bool ok = g >= 0 && di >= 0 && di < a.x.d && hi >= 0 && hi < a.x.h && wi >= 0 && wi < a.x.w;
      pv[k] = *(ok ? base + p_rel[k] : xb);
      pmask |= (ok ? 1u : 0u) << k;
    }
  };
  if (t0 < t1) fetch(t0);
  for (int t = t0; t < t1; ++t) {
    const TileIdx ti = tile_at(t, a.tiles_w, a.tiles_h, a.y.d);
#pragma unroll
    for (int k = 0; k < NPF; ++k) {
      const int i = tid + k * THR;
      if (p_geo[k] >= 0) {
        float v = 0.f;
        if ((pmask >> k) & 1) {
          v = (float)pv[k];
          if (a.prologue) v = pro_el(a.prologue, a.pro_scale, a.pro_shift, v, i / (a.kd * HH * WW));
        }
        patch[i] = (H)v;
      }
    }
    __syncthreads();
    if (t + 1 < t1) fetch(t + 1);
    typename V8<H>::type bfr[2][KS];
#pragma unroll
    for (int rr = 0; rr < 2; ++rr) {
      const int vo = (wave + 4 * rr) * WW + n;
#pragma unroll
      for (int s = 0; s < KS; ++s)
#pragma unroll
        for (int j = 0; j < 8; ++j) bfr[rr][s][j] = boff[s][j] >= 0 ? patch[boff[s][j] + vo] : (H)0.f;
    }
    const int64_t yc = corner(a.y, ti.nb, ti.dz, ti.h0, ti.w0);
    const int64_t rc = corner(a.res, ti.nb, ti.dz, ti.h0, ti.w0);
    const int64_t mc = corner(a.msk, ti.nb, ti.dz, ti.h0, ti.w0);
    const int hlim = a.y.h - ti.h0, wlim = a.y.w - ti.w0;
#pragma unroll
    for (int cb = 0; cb < NCBM; ++cb) {
      if (cb >= ncb) break;  // uniform
#pragma unroll
      for (int rr = 0; rr < 2; ++rr) {
        const int vrow = wave + 4 * rr;
        f32x16 acc;
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[i] = 0.f;
#pragma unroll
        for (int s = 0; s < KS; ++s) acc = mfma32x16(afr[cb][s], bfr[rr][s], acc);
        float* dst = lout + (vrow * 32 + n) * OROW + 4 * hf;
#pragma unroll
        for (int j = 0; j < 4; ++j)
          *reinterpret_cast<f32x4*>(dst + 8 * j) = f32x4{acc[4 * j], acc[4 * j + 1], acc[4 * j + 2], acc[4 * j + 3]};
      }
      __syncthreads();
      const int co = cb * 32 + qe;
      float bsv[E];
#pragma unroll
      for (int e = 0; e < E; ++e) bsv[e] = (a.bias && co + e < a.cout) ? a.bias[co + e] * a.out_scale : 0.f;
#pragma unroll
      for (int k = 0; k < NIT; ++k) {
        const int vr = e_vx[k] >> 8, vc = e_vx[k] & 255;
        if (co < a.cout && vr < hlim && vc < wlim) {
          const float* src = lout + (vr * 32 + vc) * OROW + qe;
          float accv[E];
#pragma unroll
          for (int e = 0; e < E; e += 4) {
            const f32x4 q4 = *reinterpret_cast<const f32x4*>(src + e);
            accv[e] = q4[0];
            accv[e + 1] = q4[1];
            accv[e + 2] = q4[2];
            accv[e + 3] = q4[3];
          }
          epi_chunk<YT, E>(a, accv, bsv, yc + y_rel[k] + cb * 32, rc + r_rel[k] + cb * 32, mc + m_rel[k] + cb * 32,
                           co, aslope, mslope);
        }
      }
      __syncthreads();
    }
  }
}

// ---------------------------------------------------------------------------
// thin output: M = (tap, co)
// ---------------------------------------------------------------------------
// Per tile and 32-channel chunk the (8+KK-1) x (32+KK-1) halo voxels are staged
// in LDS (80-byte rows: conflict-free ds_read_b128) and wave w accumulates the
// 32-voxel blocks w, w+4, w+8 of P in registers across chunks.  P then goes to
// LDS and thread v sums its KK*KK shifted entries per output channel.  Stages
// (tile, chunk) are software-pipelined through registers, and every
// per-thread index is an offset from the stage's corner fixed for the launch.
template <typename YT, int KK, typename H>
__global__ __launch_bounds__(THR) __attribute__((amdgpu_waves_per_eu(3))) void conv_thin_out_kernel(ThinArgs a) {
  constexpr int HH = TH + KK - 1, WW = TWT + KK - 1;
  constexpr int U = HH * WW, UB = (U + 31) / 32;
  extern __shared__ __attribute__((aligned(16))) char lds[];
  char* xs = lds;                                          // [UMAX][XROW]
  float* P = reinterpret_cast<float*>(lds + UMAX * XROW);  // [M][UMAX]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, n = lane & 31, hf = lane >> 5;
  const int M = KK * KK * a.cout;
  const float aslope = a.act == VSRK_ACT_PRELU ? *a.act_param : 0.f;
  const float mslope = a.mask_slope ? *a.mask_slope : 0.f;
  const int mtap = n / a.cout, mco = n % a.cout;  // this lane's A row (tap, co)
  const H* xb = reinterpret_cast<const H*>(a.x.ptr);
  const int nch = ceil_div(a.cin, 32);

  // staging slots: chunk i = tid + k*THR is piece i&3 of halo voxel u = i>>2
  int x_rel[NLX], x_geo[NLX];
#pragma unroll
  for (int k = 0; k < NLX; ++k) {
    const int i = tid + k * THR, u = i >> 2, p = i & 3;
    const int hh = u / WW, ww = u % WW;
    x_rel[k] = (int)((int64_t)hh * a.x.sh + (int64_t)ww * a.x.sw) + 8 * p;
    x_geo[k] = (i < UMAX * 4 && u < U) ? ((p << 16) | (hh << 8) | ww) : -1;
  }
  const int vr = tid / 32, vc = tid % 32;  // this thread's output voxel in the epilogue
  const int y_rel = (int)(vr * a.y.sh + vc * a.y.sw);
  const int r_rel = (int)(vr * a.res.sh + vc * a.res.sw);
  const int m_rel = (int)(vr * a.msk.sh + vc * a.msk.sw);

  const int L = xcd_remap(blockIdx.x, gridDim.x);
  const int t0 = L * a.tiles_per_blk, t1 = min(a.ntiles, t0 + a.tiles_per_blk);
  const int s0 = t0 * nch, s1 = t1 * nch;
  uint4 rv[NLX];
  typename V8<H>::type afn[2], afr[2];  // A fragments (weights of the stage's chunk): next / current
  unsigned rmask = 0;
  auto fetch = [&](int sg) __attribute__((always_inline)) {
    const TileIdx ti = tile_at(sg / nch, a.tiles_w, a.tiles_h, a.y.d);
    const int c0 = (sg % nch) * 32;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int c = c0 + 16 * s + 8 * hf;
      afn[s] = (n < M) ? *reinterpret_cast<const typename V8<H>::type*>(reinterpret_cast<const H*>(a.w) + ((int64_t)mtap * a.cout_pad + mco) * a.cin_pad + c)
                       : typename V8<H>::type{};
    }
    const int hb = ti.h0 - a.ph, wb = ti.w0 - a.pw;
    const H* base = xb + corner(a.x, ti.nb, ti.dz, hb, wb) + c0;
    rmask = 0;
#pragma unroll
    for (int k = 0; k < NLX; ++k) {
      const int g = x_geo[k];
      const int hi = hb + ((g >> 8) & 255), wi = wb + (g & 255), ch = c0 + 8 * (g >> 16);
      const bool ok = g >= 0 && hi >= 0 && hi < a.x.h && wi >= 0 && wi < a.x.w && ch < a.cin;
      rv[k] = *reinterpret_cast<const uint4*>(ok ? base + x_rel[k] : xb);
      rmask |= (ok ? 1u : 0u) << k;
    }
  };
  f32x16 acc[3];
  if (s0 < s1) fetch(s0);
  for (int sg = s0; sg < s1; ++sg) {
    const int q = sg % nch;
    if (q == 0) {
#pragma unroll
      for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[i][e] = 0.f;
    }
#pragma unroll
    for (int k = 0; k < NLX; ++k) {
      const int i = tid + k * THR;
      if (i < UMAX * 4) {
        uint4 v = make_uint4(0, 0, 0, 0);
        if ((rmask >> k) & 1) {
          v = rv[k];
          if (a.prologue) {
            const int ch = q * 32 + 8 * (i & 3);
            float f[8];
            Chunk<H>::unpack(v, f);
#pragma unroll
            for (int e = 0; e < 8; ++e) f[e] = pro_el(a.prologue, a.pro_scale, a.pro_shift, f[e], ch + e);
            v = Chunk<H>::pack(f);
          }
        }
        *reinterpret_cast<uint4*>(xs + (i >> 2) * XROW + (i & 3) * 16) = v;
      }
    }
    afr[0] = afn[0];
    afr[1] = afn[1];
    __syncthreads();
    if (sg + 1 < s1) fetch(sg + 1);
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const int ub = wave + 4 * i;
      if (ub < UB) {
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          const typename V8<H>::type bfr = *reinterpret_cast<const typename V8<H>::type*>(xs + (ub * 32 + n) * XROW + (16 * s + 8 * hf) * 2);
          acc[i] = mfma32x16(afr[s], bfr, acc[i]);
        }
      }
    }
    if (q + 1 < nch) {
      __syncthreads();  // xs is restaged by the next stage
      continue;
    }
    const TileIdx ti = tile_at(sg / nch, a.tiles_w, a.tiles_h, a.y.d);
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const int ub = wave + 4 * i;
      if (ub < UB) {
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int m = 8 * j + 4 * hf + e;
            if (m < M) P[m * UMAX + ub * 32 + n] = acc[i][4 * j + e];
          }
      }
    }
    __syncthreads();  // P complete; every wave is done reading xs
    if (ti.h0 + vr < a.y.h && ti.w0 + vc < a.y.w) {
      const int64_t yo = corner(a.y, ti.nb, ti.dz, ti.h0, ti.w0) + y_rel;
      const int64_t ro = corner(a.res, ti.nb, ti.dz, ti.h0, ti.w0) + r_rel;
      const int64_t mo = corner(a.msk, ti.nb, ti.dz, ti.h0, ti.w0) + m_rel;
      for (int co = 0; co < a.cout; ++co) {
        float sum = 0.f;
#pragma unroll
        for (int khk = 0; khk < KK; ++khk)
#pragma unroll
          for (int kwk = 0; kwk < KK; ++kwk)
            sum += P[((khk * KK + kwk) * a.cout + co) * UMAX + (vr + khk) * WW + vc + kwk];
        const float bs = a.bias ? a.bias[co] * a.out_scale : 0.f;
        epi_chunk<YT, 1>(a, &sum, &bs, yo + co, ro + co, mo + co, co, aslope, mslope);
      }
    }
    // P is rewritten only after the next tile's first stage barrier
  }
}

// ---------------------------------------------------------------------------
// thin weight gradient: M = (tap, co), K = input voxels, N = input channels
// ---------------------------------------------------------------------------
// A workgroup = (split, 32*NCI input-channel chunk), as conv_wgrad_kernel.
// Per 8x32 tile: the x tile (no halo: u runs over the tile's own voxels) is
// staged as NCI planes of 64-byte rows and read transposed (ds_read_b64_tr_b16)
// as the B operand; the dY patch (cout x (8+kh-1) x (32+kw-1), origin shifted
// by pad - (k-1)) gives the A operand A[(tap, co)][u] = dy[u - tap + pad][co].
// Wave w runs k-steps w, w+4, w+8, w+12 (16 voxels each); the four wave
// partials and the dbias partials are summed in a fixed order at the end.
template <int NCI, typename H>
__global__ __launch_bounds__(THR) __attribute__((amdgpu_waves_per_eu(NCI == 1 ? 3 : 2))) void conv_wgrad_thin_kernel(WgradArgs a) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  char* xs = lds;                                           // [NCI][256][64 B]
  H* dyp = reinterpret_cast<H*>(lds + NCI * 256 * 64);  // [cout][HH][WW]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, n = lane & 31, hf = lane >> 5;
  const int HH = GTH + a.kh - 1, WW = TW + a.kw - 1;
  const int taps2 = a.kh * a.kw, M = taps2 * a.cout;
  const int oh = a.ph - (a.kh - 1), ow = a.pw - (a.kw - 1);  // dY patch origin relative to the tile
  const int L = xcd_remap(blockIdx.x, a.nblk);
  const int split = L / a.ncombos;
  const int cic = (L - split * a.ncombos) % a.n_ci_chunks;
  const int ci0 = cic * 32 * NCI;
  const bool do_bias = a.want_bias && cic == 0;
  const int mtap = n / a.cout, mco = n % a.cout;
  const int mkh = mtap / a.kw, mkw = mtap % a.kw;
  // transposed-read geometry (as conv_wgrad_kernel)
  const int g = lane >> 4, i16 = lane & 15, qq = i16 >> 2, pp = i16 & 3;
  const int hfk = g >> 1, colb = ((g & 1) * 16 + 4 * pp) * 2;
  const H* xb = reinterpret_cast<const H*>(a.x.ptr);
  const H* yb = reinterpret_cast<const H*>(a.dy.ptr);

  f32x16 acc[NCI];
#pragma unroll
  for (int p = 0; p < NCI; ++p)
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[p][e] = 0.f;
  float bsum[3] = {0.f, 0.f, 0.f};

  // Staging is software-pipelined: tile t+1's x chunks and dY patch are
  // loaded into registers while tile t computes.
  const int t_begin = split * a.tiles_per_split;
  const int t_end = min(a.ntiles, t_begin + a.tiles_per_split);
  const int npat = a.cout * HH * WW;
  uint4 xr[4 * NCI];
  H yv[NPW];
  unsigned xmask = 0, ymask = 0;
  auto fetch = [&](int t) __attribute__((always_inline)) {
    const TileIdx ti = tile_at(t, a.tiles_w, a.tiles_h, a.dy.d);
    xmask = 0;
    ymask = 0;
#pragma unroll
    for (int k = 0; k < 4 * NCI; ++k) {
      const int i = tid + k * THR;
      const int pl = i >> 10, rem = i & 1023, v = rem >> 2, p = rem & 3;
      const int hi = ti.h0 + v / TW, wi = ti.w0 + v % TW, ch = ci0 + pl * 32 + 8 * p;
      const bool ok = hi < a.x.h && wi < a.x.w && ch < a.cin;
      xr[k] = *reinterpret_cast<const uint4*>(xb + (ok ? view_off(a.x, ti.nb, ti.dz, hi, wi, ch) : 0));
      xmask |= (ok ? 1u : 0u) << k;
    }
#pragma unroll
    for (int k = 0; k < NPW; ++k) {
      const int i = tid + k * THR;
      const int co = i / (HH * WW), rr = i % (HH * WW), hh = rr / WW, ww = rr % WW;
      const int hd = ti.h0 + oh + hh, wd = ti.w0 + ow + ww;
      const bool ok = i < npat && hd >= 0 && hd < a.dy.h && wd >= 0 && wd < a.dy.w;
      yv[k] = yb[ok ? view_off(a.dy, ti.nb, ti.dz, hd, wd, co) : 0];
      ymask |= (ok ? 1u : 0u) << k;
    }
  };
  if (t_begin < t_end) fetch(t_begin);
  for (int t = t_begin; t < t_end; ++t) {
    const TileIdx ti = tile_at(t, a.tiles_w, a.tiles_h, a.dy.d);
#pragma unroll
    for (int k = 0; k < 4 * NCI; ++k) {
      const int i = tid + k * THR;
      const int pl = i >> 10, rem = i & 1023, v = rem >> 2, p = rem & 3;
      uint4 val = make_uint4(0, 0, 0, 0);
      if ((xmask >> k) & 1) {
        val = xr[k];
        if (a.prologue) {
          const int ch = ci0 + pl * 32 + 8 * p;
          float f[8];
          Chunk<H>::unpack(val, f);
#pragma unroll
          for (int e = 0; e < 8; ++e) f[e] = pro_el(a.prologue, a.pro_scale, a.pro_shift, f[e], ch + e);
          val = Chunk<H>::pack(f);
        }
      }
      *reinterpret_cast<uint4*>(xs + (pl * 256 + v) * 64 + p * 16) = val;
    }
#pragma unroll
    for (int k = 0; k < NPW; ++k) {
      const int i = tid + k * THR;
      if (i < npat) dyp[i] = ((ymask >> k) & 1) ? yv[k] : (H)0.f;
    }
    __syncthreads();
    if (t + 1 < t_end) fetch(t + 1);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int vb = (wave + 4 * i) * 16;
      const int vrow = vb / TW, vc0 = vb % TW;
      typename V8<H>::type af;
      if (n < M) {
        const int base = (mco * HH + vrow - mkh + a.kh - 1) * WW + vc0 + 8 * hf - mkw + a.kw - 1;
#pragma unroll
        for (int j = 0; j < 8; ++j) af[j] = dyp[base + j];
      } else {
        af = typename V8<H>::type{};
      }
#pragma unroll
      for (int p = 0; p < NCI; ++p) {
        const char* px = xs + (p * 256 + vrow * TW + vc0 + 8 * hfk + qq) * 64 + colb;
        const v4i16 x0 = ds_read_tr(px), x1 = ds_read_tr(px + 4 * 64);
        const typename V8<H>::type bfr = __builtin_bit_cast(typename V8<H>::type, __builtin_shufflevector(x0, x1, 0, 1, 2, 3, 4, 5, 6, 7));
        acc[p] = mfma32x16(af, bfr, acc[p]);
      }
    }
    if (do_bias) {
      const int vr = tid / TW, vc = tid % TW;
      if (ti.h0 + vr < a.dy.h && ti.w0 + vc < a.dy.w) {
        for (int co = 0; co < a.cout; ++co) bsum[co] += (float)dyp[(co * HH + vr - oh) * WW + vc - ow];
      }
    }
    __syncthreads();
  }

  // fixed-order sum of the wave partials: red[wave][plane][m][n]
  float* red = reinterpret_cast<float*>(lds);
#pragma unroll
  for (int p = 0; p < NCI; ++p)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) red[((wave * NCI + p) * 32 + 8 * j + 4 * hf + e) * 32 + n] = acc[p][4 * j + e];
  __syncthreads();
  float* out = a.ws + (int64_t)L * a.slab;
  const int CW = 32 * NCI;
  const int nw = taps2 * 32 * CW;  // slab layout [tap][co (32)][ci (32*NCI)], dbias after
  for (int i = tid; i < nw; i += THR) {
    const int ci = i % CW, t2 = i / CW, co = t2 % 32, tap = t2 / 32;
    float s = 0.f;
    if (co < a.cout) {
      const int m = tap * a.cout + co, p = ci / 32, nn = ci % 32;
      s = red[((0 * NCI + p) * 32 + m) * 32 + nn];
      s += red[((1 * NCI + p) * 32 + m) * 32 + nn];
      s += red[((2 * NCI + p) * 32 + m) * 32 + nn];
      s += red[((3 * NCI + p) * 32 + m) * 32 + nn];
    }
    out[i] = s;
  }
  if (do_bias) {
    __syncthreads();
#pragma unroll
    for (int co = 0; co < 3; ++co) red[tid * 3 + co] = bsum[co];
    __syncthreads();
    if (tid < 32) {
      float s = 0.f;
      if (tid < a.cout)
        for (int th = 0; th < THR; ++th) s += red[th * 3 + tid];
      out[nw + tid] = s;
    }
  }
}

int num_cus_thin() {
  static int cus = 0;
  if (cus == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
  }
  return cus;
}

template <typename KF>
void launch_persistent(KF kern, ThinArgs& a, size_t lds, hipStream_t s) {
  (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  int per_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)kern, THR, lds) != hipSuccess || per_cu < 1)
    per_cu = 1;
  const int want = (int)vsrk_capped_grid(num_cus_thin() * per_cu);
  a.tiles_per_blk = ceil_div(a.ntiles, want);
  const int grid = ceil_div(a.ntiles, a.tiles_per_blk);
  kern<<<grid, THR, lds, s>>>(a);
}

}  // namespace

int vsrk_g_thin_mode = -1;  // -1: from VSRK_CONV_THIN (default on), 0 off, 1 on (vsrk_conv_set_path)

static bool thin_enabled() {
  int m = vsrk_g_thin_mode;
  if (m < 0) {
    const char* e = getenv("VSRK_CONV_THIN");
    m = (e && e[0] == '0') ? 0 : 1;
  }
  return m != 0;
}

// 1 = launched; 0 = not a thin conv (the implicit-GEMM kernels run); < 0 = -(error status).
int vsrk_conv_fwd_thin(const vsrk_conv_desc* d, const vsrk_tensor5* x, const void* w_packed, const float* bias,
                       const float* pro_scale, const float* pro_shift, const vsrk_tensor5* residual,
                       const vsrk_tensor5* mask, const vsrk_tensor5* y, hipStream_t s) {
  if (!thin_enabled()) return 0;
  if (!vsrk_is16(x->dtype)) return 0;
  if (const int st = vsrk_conv_fwd_stencil(d, x, w_packed, bias, residual, mask, y, s)) return st;
  if (const int st = vsrk_conv_fwd_stencil_out(d, x, w_packed, bias, residual, mask, y, s)) return st;
  if (x->shuffle > 1 || y->shuffle > 1 || d->bias_perm_r > 1) return 0;
  if ((residual && residual->shuffle > 1) || (mask && mask->shuffle > 1)) return 0;
  const int K = d->kd * d->kh * d->kw * x->c;
  const bool thin_in = x->c <= 4 && K <= 32 && y->c >= 8 && y->c <= 256;
  const bool thin_out = !thin_in && y->c <= 3 && d->kd == 1 && d->pd == 0 && x->c % 8 == 0 &&
                        d->kh * d->kw * y->c <= 32 && chunk_ok(x, 2) && x->d == y->d;
  if (!thin_in && !thin_out) return 0;
  const int HH = TH + d->kh - 1, WW = TWT + d->kw - 1;
  if (thin_in && x->c * d->kd * HH * WW > PATCH_MAX) return 0;
  ThinArgs a;
  a.x = make_view(x);
  a.y = make_view(y);
  a.res = residual ? make_view(residual) : a.y;
  a.msk = mask ? make_view(mask) : a.y;
  a.w = w_packed;
  a.bias = bias;
  a.pro_scale = pro_scale;
  a.pro_shift = pro_shift;
  a.act_param = d->act_param;
  a.mask_slope = d->mask_slope;
  a.cin = x->c;
  a.cout = y->c;
  a.cin_pad = round_up(x->c, 32);
  a.cout_pad = round_up(y->c, 128);
  a.kd = d->kd; a.kh = d->kh; a.kw = d->kw;
  a.pd = d->pd; a.ph = d->ph; a.pw = d->pw;
  a.prologue = d->prologue;
  a.act = d->act;
  a.accumulate = d->accumulate;
  a.has_res = residual != nullptr;
  a.has_mask = mask != nullptr;
  const int yes = vsrk_esize(y->dtype);
  a.vec = chunk_ok(y, yes) && (!residual || chunk_ok(residual, yes)) && (!mask || chunk_ok(mask, yes));
  a.out_scale = d->out_scale;
  a.tiles_h = ceil_div(y->h, TH);
  a.tiles_w = ceil_div(y->w, TWT);
  const int64_t ntiles = (int64_t)y->n * y->d * a.tiles_h * a.tiles_w;
  if (ntiles >= (1ll << 31)) {
    vsrk_set_error("conv_fwd: too many tiles");
    return -VSRK_ERR_INVALID;
  }
  a.ntiles = (int)ntiles;
  if (a.ntiles == 0) return 1;
  const bool yb = y->dtype != VSRK_F32;  // 16-bit output (the input's type)
  if (thin_in) {
    const size_t lds = (size_t)256 * OROW * 4 + PATCH_MAX * 2;  // 36.9 KB + 2 KB: 3 workgroups per CU
    const int ncb = ceil_div(y->c, 32);
#define VSRK_THIN_IN(KS, NCB)                                                     \
  do {                                                                            \
    vsrk_dispatch16(x->dtype, [&](auto tag) {                                     \
      using H = decltype(tag);                                                    \
      if (yb) launch_persistent(conv_thin_in_kernel<H, KS, NCB, H>, a, lds, s);   \
      else launch_persistent(conv_thin_in_kernel<float, KS, NCB, H>, a, lds, s);  \
      return 0;                                                                   \
    });                                                                           \
  } while (0)
    if (K <= 16) {
      if (ncb <= 2) VSRK_THIN_IN(1, 2);
      else if (ncb <= 4) VSRK_THIN_IN(1, 4);
      else VSRK_THIN_IN(1, 8);
    } else {
      if (ncb <= 2) VSRK_THIN_IN(2, 2);
      else if (ncb <= 4) VSRK_THIN_IN(2, 4);
      else VSRK_THIN_IN(2, 8);
    }
#undef VSRK_THIN_IN
  } else {
    const size_t lds = (size_t)UMAX * XROW + (size_t)d->kh * d->kw * y->c * UMAX * 4;
    vsrk_dispatch16(x->dtype, [&](auto tag) {
      using H = decltype(tag);
      if (d->kh == 3) {
        if (yb) launch_persistent(conv_thin_out_kernel<H, 3, H>, a, lds, s);
        else launch_persistent(conv_thin_out_kernel<float, 3, H>, a, lds, s);
      } else {
        if (yb) launch_persistent(conv_thin_out_kernel<H, 1, H>, a, lds, s);
        else launch_persistent(conv_thin_out_kernel<float, 1, H>, a, lds, s);
      }
      return 0;
    });
  }
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    vsrk_set_error("conv_fwd(thin): launch failed: %s", hipGetErrorString(e));
    return -VSRK_ERR_LAUNCH;
  }
  return 1;
}

// Weight gradient of a conv with cout <= 3 (the tail conv F -> 1): same plan
// (splits x combos, slab size) as vsrk_conv_wgrad, so the reduce is shared.
int vsrk_conv_wgrad_thin(const vsrk_conv::WgradArgs& a, int nco, int nci, int perm_r, int dtype, hipStream_t s) {
  if (!thin_enabled()) return 0;
  if (nco != 1 || a.cout > 3 || a.kd != 1 || a.pd != 0 || a.kh != a.kw || a.kh * a.kw * a.cout > 32) return 0;
  if (a.cin % 8 || !a.xvec || a.x.r > 1 || a.dy.r > 1 || perm_r > 1) return 0;
  if (a.x.h != a.dy.h || a.x.w != a.dy.w || a.x.d != a.dy.d) return 0;
  if (a.cout * (GTH + a.kh - 1) * (TW + a.kw - 1) > NPW * THR) return 0;
  const size_t stage = (size_t)nci * 256 * 64 + (size_t)a.cout * (GTH + a.kh - 1) * (TW + a.kw - 1) * 2;
  const size_t lds = std::max(stage, (size_t)4 * nci * 1024 * 4);
  vsrk_dispatch16(dtype, [&](auto tag) {
    using H = decltype(tag);
    auto kern = nci == 2 ? conv_wgrad_thin_kernel<2, H> : conv_wgrad_thin_kernel<1, H>;
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    kern<<<a.nblk, THR, lds, s>>>(a);
    return 0;
  });
  return 1;
}
