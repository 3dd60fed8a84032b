#include <cstdio>
// Implicit-GEMM convolution forward / data-gradient on CDNA4 MFMA (gfx950).
//
// Replaces the nn.Conv2d / nn.Conv3d forward and backward the reference runs on
// every train step (edsr_net.py:28-64, duf_net.py:35-49,116-214,
// drf_net.py:55-147; backward via loss.backward(), base_trainer.py:128).
//
// Layout: activations channels-last (N,D,H,W,C) in bf16 or fp32; weights
// pre-packed [kd][kh][kw][cout_pad][cin_pad].  One workgroup (8 waves) owns an
// output tile of (8*MS) rows x 32 columns of one (n, d) slice and NT output
// channels.  Per (kd, 32-channel chunk) stage the input tile plus its halo is
// staged into LDS (80-byte rows: 64 data + 16 pad, conflict-free for
// ds_read_b128 column slices) and the stage's weights by LDS-DMA (64-byte
// rows, XOR-swizzled), then all KK*KK taps run out of LDS.  MFMA orientation
// is "weights x voxels" so that each lane's accumulator column is one voxel
// and its registers hold 4 consecutive output channels -> 8/16-byte
// channels-last stores.
//   bf16: v_mfma_f32_32x32x16_bf16, one per 16 channels.
//   fp32: v_mfma_f32_32x32x2_f32, four per 8 channels (exact fp32, parity path).
#include <type_traits>
#include "conv_common.h"

namespace {
using namespace vsrk_conv;

// ---------------------------------------------------------------------------
// forward / data-gradient
// ---------------------------------------------------------------------------
// Persistent: a workgroup walks a run of output tiles (runs are grouped per
// XCD so concurrently processed tiles are neighbours sharing halo rows and
// weight slices in one L2).  Its work is a flat sequence of stages
// (tile, kd tap, 32-channel chunk).  While the MFMAs of stage g run, the input
// chunks of stage g+1 are loading into registers (unconditional loads from
// clamped addresses, validity applied on commit) and its weights are landing
// in the other half of a double-buffered LDS weight area by LDS-DMA — across
// tile boundaries too, so only the very first stage of a workgroup is
// exposed.  A tile's epilogue runs right after its last stage's MFMAs (no LDS
// use) and overlaps other waves' compute.  KK is a template parameter so the
// tap loop is straight-line code (LDS reads pipelined, rows shared by
// neighbouring taps read once).
// XM: input addressing mode — 0 plain channels-last view (precomputed
// offsets), 1 sub-pixel view (generic addressing), 2 element loads (views
// that cannot be read in 16-byte chunks).
template <typename T, int NT, int MS, int KK, int XM, typename YT>
__global__ __launch_bounds__(NTHR) void conv_fwd_kernel(ConvArgs a) {
  constexpr int NS = NT / 32;
  constexpr int FTH = 8 * MS;  // tile rows: MS rows (of 32 voxels) per wave
  constexpr int E = Chunk<T>::E;
  constexpr int CK = 4 * E;  // channels per stage: 64 bytes
  constexpr int HWd = TW + KK - 1;
  constexpr int SLOTS = (FTH + KK - 1) * HWd;
  constexpr int MAXA = (SLOTS * 4 + NTHR - 1) / NTHR;
  constexpr int TAPS = KK * KK;
  constexpr int NBI = TAPS * NT / 16;  // 1 KiB LDS-DMA wave-instructions per stage
  constexpr int BBYTES = TAPS * NT * 64;
  static_assert(MS == 1 || MS == 2, "rows per wave");
  extern __shared__ __attribute__((aligned(16))) char lds[];

  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, r = lane & 31, hf = lane >> 5;
  char* ldsA = lds;
  char* ldsB = lds + SLOTS * ROWB;  // two buffers of BBYTES
  float* lbias_all = reinterpret_cast<float*>(ldsB + 2 * BBYTES);  // [cout_pad], view order
  float* lsc = lbias_all + a.cout_pad;
  float* lsh = lsc + a.cin_pad;
  const bool relu_in = (a.prologue & VSRK_PRO_RELU) != 0;
  const float aslope = a.act == VSRK_ACT_PRELU ? *a.act_param : 0.f;
  const float mslope = a.mask_slope ? *a.mask_slope : 0.f;
  if (a.prologue) stage_prologue(lsc, lsh, a.prologue, a.pro_scale, a.pro_shift, a.cin, a.cin_pad, tid, NTHR);
  for (int i = tid; i < a.cout_pad; i += NTHR) {
    float b = 0.f;
    if (a.bias && i < a.cout) {
      int cb = i;
      if (a.bias_r > 1) {  // view order (sub, c') -> torch order c'*r*r + sub
        const int rr = a.bias_r * a.bias_r, cp = a.cout / rr;
        const int sub = cb / cp;
        cb = (cb - sub * cp) * rr + sub;
      }
      b = a.bias[cb];
    }
    lbias_all[i] = b;
  }

  // this workgroup's tiles: XCD group x = blockIdx % 8 owns a contiguous
  // range of tiles; its workgroups take them round-robin.
  const int G = gridDim.x;
  const int x = blockIdx.x & 7, j = blockIdx.x >> 3;
  const int gx = (G >> 3) + (x < (G & 7) ? 1 : 0);      // workgroups in this XCD group
  const int cx = x * (G >> 3) + min(x, G & 7);           // workgroups in groups before it
  const int t_lo = (int)((int64_t)a.ntiles * cx / G);    // its share of tiles, by size
  const int t_hi = (int)((int64_t)a.ntiles * (cx + gx) / G);
  const int nchunk = (a.cin + CK - 1) / CK;

  struct Tile {
    int nb, dz, h0, w0, n0, kd_lo, nst;
  };
  auto decode = [&](int t) __attribute__((always_inline)) {
    Tile tl;
    const int tn = t % a.ntn;
    int tm = t / a.ntn;
    const int tw_i = tm % a.tiles_w;
    tm /= a.tiles_w;
    const int th_i = tm % a.tiles_h;
    tm /= a.tiles_h;
    tl.dz = tm % a.y.d;
    tl.nb = tm / a.y.d;
    tl.h0 = th_i * FTH;
    tl.w0 = tw_i * TW;
    tl.n0 = tn * NT;
    tl.kd_lo = max(0, a.pd - tl.dz);
    const int kd_hi = min(a.kd, a.x.d + a.pd - tl.dz);
    tl.nst = max(1, kd_hi - tl.kd_lo) * nchunk;
    return tl;
  };

  // Per-thread staging geometry, fixed for the launch: each owned 16-byte
  // chunk's halo position, its element offset from the tile's corner (mode 0)
  // and its LDS address.  Per stage only wave-uniform terms change, so the
  // address of a chunk costs a 32->64-bit add and a select.
  constexpr int NBJ = (NBI + 7) / 8;
  int a_hw[MAXA], a_rel[MAXA], a_lds[MAXA], b_rel[NBJ];
#pragma unroll
  for (int i = 0; i < MAXA; ++i) {
    const int q = tid + i * NTHR;
    const int slot = q >> 2;
    const int hh = slot / HWd, ww = slot - hh * HWd;
    a_hw[i] = q < SLOTS * 4 ? ((hh << 8) | ww) : -1;
    a_rel[i] = (int)(hh * a.x.sh + ww * a.x.sw) + (q & 3) * E;
    a_lds[i] = slot * ROWB + (q & 3) * 16;
  }
#pragma unroll
  for (int jj = 0; jj < NBJ; ++jj) {
    const int row = (wave + 8 * jj) * 16 + (lane >> 2);
    const int kc = (lane & 3) ^ ((row >> 2) & 3);
    const int tap = row / NT, nn = row - tap * NT;
    b_rel[jj] = (tap * a.cout_pad + nn) * a.cin_pad + kc * E;
  }
  const int cpart = (tid & 3) * E;  // channel offset of every owned chunk within a stage

  uint4 ra[MAXA];
  unsigned okmask = 0, tinb = 0;
  auto issue = [&](const Tile& tl, int s, int buf) __attribute__((always_inline)) {
    const int kdi = tl.kd_lo + s / nchunk;
    const int c0 = (s % nchunk) * CK;
    const int di = tl.dz + kdi - a.pd;
    const int hb = tl.h0 - a.ph, wb0 = tl.w0 - a.pw;  // halo corner
    if (s == 0) {  // spatial validity of the owned chunks for this tile
      tinb = 0;
#pragma unroll
      for (int i = 0; i < MAXA; ++i) {
        const int hh = a_hw[i] >> 8, ww = a_hw[i] & 0xff;
        const bool ok = a_hw[i] >= 0 && hb + hh >= 0 && hb + hh < a.x.h && wb0 + ww >= 0 && wb0 + ww < a.x.w;
        tinb |= (ok ? 1u : 0u) << i;
      }
    }
    const bool sok = di >= 0 && di < a.x.d && c0 + cpart < a.cin;  // depth / channel validity of the stage
    okmask = sok ? tinb : 0u;
    if constexpr (XM == 0) {
      const T* xb = reinterpret_cast<const T*>(a.x.ptr);
      const T* base = xb + (tl.nb * a.x.sn + (int64_t)di * a.x.sd + (int64_t)hb * a.x.sh + (int64_t)wb0 * a.x.sw + c0);
#pragma unroll
      for (int i = 0; i < MAXA; ++i)
        ra[i] = *reinterpret_cast<const uint4*>(((okmask >> i) & 1) ? base + a_rel[i] : xb);
    } else {
#pragma unroll
      for (int i = 0; i < MAXA; ++i) {
        const bool ok = (okmask >> i) & 1;
        const int hi = hb + (a_hw[i] >> 8), wi = wb0 + (a_hw[i] & 0xff);
        const int c = c0 + cpart;
        if constexpr (XM == 1) {
          ra[i] = *reinterpret_cast<const uint4*>(reinterpret_cast<const T*>(a.x.ptr) +
                                                  view_off(a.x, tl.nb, ok ? di : 0, ok ? hi : 0, ok ? wi : 0,
                                                           ok ? c : 0));
        } else {
          ra[i] = ok ? load_raw<T>(a.x, tl.nb, di, hi, wi, c, a.cin, false) : make_uint4(0, 0, 0, 0);
        }
      }
    }
    // B (weights, identical for every workgroup): LDS-DMA into buffer `buf`,
    // 64-byte rows [tap*NT + n]; chunk position p of row n holds k-chunk
    // p ^ ((n>>2)&3) (swizzle applied on the source address: LDS-DMA writes
    // lane-linear) so the ds_read_b128 column slices are conflict-free.
    const T* wb = reinterpret_cast<const T*>(a.w) + (int64_t)kdi * TAPS * a.cout_pad * a.cin_pad +
                  (int64_t)tl.n0 * a.cin_pad + c0;
    char* bdst = ldsB + buf * BBYTES;
#pragma unroll
    for (int jj = 0; jj < NBJ; ++jj) {
      const int gi = wave + 8 * jj;
      if (gi < NBI) glds16(wb + b_rel[jj], __builtin_amdgcn_readfirstlane(lds_addr(bdst + gi * 1024)));
    }
  };
  auto commit = [&](int s) __attribute__((always_inline)) {
    const int c = (s % nchunk) * CK + cpart;
    const bool partial = c + E > a.cin;
#pragma unroll
    for (int i = 0; i < MAXA; ++i) {
      if (a_hw[i] >= 0) {
        uint4 v = ra[i];
        if (XM != 2 && partial) v = mask_tail<T>(v, a.cin - c);
        if (a.prologue) v = prologue_lds<T>(v, c, relu_in, lsc, lsh);
        if (!((okmask >> i) & 1)) v = make_uint4(0, 0, 0, 0);
        *reinterpret_cast<uint4*>(ldsA + a_lds[i]) = v;
      }
    }
  };

  f32x16 acc[MS][NS];
#pragma unroll
  for (int m = 0; m < MS; ++m)
#pragma unroll
    for (int n = 0; n < NS; ++n)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[m][n][i] = 0.f;

  // Epilogue, per (row, 32-channel block): all of its loads (mask, residual,
  // accumulate target; kept packed) are issued before any of its stores,
  // since a store might alias them and would otherwise serialise one round
  // trip per 4-channel group.
  auto epilogue = [&](const Tile& tl) __attribute__((always_inline)) {
    using Pk = typename std::conditional<sizeof(YT) == 4, uint4, uint2>::type;
#pragma unroll
    for (int ms = 0; ms < MS; ++ms) {
      const int ho = tl.h0 + wave * MS + ms, wo = tl.w0 + r;
      const bool row_ok = ho < a.y.h && wo < a.y.w;
#pragma unroll
      for (int ns = 0; ns < NS; ++ns) {
        Pk mv[4], rv[4], ov[4];
        int64_t yoff[4];
        int valid[4];
        bool vecs[4];
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int co = tl.n0 + ns * 32 + 8 * g + 4 * hf;
          const bool ok = row_ok && co < a.cout;
          valid[g] = ok ? min(4, a.cout - co) : 0;
          const int64_t yo = ok ? view_off(a.y, tl.nb, tl.dz, ho, wo, co) : 0;
          vecs[g] = (valid[g] == 4) && ((yo & 3) == 0) && ((((uintptr_t)a.y.ptr) & (4 * sizeof(YT) - 1)) == 0);
          yoff[g] = yo;
          if (ok) {
            if (a.has_mask) mv[g] = load_pk<YT, Pk>(a.msk.ptr, view_off(a.msk, tl.nb, tl.dz, ho, wo, co), vecs[g], valid[g]);
            if (a.has_res) rv[g] = load_pk<YT, Pk>(a.res.ptr, view_off(a.res, tl.nb, tl.dz, ho, wo, co), vecs[g], valid[g]);
            if (a.accumulate) ov[g] = load_pk<YT, Pk>(a.y.ptr, yo, vecs[g], valid[g]);
          }
        }
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int co = tl.n0 + ns * 32 + 8 * g + 4 * hf;
          if (valid[g] > 0) {
            float v[4], m[4], rr[4], o[4];
            if (a.has_mask) unpack_pk<YT>(mv[g], m);
            if (a.has_res) unpack_pk<YT>(rv[g], rr);
            if (a.accumulate) unpack_pk<YT>(ov[g], o);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              float t = (acc[ms][ns][4 * g + e] + lbias_all[co + e]) * a.out_scale;
              t = act_apply(a.act, t, aslope);
              if (a.has_mask) t = mask_apply(m[e], t, mslope);
              if (a.has_res) t += rr[e];
              if (a.accumulate) t += o[e];
              v[e] = t;
            }
            YT* yp = reinterpret_cast<YT*>(a.y.ptr) + yoff[g];
            if (vecs[g]) {
              *reinterpret_cast<Pk*>(yp) = pack_pk<YT, Pk>(v);
            } else {
              for (int e = 0; e < valid[g]; ++e) yp[e] = from_f32<YT>(v[e]);
            }
          }
        }
      }
    }
#pragma unroll
    for (int m = 0; m < MS; ++m)
#pragma unroll
      for (int n = 0; n < NS; ++n)
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[m][n][i] = 0.f;
  };

  int t = t_lo + j;
  if (t >= t_hi) return;
  Tile cur = decode(t);
  int s = 0, buf = 0;
  issue(cur, 0, 0);
  __syncthreads();  // bias / prologue tables visible
  commit(0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  const int xr = (r >> 2) & 3;  // B swizzle of this lane's rows
  const char* pa0 = ldsA + (wave * MS * HWd + r) * ROWB + hf * 16;
  while (true) {
    // next stage (possibly the first stage of the next tile)
    Tile nxt = cur;
    int ns_ = s + 1;
    bool have_next = true;
    if (ns_ >= cur.nst) {
      ns_ = 0;
      const int tn = t + gx;
      if (tn < t_hi) nxt = decode(tn); else have_next = false;
    }
    if (have_next) issue(nxt, ns_, buf ^ 1);
    const char* pb0 = ldsB + buf * BBYTES + r * 64;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
      for (int khi = 0; khi < KK; ++khi) {
#pragma unroll
        for (int kwi = 0; kwi < KK; ++kwi) {
          const int tap = khi * KK + kwi;
          uint4 bx[MS], aw[NS];
#pragma unroll
          for (int ms = 0; ms < MS; ++ms)
            bx[ms] = *reinterpret_cast<const uint4*>(pa0 + ((ms + khi) * HWd + kwi) * ROWB + ks * 32);
#pragma unroll
          for (int ns = 0; ns < NS; ++ns)
            aw[ns] = *reinterpret_cast<const uint4*>(pb0 + (tap * NT + ns * 32) * 64 + (((ks * 2 + hf) ^ xr) << 4));
#pragma unroll
          for (int ms = 0; ms < MS; ++ms)
#pragma unroll
            for (int ns = 0; ns < NS; ++ns) mma<T>(acc[ms][ns], aw[ns], bx[ms]);
        }
      }
    }
    if (s + 1 >= cur.nst) epilogue(cur);
    if (!have_next) break;
    __syncthreads();  // every wave is done reading A and B[buf]
    commit(ns_);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // B[buf^1] has landed
    __syncthreads();
    if (ns_ == 0) t += gx;
    cur = nxt;
    s = ns_;
    buf ^= 1;
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

// one launch for many weights: blockIdx.y = weight, grid-stride in x
template <typename T>
__global__ void pack_weights_kernel(const vsrk_pack_desc* __restrict__ descs) {
  const vsrk_pack_desc d = descs[blockIdx.y];
  const int co_pad = round_up(d.mode == 0 ? d.cout : d.cin, 128), ci_pad = round_up(d.mode == 0 ? d.cin : d.cout, 32);
  const int64_t total = (int64_t)d.kd * d.kh * d.kw * co_pad * ci_pad;
  T* out = reinterpret_cast<T*>(d.packed);
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total; idx += (int64_t)gridDim.x * blockDim.x) {
    const int i = idx % ci_pad;
    const int64_t t1 = idx / ci_pad;
    const int o = t1 % co_pad;
    const int tap = t1 / co_pad;
    const int kwi = tap % d.kw, khi = (tap / d.kw) % d.kh, kdi = tap / (d.kw * d.kh);
    int co, ci, sd, sh, sw;
    if (d.mode == 0) {
      co = o; ci = i; sd = kdi; sh = khi; sw = kwi;
    } else {
      co = i; ci = o; sd = d.kd - 1 - kdi; sh = d.kh - 1 - khi; sw = d.kw - 1 - kwi;
    }
    float v = 0.f;
    if (co < d.cout && ci < d.cin) {
      int cot = co;
      if (d.perm_r > 1) {
        const int rr = d.perm_r * d.perm_r, cp = d.cout / rr;
        const int sub = co / cp, cc = co - sub * cp;
        cot = cc * rr + sub;
      }
      v = d.w[((((int64_t)cot * d.cin + ci) * d.kd + sd) * d.kh + sh) * d.kw + sw];
    }
    out[idx] = from_f32<T>(v);
  }
}

}  // namespace
extern "C" size_t vsrk_conv_packed_elems(int32_t cout, int32_t cin, int32_t kd, int32_t kh, int32_t kw,
                                         int32_t mode) {
  const int co = mode == 0 ? cout : cin, ci = mode == 0 ? cin : cout;
  return (size_t)kd * kh * kw * round_up(co, 128) * round_up(ci, 32);
}

extern "C" int vsrk_conv_pack_weight(int32_t dtype, const float* w, int32_t cout, int32_t cin, int32_t kd,
                                     int32_t kh, int32_t kw, int32_t mode, int32_t perm_r, void* packed,
                                     void* stream) {
  VSRK_CHECK(w && packed, "conv_pack_weight: null pointer");
  VSRK_CHECK(mode == 0 || mode == 1, "conv_pack_weight: mode must be 0 or 1");
  VSRK_CHECK(perm_r <= 1 || cout % (perm_r * perm_r) == 0, "conv_pack_weight: cout %% r^2 != 0");
  const int co = mode == 0 ? cout : cin, ci = mode == 0 ? cin : cout;
  const int co_pad = round_up(co, 128), ci_pad = round_up(ci, 32);
  const int64_t total = (int64_t)kd * kh * kw * co_pad * ci_pad;
  const int blk = 256;
  const int grid = (int)ceil_div64(total, blk);
  hipStream_t s = (hipStream_t)stream;
  if (dtype == VSRK_BF16)
    pack_weight_kernel<bf16><<<grid, blk, 0, s>>>(w, (bf16*)packed, cout, cin, kd, kh, kw, mode, perm_r,
                                                  co_pad, ci_pad, total);
  else if (dtype == VSRK_F16)
    pack_weight_kernel<f16><<<grid, blk, 0, s>>>(w, (f16*)packed, cout, cin, kd, kh, kw, mode, perm_r,
                                                 co_pad, ci_pad, total);
  else
    pack_weight_kernel<float><<<grid, blk, 0, s>>>(w, (float*)packed, cout, cin, kd, kh, kw, mode, perm_r,
                                                   co_pad, ci_pad, total);
  VSRK_LAUNCH_CHECK("conv_pack_weight");
  return VSRK_OK;
}

extern "C" int vsrk_conv_pack_weights(int32_t dtype, int32_t n, const vsrk_pack_desc* descs, int64_t max_elems,
                                      void* stream) {
  VSRK_CHECK(descs && n >= 0 && n < 65536 && max_elems >= 0, "conv_pack_weights: bad argument");
  if (n == 0 || max_elems == 0) return VSRK_OK;
  const int gx = (int)std::min<int64_t>(ceil_div64(max_elems, 256), 256);
  hipStream_t s = (hipStream_t)stream;
  if (dtype == VSRK_BF16) pack_weights_kernel<bf16><<<dim3(gx, n), 256, 0, s>>>(descs);
  else if (dtype == VSRK_F16) pack_weights_kernel<f16><<<dim3(gx, n), 256, 0, s>>>(descs);
  else pack_weights_kernel<float><<<dim3(gx, n), 256, 0, s>>>(descs);
  VSRK_LAUNCH_CHECK("conv_pack_weights");
  return VSRK_OK;
}

static int num_cus() {
  static int n = 0;
  if (n == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
  }
  return n;
}

template <typename T, int NT, int KK, int XM, typename YT>
static int launch_fwd(ConvArgs a, hipStream_t s) {
  constexpr int MS = NT >= 128 ? 1 : 2;  // rows per wave: keeps acc + staging under 256 VGPRs
  constexpr int FTH = 8 * MS;
  a.tiles_h = ceil_div(a.y.h, FTH);
  const int64_t ntiles = (int64_t)a.y.n * a.y.d * a.tiles_h * a.tiles_w * a.ntn;
  VSRK_CHECK(ntiles < (1ll << 31), "conv_fwd: too many tiles");
  a.ntiles = (int)ntiles;
  if (a.ntiles == 0) return VSRK_OK;
  const int slots = (FTH + KK - 1) * (TW + KK - 1);
  const size_t lds = (size_t)slots * ROWB + 2 * (size_t)KK * KK * NT * 64 + (size_t)a.cout_pad * 4 +
                     (a.prologue ? 2 * a.cin_pad * 4 : 0);
  auto kern = conv_fwd_kernel<T, NT, MS, KK, XM, YT>;
  if (lds > 64 * 1024) (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  int per_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)kern, NTHR, lds) != hipSuccess || per_cu < 1)
    per_cu = 1;
  const int64_t grid = vsrk_capped_grid(std::min<int64_t>(ntiles, (int64_t)num_cus() * per_cu));
  a.nblk = (int)grid;
  kern<<<a.nblk, NTHR, lds, s>>>(a);
  VSRK_LAUNCH_CHECK("conv_fwd");
  return VSRK_OK;
}

template <typename T, int KK, int XM, typename YT>
static int dispatch_nt(const ConvArgs& a, int nt, hipStream_t s) {
  if (nt == 32) return launch_fwd<T, 32, KK, XM, YT>(a, s);
  if (nt == 64) return launch_fwd<T, 64, KK, XM, YT>(a, s);
  return launch_fwd<T, 128, KK, XM, YT>(a, s);
}

template <typename T, int KK, typename YT>
static int dispatch_xm(const ConvArgs& a, int nt, int xm, hipStream_t s) {
  if (xm == 0) return dispatch_nt<T, KK, 0, YT>(a, nt, s);
  if (xm == 1) return dispatch_nt<T, KK, 1, YT>(a, nt, s);
  return dispatch_nt<T, KK, 2, YT>(a, nt, s);
}

template <typename T, typename YT>
static int dispatch_k(const ConvArgs& a, int nt, hipStream_t s) {
  // addressing mode of the input view (see conv_fwd_kernel)
  const int64_t span = (int64_t)(8 * 2 + 2) * a.x.sh + (int64_t)(TW + 2) * a.x.sw + 64;
  const int xm = !a.xvec ? 2 : (a.x.r > 1 || span >= (1ll << 31)) ? 1 : 0;
  if (a.kh == 1) return dispatch_xm<T, 1, YT>(a, nt, xm, s);
  return dispatch_xm<T, 3, YT>(a, nt, xm, s);
}

extern "C" int vsrk_conv_fwd(const vsrk_conv_desc* d, const vsrk_tensor5* x, const void* w_packed,
                             const float* bias, const float* pro_scale, const float* pro_shift,
                             const vsrk_tensor5* residual, const vsrk_tensor5* mask, const vsrk_tensor5* y,
                             void* stream) {
  VSRK_CHECK(d && x && y && w_packed, "conv_fwd: null argument");
  const int xdt = x->dtype, ydt = y->dtype;
  VSRK_CHECK(xdt == VSRK_F32 || vsrk_is16(xdt), "conv_fwd: bad x dtype");
  VSRK_CHECK(ydt == xdt || ydt == VSRK_F32, "conv_fwd: y dtype must equal x dtype or be f32");
  const int es = vsrk_esize(xdt);
  if (!view_ok(x, "conv_fwd x") || !view_ok(y, "conv_fwd y")) return VSRK_ERR_INVALID;
  VSRK_CHECK(d->kh == d->kw && (d->kh == 1 || d->kh == 3) && d->kd >= 1,
             "conv_fwd: kernel %dx%dx%d unsupported (kh = kw in {1, 3})", d->kd, d->kh, d->kw);
  VSRK_CHECK(x->n == y->n, "conv_fwd: batch mismatch");
  VSRK_CHECK(x->h < 32768 && x->w < 32768, "conv_fwd: spatial size too large");
  VSRK_CHECK(!(d->prologue & VSRK_PRO_AFFINE) || (pro_scale && pro_shift), "conv_fwd: affine prologue needs scale/shift");
  VSRK_CHECK(d->act != VSRK_ACT_PRELU || d->act_param, "conv_fwd: PReLU activation needs act_param");
  VSRK_CHECK(d->act >= VSRK_ACT_NONE && d->act <= VSRK_ACT_PRELU, "conv_fwd: bad act %d", d->act);
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
  a.res = residual ? make_view(residual) : a.y;
  a.msk = mask ? make_view(mask) : a.y;
  a.w = (const char*)w_packed;
  a.bias = bias;
  a.pro_scale = pro_scale;
  a.pro_shift = pro_shift;
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
  a.xvec = chunk_ok(x, es);
  a.bias_r = d->bias_perm_r;
  a.out_scale = d->out_scale;
  a.act_param = d->act_param;
  a.mask_slope = d->mask_slope;
  a.tiles_w = ceil_div(y->w, TW);
  // NT=128 only for 1x1 kernels (a double-buffered 3x3 weight slice of 128
  // channels would not fit LDS); wider 3x3 outputs use several 64-wide tiles
  const int NT = y->c <= 32 ? 32 : ((y->c <= 64 || d->kh == 3) ? 64 : 128);
  a.ntn = ceil_div(y->c, NT);
  hipStream_t s = (hipStream_t)stream;
  // VSRK_LOG_DISPATCH=1: one stderr line per launch -- the path taken and the shapes (diagnostics)
  static int log_dispatch = -1;
  if (log_dispatch < 0) {
    const char* e = getenv("VSRK_LOG_DISPATCH");
    log_dispatch = (e && e[0] == '1') ? 1 : 0;
  }
  auto logd = [&](const char* path) {
    if (log_dispatch)
      fprintf(stderr, "vsrk_conv_fwd %s k=%dx%dx%d x=(%d,%d,%d,%d,%d) y=(%d,%d,%d,%d,%d)%s pro=%d act=%d mask=%d res=%d acc=%d\n",
              path, d->kd, d->kh, d->kw, x->n, x->d, x->h, x->w, x->c, y->n, y->d, y->h, y->w, y->c,
              ydt == VSRK_F32 ? " f32out" : "", d->prologue, d->act, mask != nullptr, residual != nullptr, d->accumulate);
  };
  const int wide = vsrk_conv_fwd_pw_wide(d, x, w_packed, bias, residual, mask, y, s);
  if (wide != 0) {
    logd("pw_wide");
    return wide > 0 ? VSRK_OK : -wide;
  }
  const int pw = vsrk_conv_fwd_pw(d, x, w_packed, bias, pro_scale, pro_shift, residual, mask, y, s);
  if (pw != 0) {
    logd("pw");
    return pw > 0 ? VSRK_OK : -pw;
  }
  const int thin = vsrk_conv_fwd_thin(d, x, w_packed, bias, pro_scale, pro_shift, residual, mask, y, s);
  if (thin != 0) {
    logd("thin");
    return thin > 0 ? VSRK_OK : -thin;
  }
  const int fast = vsrk_conv_fwd_fast(d, x, w_packed, bias, pro_scale, pro_shift, residual, mask, y, s);
  if (fast != 0) {
    logd("fast");
    return fast > 0 ? VSRK_OK : -fast;
  }
  logd("tile");
  if (xdt == VSRK_BF16) {
    if (ydt == VSRK_BF16) return dispatch_k<bf16, bf16>(a, NT, s);
    return dispatch_k<bf16, float>(a, NT, s);
  }
  if (xdt == VSRK_F16) {
    if (ydt == VSRK_F16) return dispatch_k<f16, f16>(a, NT, s);
    return dispatch_k<f16, float>(a, NT, s);
  }
  return dispatch_k<float, float>(a, NT, s);
}

