// Implicit-GEMM convolution weight/bias gradient on CDNA4 MFMA (gfx950).
// Design notes: conv_fwd.hip (layout) and the comment block below.
#include <cstdlib>
#include "conv_common.h"

namespace {
using namespace vsrk_conv;

// ---------------------------------------------------------------------------
// weight gradient
// ---------------------------------------------------------------------------
// dW[tap][co][ci] = sum_m dY[m][co] * X[m + tap][ci]: the voxel index m is the
// MFMA k dimension.  A workgroup owns a (32*NCO output x 32*NCI input channel,
// kd tap) combo and a run of 8x32-voxel tiles (split-K over voxels).  Per tile
// it stages dY (NCO planes of 32 channels) and the input halo (NCI planes,
// prologue applied) into LDS once and its 8 waves = NCO x NCI channel blocks x
// NV voxel parts run all kh*kw taps; both operands are read transposed with
// ds_read_b64_tr_b16 (64-byte plane rows: conflict-free).  The next tile's
// loads are in flight during the current tile's MFMAs.  Wave partials are
// summed through LDS in a fixed order into one fp32 slab per (split, combo);
// combos at (ci chunk 0, kd = kd_bias) also produce dbias partials from the
// staged dY.  wgrad_reduce sums slabs in split order: deterministic.
template <typename T, int NCO, int NCI, int KK, bool VEC>
__global__ __attribute__((amdgpu_waves_per_eu(1, 1))) __launch_bounds__(GTHR) void conv_wgrad_kernel(WgradArgs a) {
  constexpr int E = Chunk<T>::E;
  constexpr int PB = 32 * (int)sizeof(T);  // plane row bytes: 32 channels
  constexpr int CPP = PB / 16;             // 16-byte chunks per plane row
  constexpr int NV = 4 / (NCO * NCI);      // voxel parts (waves sharing a channel block)
  constexpr int VOX = GTH * TW;
  constexpr int VPW = VOX / NV;            // voxels per wave
  constexpr int YCPV = NCO * CPP;          // dY chunks per voxel
  constexpr int XCPV = NCI * CPP;          // X chunks per slot
  constexpr int HWd = TW + KK - 1;
  constexpr int SLOTS = (GTH + KK - 1) * HWd;
  constexpr int TAPS = KK * KK;
  constexpr int MAXY = (VOX * YCPV) / GTHR;
  constexpr int MAXX = (SLOTS * XCPV + GTHR - 1) / GTHR;
  extern __shared__ __attribute__((aligned(16))) char lds[];

  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int cis = wave % NCI, cos_ = (wave / NCI) % NCO, vp = wave / (NCI * NCO);
  char* ldsY = lds;                          // [NCO][VOX][PB]
  char* ldsX = lds + NCO * VOX * PB;         // [NCI][SLOTS][PB]
  float* lsc = reinterpret_cast<float*>(ldsX + NCI * SLOTS * PB);
  float* lsh = lsc + a.cin_pad;

  const int L = xcd_remap(blockIdx.x, a.nblk);
  const int split = L / a.ncombos;
  int combo = L - split * a.ncombos;
  const int cot = combo % a.n_co_tiles;
  combo /= a.n_co_tiles;
  const int cic = combo % a.n_ci_chunks;
  const int kdi = combo / a.n_ci_chunks;
  const int co0 = cot * 32 * NCO, ci0 = cic * 32 * NCI;
  const bool do_bias = a.want_bias && cic == 0 && kdi == a.kd_bias;
  const bool relu_in = (a.prologue & VSRK_PRO_RELU) != 0;
  if (a.prologue) {
    stage_prologue(lsc, lsh, a.prologue, a.pro_scale, a.pro_shift, a.cin, a.cin_pad, tid, GTHR);
    __syncthreads();
  }

  // fixed per-thread chunk roles (GTHR is a multiple of YCPV and XCPV)
  const int yrem = tid % YCPV, xrem = tid % XCPV;
  const int yc = co0 + (yrem / CPP) * 32 + (yrem % CPP) * E;  // dY channel of every y chunk
  const int xc = ci0 + (xrem / CPP) * 32 + (xrem % CPP) * E;  // X channel of every x chunk
  const int ydst = (yrem / CPP) * VOX * PB + (yrem % CPP) * 16;
  const int xdst = (xrem / CPP) * SLOTS * PB + (xrem % CPP) * 16;
  const bool yc_ok = yc < a.cout, xc_ok = xc < a.cin;
  const int ycc = yc_ok ? yc : 0, xcc = xc_ok ? xc : 0;

  uint4 ry[MAXY], rx[MAXX];
  unsigned ymask = 0, xmask = 0;  // validity of the chunks in flight
  float bsum[E];
#pragma unroll
  for (int e = 0; e < E; ++e) bsum[e] = 0.f;

  auto tile_ok = [&](int t) __attribute__((always_inline)) {
    const int dz = (t / (a.tiles_w * a.tiles_h)) % a.dy.d;
    const int di = dz + kdi - a.pd;
    return di >= 0 && di < a.x.d;
  };
  auto issue = [&](int t) __attribute__((always_inline)) {
    int b = t;
    const int tw_i = b % a.tiles_w;
    b /= a.tiles_w;
    const int th_i = b % a.tiles_h;
    b /= a.tiles_h;
    const int dz = b % a.dy.d;
    const int nb = b / a.dy.d;
    const int di = dz + kdi - a.pd;
    const int h0 = th_i * GTH, w0 = tw_i * TW;
    ymask = 0;
    xmask = 0;
#pragma unroll
    for (int i = 0; i < MAXY; ++i) {
      const int vox = (tid + i * GTHR) / YCPV;
      const int ho = h0 + vox / TW, wo = w0 + (vox % TW);
      const bool ok = ho < a.dy.h && wo < a.dy.w && yc_ok;
      ymask |= (ok ? 1u : 0u) << i;
      if constexpr (VEC) {
        ry[i] = *reinterpret_cast<const uint4*>(reinterpret_cast<const T*>(a.dy.ptr) +
                                                view_off(a.dy, nb, dz, ok ? ho : 0, ok ? wo : 0, ycc));
      } else {
        ry[i] = ok ? load_raw<T>(a.dy, nb, dz, ho, wo, yc, a.cout, false) : make_uint4(0, 0, 0, 0);
      }
    }
#pragma unroll
    for (int i = 0; i < MAXX; ++i) {
      const int slot = (tid + i * GTHR) / XCPV;
      const int hh = slot / HWd, ww = slot - hh * HWd;
      const int hi = h0 + hh - a.ph, wi = w0 + ww - a.pw;
      const bool ok = slot < SLOTS && hi >= 0 && hi < a.x.h && wi >= 0 && wi < a.x.w && xc_ok;
      xmask |= (ok ? 1u : 0u) << i;
      if constexpr (VEC) {
        rx[i] = *reinterpret_cast<const uint4*>(reinterpret_cast<const T*>(a.x.ptr) +
                                                view_off(a.x, nb, di, ok ? hi : 0, ok ? wi : 0, xcc));
      } else {
        rx[i] = ok ? load_raw<T>(a.x, nb, di, hi, wi, xc, a.cin, false) : make_uint4(0, 0, 0, 0);
      }
    }
  };
  auto commit = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < MAXY; ++i) {
      const int vox = (tid + i * GTHR) / YCPV;
      const uint4 v = ((ymask >> i) & 1) ? ry[i] : make_uint4(0, 0, 0, 0);
      *reinterpret_cast<uint4*>(ldsY + ydst + vox * PB) = v;
      if (do_bias) {
        float f[E];
        Chunk<T>::unpack(v, f);
#pragma unroll
        for (int e = 0; e < E; ++e) bsum[e] += f[e];
      }
    }
#pragma unroll
    for (int i = 0; i < MAXX; ++i) {
      const int slot = (tid + i * GTHR) / XCPV;
      if (slot < SLOTS) {
        uint4 v = rx[i];
        if (a.prologue) v = prologue_lds<T>(v, xc, relu_in, lsc, lsh);
        if (!((xmask >> i) & 1)) v = make_uint4(0, 0, 0, 0);
        *reinterpret_cast<uint4*>(ldsX + xdst + slot * PB) = v;
      }
    }
  };

  f32x16 acc[TAPS];
#pragma unroll
  for (int t = 0; t < TAPS; ++t)
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[t][i] = 0.f;

  const int t_begin = split * a.tiles_per_split;
  const int t_end = min(a.ntiles, t_begin + a.tiles_per_split);
  int t = t_begin;
  while (t < t_end && !tile_ok(t)) ++t;
  if (t < t_end) {
    issue(t);
    commit();
    __syncthreads();
  }
  const char* py = ldsY + cos_ * VOX * PB;
  const char* px = ldsX + cis * SLOTS * PB;
  while (t < t_end) {
    int tn = t + 1;
    while (tn < t_end && !tile_ok(tn)) ++tn;
    if (tn < t_end) issue(tn);
    if constexpr (sizeof(T) == 2) {
      // Group g = lane>>4 reads a 4-row x 16-column block; lane 4q+p
      // addresses row q, columns 4p..4p+3, and receives column lane&15.
      const int g = lane >> 4, i16 = lane & 15, q = i16 >> 2, p = i16 & 3;
      const int hfk = g >> 1, colb = ((g & 1) * 16 + 4 * p) * 2;
#pragma unroll
      for (int ks = 0; ks < VPW / 16; ++ks) {
        const int vb = vp * VPW + ks * 16;
        const int vrow = vb / TW, vcol0 = (vb % TW) + 8 * hfk;
        v4i16 y0 = ds_read_tr(py + (vrow * TW + vcol0 + q) * PB + colb);
        v4i16 y1 = ds_read_tr(py + (vrow * TW + vcol0 + 4 + q) * PB + colb);
        const uint4 af = __builtin_bit_cast(uint4, __builtin_shufflevector(y0, y1, 0, 1, 2, 3, 4, 5, 6, 7));
#pragma unroll
        for (int khi = 0; khi < KK; ++khi) {
#pragma unroll
          for (int kwi = 0; kwi < KK; ++kwi) {
            const char* xs = px + ((vrow + khi) * HWd + vcol0 + kwi + q) * PB + colb;
            v4i16 x0 = ds_read_tr(xs);
            v4i16 x1 = ds_read_tr(xs + 4 * PB);
            const uint4 bfr = __builtin_bit_cast(uint4, __builtin_shufflevector(x0, x1, 0, 1, 2, 3, 4, 5, 6, 7));
            mma<T>(acc[khi * KK + kwi], af, bfr);
          }
        }
      }
    } else {
      // fp32: 32x32x2, lane l: A[co=l&31][k=l>>5], B[k=l>>5][ci=l&31]
      const int r = lane & 31, hfk = lane >> 5;
      for (int kk = 0; kk < VPW; kk += 2) {
        const int vox = vp * VPW + kk + hfk;
        const int vrow = vox / TW, vcol = vox % TW;
        const float av = *reinterpret_cast<const float*>(py + vox * PB + r * 4);
#pragma unroll
        for (int khi = 0; khi < KK; ++khi) {
#pragma unroll
          for (int kwi = 0; kwi < KK; ++kwi) {
            const int sl = (vrow + khi) * HWd + vcol + kwi;
            const float bv = *reinterpret_cast<const float*>(px + sl * PB + r * 4);
            acc[khi * KK + kwi] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bv, acc[khi * KK + kwi], 0, 0, 0);
          }
        }
      }
    }
    if (tn < t_end) {
      __syncthreads();
      commit();
      __syncthreads();
    }
    t = tn;
  }

  // slab layout: [tap][co (32*NCO)][ci (32*NCI)] then dbias[32*NCO]
  float* out = a.ws + (int64_t)L * a.slab;
  constexpr int NW = TAPS * 1024 * NCO * NCI;
  const int r = lane & 31, hfo = lane >> 5;
  if constexpr (NV == 1) {
#pragma unroll
    for (int tap = 0; tap < TAPS; ++tap) {
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int co = cos_ * 32 + (i & 3) + 8 * (i >> 2) + 4 * hfo;
        out[(tap * 32 * NCO + co) * (32 * NCI) + cis * 32 + r] = acc[tap][i];
      }
    }
  } else {
    // fixed-order sum of the NV voxel-part partials: red[cos][cis][tap][co][ci]
    __syncthreads();
    float* red = reinterpret_cast<float*>(lds);
    for (int v = 0; v < NV; ++v) {
      if (vp == v) {
#pragma unroll
        for (int tap = 0; tap < TAPS; ++tap) {
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            const int co = (i & 3) + 8 * (i >> 2) + 4 * hfo;
            float* dst = red + (((cos_ * NCI + cis) * TAPS + tap) * 32 + co) * 32 + r;
            *dst = (v == 0) ? acc[tap][i] : *dst + acc[tap][i];
          }
        }
      }
      __syncthreads();
    }
    for (int i = tid; i < NW; i += GTHR) {
      const int ci = i % (32 * NCI);
      const int t2 = i / (32 * NCI);
      const int co = t2 % (32 * NCO);
      const int tap = t2 / (32 * NCO);
      out[i] = red[((((co / 32) * NCI + ci / 32) * TAPS + tap) * 32 + (co % 32)) * 32 + (ci % 32)];
    }
  }
  if (do_bias) {
    __syncthreads();
    float* red = reinterpret_cast<float*>(lds);
#pragma unroll
    for (int e = 0; e < E; ++e) red[tid * E + e] = bsum[e];
    __syncthreads();
    if (tid < 32 * NCO) {
      const int plane = tid / 32, within = tid % 32;
      const int grp = plane * CPP + within / E, e = within % E;
      float sacc = 0.f;
      for (int kk = grp; kk < GTHR; kk += YCPV) sacc += red[kk * E + e];
      out[NW + tid] = sacc;
    }
  }
}

// dw[co][ci][kd][kh][kw] (torch, fp32) = scale * sum_split slab[split][combo][tap][co][ci]
// (+ dbias from the bias tails).  A block = 64 outputs x 4 split groups; each
// thread sums a strided quarter of the splits, then the 4 partials are added
// in a fixed order: deterministic.
__global__ __launch_bounds__(256) void wgrad_reduce_kernel(
    const float* __restrict__ ws, float* __restrict__ dw, float* __restrict__ db, int nsplit, int ncombos,
    int slab, int cout, int cin, int kd, int kh, int kw, int nco_t, int nci_t, int cot_w, int cit_w, int kd_bias,
    int perm_r, float scale, int accumulate) {
  __shared__ float part[4][64];
  const int taps2 = kh * kw;
  const int64_t nw = (int64_t)cout * cin * kd * taps2;
  const int64_t idx = (int64_t)blockIdx.x * 64 + (threadIdx.x & 63);
  const int grp = threadIdx.x >> 6;
  const int64_t total = nw + (db ? cout : 0);
  const int64_t sstride = (int64_t)ncombos * slab;
  const float* p = nullptr;
  int co = 0, ci = 0, tap = 0, kdi = 0;
  if (idx < nw) {
    ci = idx % cin;
    int64_t t = idx / cin;
    co = t % cout;
    t /= cout;
    tap = t % taps2;
    kdi = t / taps2;
    const int combo = (kdi * nci_t + ci / cit_w) * nco_t + co / cot_w;
    p = ws + (int64_t)combo * slab + ((int64_t)tap * cot_w + (co % cot_w)) * cit_w + (ci % cit_w);
  } else if (idx < total) {
    co = (int)(idx - nw);
    const int combo = (kd_bias * nci_t + 0) * nco_t + co / cot_w;
    p = ws + (int64_t)combo * slab + (int64_t)taps2 * cot_w * cit_w + (co % cot_w);
  }
  float s = 0.f;
  if (p) {
    int k = grp;
    for (; k + 12 < nsplit; k += 16) {
      const float a0 = p[k * sstride], a1 = p[(k + 4) * sstride], a2 = p[(k + 8) * sstride],
                  a3 = p[(k + 12) * sstride];
      s += a0;
      s += a1;
      s += a2;
      s += a3;
    }
    for (; k < nsplit; k += 4) s += p[k * sstride];
  }
  part[grp][threadIdx.x & 63] = s;
  __syncthreads();
  if (grp != 0 || idx >= total) return;
  const int l = threadIdx.x;
  s = ((part[0][l] + part[1][l]) + part[2][l]) + part[3][l];
  int cot = co;
  if (perm_r > 1) {
    const int rr = perm_r * perm_r, cp = cout / rr;
    const int sub = co / cp, cc = co - sub * cp;
    cot = cc * rr + sub;
  }
  s *= scale;
  if (idx < nw) {
    const int khi = tap / kw, kwi = tap % kw;
    float* d = dw + ((((int64_t)cot * cin + ci) * kd + kdi) * kh + khi) * kw + kwi;
    *d = accumulate ? *d + s : s;
  } else {
    db[cot] = accumulate ? db[cot] + s : s;
  }
}

// The same sums as wgrad_reduce_kernel, in dw's memory order: a workgroup
// owns one (output channel, input block of cit_w channels, kd) and its
// cit_w x taps outputs, reads each split's [tap][ci] rows of the slab
// coalesced (8 splits of loads in flight per output), sums the splits in
// order 0, 1, 2, ... in fp32, and writes the (ci, tap) run of dw through LDS.
// Workgroups past the weights sum the dbias tails, one output channel per
// lane.  (wgrad_reduce_kernel writes dw with a 9-float stride per lane: the
// DRF sub-pixel weight gradients spent ~27 us per reduce in it.)
__global__ __launch_bounds__(256) void wgrad_reduce_rows_kernel(
    const float* __restrict__ ws, float* __restrict__ dw, float* __restrict__ db, int nsplit, int slab, int cout,
    int cin, int kd, int taps2, int nco_t, int nci_t, int cot_w, int cit_w, int kd_bias, int perm_r, float scale,
    int accumulate, int nblk_w) {
  constexpr int U = 8;
  __shared__ float out[64 * 9];
  const int64_t sstride = (int64_t)nco_t * nci_t * kd * slab;
  const int tid = threadIdx.x;
  auto sum_splits = [&](const float* p) __attribute__((always_inline)) {
    float s = 0.f;
    for (int k0 = 0; k0 < nsplit; k0 += U) {
      float v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) v[u] = k0 + u < nsplit ? p[(int64_t)(k0 + u) * sstride] : 0.f;
#pragma unroll
      for (int u = 0; u < U; ++u) s += v[u];
    }
    return s;
  };
  auto torch_co = [&](int co) __attribute__((always_inline)) {
    if (perm_r > 1) {
      const int rr = perm_r * perm_r, cp = cout / rr;
      const int sub = co / cp;
      return (co - sub * cp) * rr + sub;
    }
    return co;
  };
  if ((int)blockIdx.x >= nblk_w) {  // dbias
    if (!db) return;
    const int co = ((int)blockIdx.x - nblk_w) * 256 + tid;
    if (co >= cout) return;
    const int combo = (kd_bias * nci_t + 0) * nco_t + co / cot_w;
    const float s = sum_splits(ws + (int64_t)combo * slab + (int64_t)taps2 * cot_w * cit_w + (co % cot_w)) * scale;
    const int cot = torch_co(co);
    db[cot] = accumulate ? db[cot] + s : s;
    return;
  }
  int b = blockIdx.x;
  const int kdi = b % kd;
  b /= kd;
  const int cic = b % nci_t;
  const int co = b / nci_t;
  const int ci0 = cic * cit_w;
  const int nci = min(cit_w, cin - ci0);
  const int nout = nci * taps2;
  const int combo = (kdi * nci_t + cic) * nco_t + co / cot_w;
  const float* base = ws + (int64_t)combo * slab + (int64_t)(co % cot_w) * cit_w;
  for (int j = tid; j < cit_w * taps2; j += 256) {  // read order: tap-major rows of cit_w input channels
    const int tap = j / cit_w, cil = j - tap * cit_w;
    if (cil < nci) out[cil * taps2 + tap] = sum_splits(base + (int64_t)tap * cot_w * cit_w + cil) * scale;
  }
  __syncthreads();
  float* d = dw + ((int64_t)torch_co(co) * cin + ci0) * kd * taps2 + (int64_t)kdi * taps2;
  for (int j = tid; j < nout; j += 256) {  // dw order: (ci, [kd,] tap)
    const int cil = j / taps2, tap = j - cil * taps2;
    float* q = d + (int64_t)cil * kd * taps2 + tap;
    *q = accumulate ? *q + out[j] : out[j];
  }
}

// the row-order reduce where it fits; VSRK_WGRAD_REDUCE=0 keeps the per-output kernel (A/B)
static bool wgrad_reduce_rows(const float* ws, float* dw, float* db, int nsplit, int slab, int cout, int cin, int kd,
                              int taps2, int nco_t, int nci_t, int cot_w, int cit_w, int kd_bias, int perm_r,
                              float scale, int accumulate, hipStream_t s) {
  static int mode = -1;
  if (mode < 0) {
    const char* e = getenv("VSRK_WGRAD_REDUCE");
    mode = (e && e[0] == '0') ? 0 : 1;
  }
  const int nblk_w = cout * nci_t * kd;
  // one lane sums all splits of an output: only for few splits and enough
  // workgroups (EDSR's 64 -> 64 has 256 splits over 64 such workgroups)
  if (!mode || cit_w * taps2 > 64 * 9 || nsplit > 32 || nblk_w < 256) return false;
  const int nblk_b = db ? (int)ceil_div64(cout, 256) : 0;
  wgrad_reduce_rows_kernel<<<nblk_w + nblk_b, 256, 0, s>>>(ws, dw, db, nsplit, slab, cout, cin, kd, taps2, nco_t,
                                                            nci_t, cot_w, cit_w, kd_bias, perm_r, scale, accumulate,
                                                            nblk_w);
  return true;
}

}  // namespace
struct WgradPlan {
  int nco, nci;            // channel blocks per workgroup (x32)
  int n_co_tiles, n_ci_chunks, ncombos;
  int ntiles, tps, nsplit, slab;
  size_t ws_bytes;
};

static WgradPlan wgrad_plan(const vsrk_conv_desc* d, const vsrk_tensor5* x, const vsrk_tensor5* dy) {
  WgradPlan p;
  const bool f32 = x->dtype == VSRK_F32;
  p.nco = (!f32 && dy->c > 32) ? 2 : 1;
  p.nci = (!f32 && x->c > 32) ? 2 : 1;
  p.n_co_tiles = ceil_div(dy->c, 32 * p.nco);
  p.n_ci_chunks = ceil_div(x->c, 32 * p.nci);
  p.ncombos = p.n_co_tiles * p.n_ci_chunks * d->kd;
  p.ntiles = dy->n * dy->d * ceil_div(dy->h, GTH) * ceil_div(dy->w, TW);
  // Splits (workgroups per combo): about 512 workgroups (two resident per
  // CU), but no fewer than 16 tiles (of 8x32 voxels) per workgroup while that
  // still leaves one workgroup per CU: each workgroup writes a whole fp32 slab
  // and the reduce reads it back, which at 8 tiles per workgroup cost the
  // EDSR 64->64 wgrad 10 % (147 -> 133 us at 256 workgroups; DUF's 3x3x3,
  // at 24 tiles per workgroup, keeps its 512: 231 vs 324 us at 256).
  // VSRK_WGRAD_TARGET=<workgroups> overrides the rule (A/B only).
  static int target = -1;
  if (target < 0) {
    const char* e = getenv("VSRK_WGRAD_TARGET");
    target = e ? std::max(64, atoi(e)) : 0;
  }
  // 3-D (kd > 1): about 64 tiles per workgroup (at least one workgroup per
  // CU).  The pipelined kernel's sweep (profiles/r2_wgrad_pipe_ab.txt): DUF
  // 64->32 at 64 x 7 x 128 x 128 fastest at ~1024 workgroups (~84 tiles
  // each), 224->32 at ~4096 (~60 tiles each); the 2-D EDSR 64->64 is fastest
  // at 512.
  int want;
  if (target) want = ceil_div(target, p.ncombos);
  else if (d->kd > 1) want = std::max(ceil_div(p.ntiles, 64), ceil_div(256, p.ncombos));
  else want = std::min(ceil_div(512, p.ncombos), std::max(ceil_div(p.ntiles, 16), ceil_div(256, p.ncombos)));
  if (vsrk_g_grid_cap > 0) want = std::max(1, vsrk_g_grid_cap / p.ncombos);
  want = std::max(1, std::min(want, p.ntiles));
  p.tps = ceil_div(p.ntiles, want);
  p.nsplit = ceil_div(p.ntiles, p.tps);
  p.slab = d->kh * d->kw * 1024 * p.nco * p.nci + 32 * p.nco;
  p.ws_bytes = (size_t)p.nsplit * p.ncombos * p.slab * sizeof(float);
  return p;
}

// Views spanning more than the rolling weight gradient's 32-bit element
// offsets (DUF's concat buffer at cfg 5) run in sample chunks that fit: the
// chunk's sample count, 0 when no split applies
static int wgrad_roll_chunk(const vsrk_tensor5* x, const vsrk_tensor5* dy) {
  auto fits = [&](int64_t n) {
    for (const vsrk_tensor5* t : {x, dy})
      if (n * t->sn + (int64_t)t->d * t->sd + (int64_t)(t->h + 64) * t->sh + (int64_t)(t->w + 64) * t->sw + t->c >=
          (1ll << 31))
        return false;
    return true;
  };
  if (x->n <= 1 || x->n != dy->n || x->sn < 0 || dy->sn < 0 || fits(x->n)) return 0;
  int nc = x->n;
  while (nc > 1 && !fits(nc)) nc = (nc + 1) / 2;
  return fits(nc) ? nc : 0;
}

extern "C" size_t vsrk_conv_wgrad_workspace_size(const vsrk_conv_desc* d, const vsrk_tensor5* x,
                                                 const vsrk_tensor5* dy) {
  int ns, tps, nt, dzc;
  size_t roll = 0;
  if (!vsrk_wgrad_roll_plan(d, x, dy, &ns, &tps, &nt, &dzc, &roll)) {
    roll = 0;
    if (const int nc = wgrad_roll_chunk(x, dy)) {  // the sample chunks' plan
      vsrk_tensor5 xc = *x, gc = *dy;
      xc.n = gc.n = nc;
      if (!vsrk_wgrad_roll_plan(d, &xc, &gc, &ns, &tps, &nt, &dzc, &roll)) roll = 0;
    }
  }
  VsrkRowPlan rp;
  const size_t row = vsrk_wgrad_row_plan(d, x, dy, &rp) ? rp.ws_bytes : 0;
  return std::max(std::max(std::max(wgrad_plan(d, x, dy).ws_bytes, vsrk_conv_wgrad_pw_workspace(d, x, dy)), roll), row);
}

template <typename T, int NCO, int NCI, int KK, bool VEC>
static void launch_wgrad(const WgradArgs& a, hipStream_t s) {
  constexpr int PB = 32 * (int)sizeof(T);
  constexpr int SLOTS = (GTH + KK - 1) * (TW + KK - 1);
  const size_t stage = (size_t)(NCO * GTH * TW + NCI * SLOTS) * PB + (a.prologue ? 2 * a.cin_pad * 4 : 0);
  const size_t red = (4 / (NCO * NCI)) > 1 ? (size_t)NCO * NCI * KK * KK * 1024 * sizeof(float) : 0;
  const size_t bias = (size_t)GTHR * (16 / sizeof(T)) * sizeof(float);
  const size_t lds = std::max(stage, std::max(red, bias));
  auto kern = conv_wgrad_kernel<T, NCO, NCI, KK, VEC>;
  (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  kern<<<a.nblk, GTHR, lds, s>>>(a);
}

template <typename T, int NCO, int NCI>
static void wgrad_k(const WgradArgs& a, bool vec, hipStream_t s) {
  if (a.kh == 1) {
    if (vec) launch_wgrad<T, NCO, NCI, 1, true>(a, s); else launch_wgrad<T, NCO, NCI, 1, false>(a, s);
  } else {
    if (vec) launch_wgrad<T, NCO, NCI, 3, true>(a, s); else launch_wgrad<T, NCO, NCI, 3, false>(a, s);
  }
}

extern "C" int vsrk_conv_wgrad(const vsrk_conv_desc* d, const vsrk_tensor5* x, const vsrk_tensor5* dy,
                               const float* pro_scale, const float* pro_shift, float dy_scale, int32_t perm_r,
                               float* dw, float* dbias, int32_t accumulate, void* workspace,
                               size_t workspace_bytes, void* stream) {
  VSRK_CHECK(d && x && dy && dw, "conv_wgrad: null argument");
  VSRK_CHECK(x->dtype == dy->dtype, "conv_wgrad: x/dy dtype mismatch");
  const int es = vsrk_esize(x->dtype);
  if (!view_ok(x, "conv_wgrad x") || !view_ok(dy, "conv_wgrad dy")) return VSRK_ERR_INVALID;
  VSRK_CHECK(d->kh == d->kw && (d->kh == 1 || d->kh == 3), "conv_wgrad: kh = kw in {1, 3}");
  VSRK_CHECK(!(d->prologue & VSRK_PRO_AFFINE) || (pro_scale && pro_shift), "conv_wgrad: affine prologue needs scale/shift");
  hipStream_t s = (hipStream_t)stream;
  const int pw = vsrk_conv_wgrad_pw(d, x, dy, pro_scale, pro_shift, dy_scale, perm_r, dw, dbias, accumulate,
                                    workspace, workspace_bytes, s);
  if (pw != 0) return pw > 0 ? VSRK_OK : -pw;
  if (workspace && dy->n * dy->d * dy->h * dy->w > 0) {
    // rolling-depth 3x3x3 kernel (conv_wgrad_roll.hip): its slabs, the same reduce
    auto roll = [&](const vsrk_tensor5* xv, const vsrk_tensor5* gv, int32_t acc) -> bool {
      int ns = 0;
      if (!vsrk_conv_wgrad_roll(d, xv, gv, pro_scale, pro_shift, dbias != nullptr, (float*)workspace, workspace_bytes,
                                &ns, s))
        return false;
      const int nci = x->c / 32, nco = dy->c / 32;
      const int64_t total = (int64_t)dy->c * x->c * 27 + (dbias ? dy->c : 0);
      if (!wgrad_reduce_rows((const float*)workspace, dw, dbias, 2 * ns, 9 * 1024 + 32, dy->c, x->c, 3, 9, nco, nci,
                             32, 32, std::min(d->pd, 2), perm_r, dy_scale, acc, s))
        wgrad_reduce_kernel<<<(int)ceil_div64(total, 64), 256, 0, s>>>(
            (const float*)workspace, dw, dbias, 2 * ns, 3 * nci * nco, 9 * 1024 + 32, dy->c, x->c, 3, 3, 3, nco, nci,
            32, 32, std::min(d->pd, 2), perm_r, dy_scale, acc);
      return true;
    };
    if (roll(x, dy, accumulate)) {
      VSRK_LAUNCH_CHECK("conv_wgrad(roll)");
      return VSRK_OK;
    }
    // views spanning more than the kernel's 32-bit element offsets (DUF's
    // concat buffer at cfg 5): sample chunks that fit, each reduced onto dw
    // after the first (fixed chunk order: deterministic)
    if (const int nc = wgrad_roll_chunk(x, dy)) {
      bool ok = true;
      for (int n0 = 0; ok && n0 < x->n; n0 += nc) {
        vsrk_tensor5 xc = *x, gc = *dy;
        xc.n = gc.n = std::min(nc, x->n - n0);
        xc.ptr = (char*)x->ptr + (int64_t)n0 * x->sn * es;
        gc.ptr = (char*)dy->ptr + (int64_t)n0 * dy->sn * es;
        if (!roll(&xc, &gc, n0 == 0 ? accumulate : 1)) {
          VSRK_CHECK(n0 == 0, "conv_wgrad(roll): a sample chunk was not eligible");
          ok = false;  // nothing launched: the other paths below
        }
      }
      if (ok) {
        VSRK_LAUNCH_CHECK("conv_wgrad(roll, sample chunks)");
        return VSRK_OK;
      }
    }
  }
  if (workspace && dy->n * dy->d * dy->h * dy->w > 0) {
    // rolling-row Conv2d 3x3 kernel (conv_wgrad_row.hip): 32 x 64 channel slabs
    VsrkRowPlan rp;
    if (vsrk_conv_wgrad_row(d, x, dy, dbias != nullptr, (float*)workspace, workspace_bytes, &rp, s)) {
      VSRK_LAUNCH_CHECK("conv_wgrad(row)");
      const int64_t total = (int64_t)dy->c * x->c * 9 + (dbias ? dy->c : 0);
      wgrad_reduce_kernel<<<(int)ceil_div64(total, 64), 256, 0, s>>>(
          (const float*)workspace, dw, dbias, rp.nsplit, rp.ncot * rp.ncic, rp.slab, dy->c, x->c, 1, 3, 3,
          rp.ncot, rp.ncic, rp.cot_w, 64, 0, perm_r, dy_scale, accumulate);
      VSRK_LAUNCH_CHECK("conv_wgrad_reduce");
      return VSRK_OK;
    }
  }
  const WgradPlan p = wgrad_plan(d, x, dy);
  VSRK_CHECK(workspace && workspace_bytes >= p.ws_bytes, "conv_wgrad: workspace %zu < %zu bytes", workspace_bytes,
             p.ws_bytes);
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
  a.tiles_h = ceil_div(dy->h, GTH);
  a.tiles_w = ceil_div(dy->w, TW);
  a.ntiles = p.ntiles;
  a.tiles_per_split = p.tps;
  a.nsplit = p.nsplit;
  a.ncombos = p.ncombos;
  a.nblk = p.nsplit * p.ncombos;
  a.n_ci_chunks = p.n_ci_chunks;
  a.n_co_tiles = p.n_co_tiles;
  a.kd_bias = std::min(d->pd, d->kd - 1);
  a.slab = p.slab;
  a.want_bias = dbias != nullptr;
  a.cin_pad = round_up(x->c, 32 * p.nci);
  a.sp_by = 0;
  if (d->subpixel && d->kd == 1 && d->kh == 3 && d->kw == 3 && ((x->shuffle > 1) != (dy->shuffle > 1))) {
    const vsrk_tensor5* t = dy->shuffle > 1 ? dy : x;
    const int r = t->shuffle, cph = t->c / (r * r);
    if (cph % 32 == 0 && t->c / 32 <= 64) {
      a.sp_by = dy->shuffle > 1 ? 1 : 2;
      const int32_t code = d->subpixel & ~(1 << 25);  // gradients of the forward (unflipped) taps
      for (int b = 0; b < t->c / 32; ++b) a.sptap[b] = subpixel_tapmask(code, r, b * 32 / cph);
    }
  }
  if (p.ntiles == 0) return VSRK_OK;
  const bool vec = a.xvec && a.dyvec;
  if (vsrk_is16(x->dtype) && vsrk_conv_wgrad_thin(a, p.nco, p.nci, perm_r, x->dtype, s)) {
    // thin-channel kernel (conv_thin.hip), same slab layout
  } else if (vsrk_is16(x->dtype) && vsrk_conv_wgrad_pipe(a, p.nco, p.nci, x->dtype, s)) {
    // two-stage pipelined kernel (conv_wgrad_pipe.hip), same slab layout
  } else if (vsrk_is16(x->dtype)) {
    vsrk_dispatch16(x->dtype, [&](auto tag) {
      using H = decltype(tag);
      if (p.nco == 2 && p.nci == 2) wgrad_k<H, 2, 2>(a, vec, s);
      else if (p.nco == 2) wgrad_k<H, 2, 1>(a, vec, s);
      else if (p.nci == 2) wgrad_k<H, 1, 2>(a, vec, s);
      else wgrad_k<H, 1, 1>(a, vec, s);
      return 0;
    });
  } else {
    wgrad_k<float, 1, 1>(a, vec, s);
  }
  VSRK_LAUNCH_CHECK("conv_wgrad");
  const int64_t total = (int64_t)dy->c * x->c * d->kd * d->kh * d->kw + (dbias ? dy->c : 0);
  if (!wgrad_reduce_rows((const float*)workspace, dw, dbias, p.nsplit, p.slab, dy->c, x->c, d->kd, d->kh * d->kw,
                         p.n_co_tiles, p.n_ci_chunks, 32 * p.nco, 32 * p.nci, a.kd_bias, perm_r, dy_scale, accumulate,
                         s))
    wgrad_reduce_kernel<<<(int)ceil_div64(total, 64), 256, 0, s>>>(
        (const float*)workspace, dw, dbias, p.nsplit, p.ncombos, p.slab, dy->c, x->c, d->kd, d->kh, d->kw,
        p.n_co_tiles, p.n_ci_chunks, 32 * p.nco, 32 * p.nci, a.kd_bias, perm_r, dy_scale, accumulate);
  VSRK_LAUNCH_CHECK("conv_wgrad_reduce");
  return VSRK_OK;
}
