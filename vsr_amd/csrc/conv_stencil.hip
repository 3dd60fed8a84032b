// Stencil form of the 3x3 convolutions with ONE input channel: the network
// head nn.Conv2d(1, 64, 3, padding=1) (edsr_net.py:28; duf_net.py:35 and
// drf_net.py:25 are the same shape) and the data gradient of EDSR's tail
// conv nn.Conv2d(64, 1, 3, padding=1) (edsr_net.py:32), which at 4x
// 512 x 512 writes 64 channels for every HR voxel: 2.15 GB of output per cfg-2
// step against 0.27 GB of input, so the kernel is a store stream.
//
// out[v][co] = act(out_scale * (bias[co] + sum_tap W[tap][co] * x[v + tap]))
// is 9 multiply-adds per output element: plain VALU, no MFMA.  A workgroup
// walks tiles of 8 x 64 output voxels; the tile's 10 x 66 input patch (one
// channel, read from the 8-channel padded storage the nets keep) is converted
// to fp32 in LDS (double-buffered; the next tile's patch is loaded into
// registers while this tile computes).  Lane l of a wave owns the 8 output
// channels 8 (l & 7) .. +7 -- their 72 weights stay in registers -- of voxel
// l >> 3, so every store instruction writes 8 whole 128-byte voxel rows
// (1 KB contiguous).  The implicit-GEMM thin-input kernel (conv_thin.hip)
// it replaces for these shapes ran the tail data gradient at 2.1 TB/s.
#include <algorithm>
#include <cstdlib>
#include "conv_common.h"
#include "vsrk_internal.h"

namespace {
using namespace vsrk_conv;

constexpr int ST_THR = 256;                              // 4 waves
constexpr int ST_TR = 8, ST_TC = 64;                     // output tile rows x columns
constexpr int ST_PR = ST_TR + 2, ST_PC = ST_TC + 2;      // input patch 10 x 66
constexpr int ST_NP = ST_PR * ST_PC;                     // 660
constexpr int ST_NPL = (ST_NP + ST_THR - 1) / ST_THR;    // 3 patch elements per thread
constexpr int ST_CO = 64;                                // output channels (8 lanes x 8)
constexpr int ST_TASK = ST_TR * ST_TC * (ST_CO / 8) / ST_THR;  // 16 (voxel, chunk) tasks per thread

typedef float st_f2 __attribute__((ext_vector_type(2)));
typedef uint32_t st_u32x4 __attribute__((ext_vector_type(4)));
#ifndef ST_NT
#define ST_NT 1  // non-temporal output stores (tail data gradient 681 -> 591 us); 0 for A/B
#endif
typedef float f32x4_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ f32x4_t st_mfma(bf16x8 a, bf16x8 b, f32x4_t c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x4_t st_mfma(f16x8 a, f16x8 b, f32x4_t c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}

struct StArgs {
  const char* x;  // element (n, d, h, w, 0) at x + 2 * (n*xsn + d*xsd + h*xsh + w*xsw)
  char* y;
  const char* w;  // packed [tap][cout_pad][cin_pad] of the input's 16-bit type
  const float* bias;
  int64_t xsn, xsd, xsh, xsw, ysn, ysd, ysh, ysw;
  int D, H, W, cout_pad, cin_pad;
  int tiles_h, tiles_w, ntiles, tiles_per_blk;
  float out_scale;
  int relu;
};

template <typename H>
__global__ __launch_bounds__(ST_THR) void stencil_in_kernel(StArgs a) {
  __shared__ float patch[2][ST_NP + 4];
  const int tid = threadIdx.x;
  const int c8 = tid & 7;  // this lane's 8-channel chunk of the 64 outputs
  const H* xw = reinterpret_cast<const H*>(a.x);
  const H* wp = reinterpret_cast<const H*>(a.w);
  // channel pairs as 2-vectors: the sums run as packed v_pk_fma_f32 (36 per voxel)
  st_f2 wt[9][4], bs[4];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int e = 0; e < 4; ++e)
      wt[t][e] = st_f2{to_f32<H>(wp[((int64_t)t * a.cout_pad + 8 * c8 + 2 * e) * a.cin_pad]),
                       to_f32<H>(wp[((int64_t)t * a.cout_pad + 8 * c8 + 2 * e + 1) * a.cin_pad])};
#pragma unroll
  for (int e = 0; e < 4; ++e)
    bs[e] = a.bias ? st_f2{a.bias[8 * c8 + 2 * e], a.bias[8 * c8 + 2 * e + 1]} : st_f2{0.f, 0.f};

  struct Tile {
    int64_t xo, yo;  // element offsets of the image
    int h0, w0;
  };
  auto tile = [&](int t) __attribute__((always_inline)) {
    Tile tl;
    const int tw = t % a.tiles_w;
    t /= a.tiles_w;
    const int th = t % a.tiles_h;
    const int img = t / a.tiles_h;
    const int nb = img / a.D, dd = img - nb * a.D;
    tl.xo = nb * a.xsn + dd * a.xsd;
    tl.yo = nb * a.ysn + dd * a.ysd;
    tl.h0 = th * ST_TR;
    tl.w0 = tw * ST_TC;
    return tl;
  };
  // patch element i = tid + 256 j: input (h0 - 1 + i / 66, w0 - 1 + i % 66), zero outside
  float pv[ST_NPL];
  auto fetch = [&](const Tile& tl) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < ST_NPL; ++j) {
      const int i = tid + ST_THR * j;
      const int pr = i / ST_PC, pc = i - (i / ST_PC) * ST_PC;
      const int hh = tl.h0 - 1 + pr, ww = tl.w0 - 1 + pc;
      const bool ok = i < ST_NP && hh >= 0 && hh < a.H && ww >= 0 && ww < a.W;
      pv[j] = ok ? to_f32<H>(xw[tl.xo + hh * a.xsh + ww * a.xsw]) : 0.f;
    }
  };

  const int L = xcd_remap(blockIdx.x, gridDim.x);
  const int t0 = L * a.tiles_per_blk, t1 = min(a.ntiles, t0 + a.tiles_per_blk);
  if (t0 >= t1) return;
  Tile cur = tile(t0);
  fetch(cur);
  for (int t = t0, buf = 0; t < t1; ++t, buf ^= 1) {
    float* P = patch[buf];
#pragma unroll
    for (int j = 0; j < ST_NPL; ++j) {
      const int i = tid + ST_THR * j;
      if (i < ST_NP) P[i] = pv[j];
    }
    __syncthreads();  // the patch is complete (and the other buffer free: its tile's reads came before)
    Tile nxt = cur;
    if (t + 1 < t1) {
      nxt = tile(t + 1);
      fetch(nxt);  // in flight during this tile's stores
    }
#pragma unroll 4
    for (int k = 0; k < ST_TASK; ++k) {
      const int u = (tid >> 3) + 32 * k;  // voxel of the tile: row u / 64, column u % 64
      const int r = u >> 6, c = u & 63;
      float in[9];
#pragma unroll
      for (int kh = 0; kh < 3; ++kh)
#pragma unroll
        for (int kw = 0; kw < 3; ++kw) in[kh * 3 + kw] = P[(r + kh) * ST_PC + c + kw];
      float o[8];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        st_f2 s = bs[e];
#pragma unroll
        for (int tp = 0; tp < 9; ++tp) s = __builtin_elementwise_fma(wt[tp][e], st_f2{in[tp], in[tp]}, s);
        s *= a.out_scale;
        o[2 * e] = a.relu ? fmaxf(s.x, 0.f) : s.x;
        o[2 * e + 1] = a.relu ? fmaxf(s.y, 0.f) : s.y;
      }
      if (cur.h0 + r < a.H && cur.w0 + c < a.W) {
        H* yp = reinterpret_cast<H*>(a.y) + cur.yo + (int64_t)(cur.h0 + r) * a.ysh + (int64_t)(cur.w0 + c) * a.ysw +
                8 * c8;
#if ST_NT
        __builtin_nontemporal_store(__builtin_bit_cast(st_u32x4, Chunk<H>::pack(o)), reinterpret_cast<st_u32x4*>(yp));
#else
        *reinterpret_cast<uint4*>(yp) = Chunk<H>::pack(o);
#endif
      }
    }
    cur = nxt;
  }
}

// ---------------------------------------------------------------------------
// one OUTPUT channel: EDSR's tail nn.Conv2d(64, 1, 3, padding=1) at HR
// (edsr_net.py:32), a read stream of 128 B per voxel for 4 B written.
// ---------------------------------------------------------------------------
// A workgroup walks a band of input rows of one 128-column segment.  Per input
// row e the 9 tap partial sums P[tap][v] = sum_c W[tap][c] x[e][v][c] of its
// 130 voxels (columns w0-1 .. w0+128, nine 16-voxel blocks) come from
// v_mfma_f32_16x16x32 with the taps as M (9 of 16 rows used) and the channels
// as K: the B operand is 16 bytes of one voxel's channel row, loaded straight
// from HBM (the next row's loads in flight during this row's MFMAs), so every
// x row is read once.  P goes to a 4-slot LDS ring; output row e - 1 is then
// y[v] = bias + sum_{kh,kw} P[e-2+kh][3 kh + kw][v + kw - 1], one barrier per
// row.  The implicit-GEMM thin-output kernel it replaces staged 10 x 34 halo
// tiles (x read 1.33x through L2) at 2.6 TB/s.
constexpr int SO_SEG = 128;                 // output columns per segment
constexpr int SO_NB = 9;                    // 16-voxel blocks of P per row (144 >= 130 voxels)
constexpr int SO_PV = SO_NB * 16;           // P voxels per row
constexpr int SO_NS = 4;                    // P ring slots
constexpr int SO_MAXKS = 8;                 // channel k-steps of 32 (cin <= 256)

struct SoArgs {
  const char* x;  // element (n, d, h, w, c) at x + 2 * (n*xsn + d*xsd + h*xsh + w*xsw + c)
  char* y;        // one channel, fp32 or the input's 16-bit type
  const char* w;  // packed [tap][cout_pad][cin_pad]
  const float* bias;
  int64_t xsn, xsd, xsh, xsw, ysn, ysd, ysh, ysw;
  int D, H, W, cin, cout_pad, cin_pad;
  int bands, band_h, nseg, nsplit;
  float out_scale;
  int y16;
};

template <typename H, int KS>
__global__ __launch_bounds__(256) void stencil_out_kernel(SoArgs a) {
  using V8 = typename V8<H>::type;
  __shared__ float P[SO_NS][9][SO_PV];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int L = xcd_remap(blockIdx.x, gridDim.x);
  const int seg = L % a.nseg;
  const int t0 = L / a.nseg;
  const int band = t0 % a.bands, img = t0 / a.bands;
  const int nb = img / a.D, dd = img - nb * a.D;
  const int h0 = band * a.band_h;
  const int nst = min(a.H, h0 + a.band_h) - h0;
  const int w0 = seg * SO_SEG;
  const H* xim = reinterpret_cast<const H*>(a.x) + nb * a.xsn + dd * a.xsd;
  const int n16 = lane & 15, kg = lane >> 4;

  // A: taps as rows (m = lane & 15 < 9), 8 channels 32 ks + 8 kg.. of each k-step
  uint4 af[KS];
  const H* wp = reinterpret_cast<const H*>(a.w);
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    af[ks] = make_uint4(0, 0, 0, 0);
    if (n16 < 9) af[ks] = *reinterpret_cast<const uint4*>(wp + (int64_t)n16 * a.cout_pad * a.cin_pad + 32 * ks + 8 * kg);
  }
  // this wave's blocks b = wave + 4 j (j < 3, b < 9): lane voxel v = 16 b + n16 -> column w0 - 1 + v
  constexpr int NJ = 3;
  int64_t coff[NJ];
  bool cok[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int b = wave + 4 * j;
    const int col = w0 - 1 + 16 * b + n16;
    cok[j] = b < SO_NB && col >= 0 && col < a.W;
    coff[j] = (int64_t)(cok[j] ? col : 0) * a.xsw + 8 * kg;
  }
  auto load_row = [&](int e, uint4 (&r)[NJ][KS]) __attribute__((always_inline)) {
    const int hr = h0 - 1 + e;
    const bool rok = hr >= 0 && hr < a.H;
    const H* row = xim + (int64_t)(rok ? hr : 0) * a.xsh;
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int ks = 0; ks < KS; ++ks)
        r[j][ks] = (rok && cok[j]) ? *reinterpret_cast<const uint4*>(row + coff[j] + 32 * ks) : make_uint4(0, 0, 0, 0);
  };

  const float bias = a.bias ? a.bias[0] : 0.f;
  const int last = nst + 1;  // input rows e = 0 .. nst + 1 (image rows h0 - 1 .. h0 + nst)
  uint4 xr[NJ][KS], xn[NJ][KS];
  load_row(0, xr);
  for (int e = 0; e <= last; ++e) {
    if (e + 1 <= last) load_row(e + 1, xn);
    float* ps = &P[e % SO_NS][0][0];
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int b = wave + 4 * j;
      if (b < SO_NB) {  // wave-uniform
        f32x4_t c = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < KS; ++ks)
          c = st_mfma(__builtin_bit_cast(V8, af[ks]), __builtin_bit_cast(V8, xr[j][ks]), c);
        // lane holds P[tap 4 kg + i][voxel 16 b + n16]
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int m = 4 * kg + i;
          if (m < 9) ps[m * SO_PV + 16 * b + n16] = c[i];
        }
      }
    }
    __syncthreads();
    if (e >= 2 && tid < SO_SEG) {  // output row h0 + e - 2 from input rows e - 2 .. e
      const int col = w0 + tid;
      if (col < a.W) {
        float sum = bias;
#pragma unroll
        for (int kh = 0; kh < 3; ++kh) {
          const float* pr = &P[(e - 2 + kh) % SO_NS][3 * kh][0];
#pragma unroll
          for (int kw = 0; kw < 3; ++kw) sum += pr[kw * SO_PV + tid + kw];
        }
        sum *= a.out_scale;
        const int64_t yo = nb * a.ysn + dd * a.ysd + (int64_t)(h0 + e - 2) * a.ysh + (int64_t)col * a.ysw;
        if (a.y16) reinterpret_cast<H*>(a.y)[yo] = from_f32<H>(sum);
        else reinterpret_cast<float*>(a.y)[yo] = sum;
      }
    }
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) xr[j][ks] = xn[j][ks];
  }
}

int g_stencil_mode = -1;  // -1: VSRK_CONV_STENCIL (unset: on), 0 off, 1 on

int st_num_cus() {
  static int n = 0;
  if (n == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
  }
  return n;
}

}  // namespace

void vsrk_conv_set_stencil_mode(int mode) { g_stencil_mode = mode; }

// 1 = launched, 0 = not eligible (the thin / implicit-GEMM kernels run), < 0 = -(error status).
int vsrk_conv_fwd_stencil(const vsrk_conv_desc* d, const vsrk_tensor5* x, const void* w_packed, const float* bias,
                          const vsrk_tensor5* residual, const vsrk_tensor5* mask, const vsrk_tensor5* y,
                          hipStream_t s) {
  if (g_stencil_mode < 0) {
    const char* e = getenv("VSRK_CONV_STENCIL");
    g_stencil_mode = (e && e[0] == '0') ? 0 : 1;
  }
  if (g_stencil_mode == 0) return 0;
  if (!vsrk_is16(x->dtype) || y->dtype != x->dtype) return 0;
  if (d->kd != 1 || d->kh != 3 || d->kw != 3 || d->pd != 0 || d->ph != 1 || d->pw != 1) return 0;
  if (d->prologue != VSRK_PRO_NONE || (d->act != VSRK_ACT_NONE && d->act != VSRK_ACT_RELU)) return 0;
  if (residual || mask || d->accumulate || d->subpixel || d->bias_perm_r > 1) return 0;
  if (x->c != 1 || y->c != ST_CO || x->shuffle > 1 || y->shuffle > 1) return 0;
  if (x->n != y->n || x->d != y->d || x->h != y->h || x->w != y->w) return 0;
  if (!chunk_ok(y, 2)) return 0;
  const int tiles_h = ceil_div(y->h, ST_TR), tiles_w = ceil_div(y->w, ST_TC);
  const int64_t ntiles = (int64_t)y->n * y->d * tiles_h * tiles_w;
  if (ntiles >= (1ll << 31)) return 0;
  if (ntiles == 0) return 1;
  StArgs a;
  a.x = (const char*)x->ptr;
  a.y = (char*)y->ptr;
  a.w = (const char*)w_packed;
  a.bias = bias;
  a.xsn = x->sn; a.xsd = x->sd; a.xsh = x->sh; a.xsw = x->sw;
  a.ysn = y->sn; a.ysd = y->sd; a.ysh = y->sh; a.ysw = y->sw;
  a.D = y->d;
  a.H = y->h;
  a.W = y->w;
  a.cout_pad = round_up(y->c, 128);
  a.cin_pad = round_up(x->c, 32);
  a.tiles_h = tiles_h;
  a.tiles_w = tiles_w;
  a.ntiles = (int)ntiles;
  a.out_scale = d->out_scale;
  a.relu = d->act == VSRK_ACT_RELU;
  static int per_cu = -1;  // workgroups per CU (VSRK_STENCIL_WG A/B: 2 / 4 / 8 / 16 -> 625 / 607 / 587 / 572 us)
  if (per_cu < 0) {
    const char* e = getenv("VSRK_STENCIL_WG");
    per_cu = e ? std::max(1, atoi(e)) : 16;
  }
  const int want = (int)vsrk_capped_grid((int64_t)st_num_cus() * per_cu);
  a.tiles_per_blk = (int)ceil_div64(ntiles, want);
  // small launches (DRF's 1 -> 64 data gradient at 4 x 512^2: 2048 tiles) at
  // one tile per workgroup spend it on the per-workgroup setup (each lane's
  // 72 weights, the first patch): at least 4 tiles while the grid still
  // covers every CU
  if (vsrk_g_grid_cap <= 0)
    a.tiles_per_blk = std::max(a.tiles_per_blk, (int)std::min<int64_t>(4, std::max<int64_t>(1, ntiles / st_num_cus())));
  const int grid = (int)ceil_div64(ntiles, a.tiles_per_blk);
  vsrk_dispatch16(x->dtype, [&](auto tag) {
    using H = decltype(tag);
    stencil_in_kernel<H><<<grid, ST_THR, 0, s>>>(a);
    return 0;
  });
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    vsrk_set_error("conv_fwd(stencil): launch failed: %s", hipGetErrorString(e));
    return -VSRK_ERR_LAUNCH;
  }
  return 1;
}

// The one-output-channel form (stencil_out_kernel): 1 = launched, 0 = not eligible.
int vsrk_conv_fwd_stencil_out(const vsrk_conv_desc* d, const vsrk_tensor5* x, const void* w_packed,
                              const float* bias, const vsrk_tensor5* residual, const vsrk_tensor5* mask,
                              const vsrk_tensor5* y, hipStream_t s) {
  if (g_stencil_mode < 0) {
    const char* e = getenv("VSRK_CONV_STENCIL");
    g_stencil_mode = (e && e[0] == '0') ? 0 : 1;
  }
  if (g_stencil_mode == 0) return 0;
  if (!vsrk_is16(x->dtype) || (y->dtype != x->dtype && y->dtype != VSRK_F32)) return 0;
  if (d->kd != 1 || d->kh != 3 || d->kw != 3 || d->pd != 0 || d->ph != 1 || d->pw != 1) return 0;
  if (d->prologue != VSRK_PRO_NONE || d->act != VSRK_ACT_NONE) return 0;
  if (residual || mask || d->accumulate || d->subpixel || d->bias_perm_r > 1) return 0;
  if (y->c != 1 || x->c % 32 || x->shuffle > 1 || y->shuffle > 1) return 0;
  if (x->c != 32 && x->c != 64 && x->c != 96 && x->c != 128 && x->c != 32 * SO_MAXKS) return 0;  // instantiated k-steps
  if (x->n != y->n || x->d != y->d || x->h != y->h || x->w != y->w || !chunk_ok(x, 2)) return 0;
  const int64_t images = (int64_t)y->n * y->d;
  const int nseg = ceil_div(y->w, SO_SEG);
  if (images * nseg == 0 || y->h == 0) return 1;
  // about 4 workgroups per CU; bands of >= 16 rows
  const int64_t want = vsrk_capped_grid((int64_t)st_num_cus() * 4);
  int bands = (int)std::max<int64_t>(1, std::min<int64_t>(want / (images * nseg), ceil_div(y->h, 16)));
  SoArgs a;
  a.band_h = ceil_div(y->h, bands);
  a.bands = ceil_div(y->h, a.band_h);
  a.nseg = nseg;
  const int64_t grid = images * a.bands * nseg;
  if (grid >= (1ll << 31)) return 0;
  a.nsplit = (int)grid;
  a.x = (const char*)x->ptr;
  a.y = (char*)y->ptr;
  a.w = (const char*)w_packed;
  a.bias = bias;
  a.xsn = x->sn; a.xsd = x->sd; a.xsh = x->sh; a.xsw = x->sw;
  a.ysn = y->sn; a.ysd = y->sd; a.ysh = y->sh; a.ysw = y->sw;
  a.D = y->d;
  a.H = y->h;
  a.W = y->w;
  a.cin = x->c;
  a.cout_pad = round_up(y->c, 128);
  a.cin_pad = round_up(x->c, 32);
  a.out_scale = d->out_scale;
  a.y16 = y->dtype != VSRK_F32;
  const int ks = x->c / 32;
  vsrk_dispatch16(x->dtype, [&](auto tag) {
    using H = decltype(tag);
    switch (ks) {
      case 1: stencil_out_kernel<H, 1><<<(int)grid, 256, 0, s>>>(a); break;
      case 2: stencil_out_kernel<H, 2><<<(int)grid, 256, 0, s>>>(a); break;
      case 3: stencil_out_kernel<H, 3><<<(int)grid, 256, 0, s>>>(a); break;
      case 4: stencil_out_kernel<H, 4><<<(int)grid, 256, 0, s>>>(a); break;
      default: stencil_out_kernel<H, 8><<<(int)grid, 256, 0, s>>>(a); break;
    }
    return 0;
  });
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    vsrk_set_error("conv_fwd(stencil out): launch failed: %s", hipGetErrorString(e));
    return -VSRK_ERR_LAUNCH;
  }
  return 1;
}
