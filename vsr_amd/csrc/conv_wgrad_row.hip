// Rolling-row weight/bias gradient of a 16-bit Conv2d 3x3, padding 1: the
// autograd of EDSR's body convs nn.Conv2d(64, 64, 3, padding=1).weight /
// .bias in loss.backward() (edsr_net.py:41-53; base_trainer.py:128).
//
// dW[co][ci][kh][kw] = sum over (image, h, w) of dy[h][w][co] x[h+kh-1][w+kw-1][ci]
// is a GEMM with K = voxels: 64 x 64 x 9 outputs over 2^20 voxels per EDSR
// layer, ~290 flop per byte of x and dy -- on the MI355X ridge, so the kernel
// must stream x and dy once at HBM rate AND keep the matrix cores busy.
// conv_wgrad_pipe staged 8 x 32 tiles with their halo (x read 1.33x) through
// registers and ran at 0.28 of the bf16 peak on EDSR's layers.  Here:
//  * A workgroup owns 64 output x 64 input channels and all 9 taps of a
//    128-column segment, and walks a band of image rows top to bottom (one
//    stage per output row): the three x rows an output row meets sit in a
//    four-slot LDS ring, so every x row is fetched once per band (halo: 2 rows
//    per band) and never re-staged.
//  * Register staging, one stage ahead: during stage s each wave's buffer
//    loads (16 B per lane, coalesced 1 KB pieces; out-of-image rows, the pad
//    columns and columns past W read as zero through the buffer range) bring
//    x row s + 3 and dy row s + 1; at the end of the stage they are written
//    to LDS with the swizzle on the LDS side, then one barrier.  LDS-DMA
//    pieces cost 60-185 cycles of issue each (MI355X_MICROARCH.md, "LDS-DMA
//    piece issue cost"): with 40 per stage they kept the MFMA pipes idle at
//    every stage (96 us per EDSR layer, 83 us with the DMA removed).
//  * 8 waves = 2 output halves (32 channels) x 4 input quarters (16), two per
//    SIMD; a wave holds 9 taps x 2 blocks of 16 x 16 in 72 accumulators and
//    runs v_mfma_f32_16x16x32 on ds_read_b64_tr_b16 operands: per 32-voxel
//    k-chunk 2 dy fragments and 9 x fragments (one per tap) for 18 MFMAs, the
//    next group's reads issued before the current group's MFMAs.
//  * LDS images are voxel-major rows of 64 channels (128 B); 16-byte chunk c
//    of voxel j sits at chunk c ^ (2 bit1(j) + 4 bit3(j)).  Every transposed
//    read is conflict-free whatever its voxel offset (the kw taps shift it by
//    0..2), and so is every 16-byte store (8 lanes fill one voxel's 128 B).
//  * Deterministic: one fp32 slab per (band, channel chunk) in
//    wgrad_reduce_kernel's layout ([9 taps][64 co][64 ci] + dbias), summed
//    over bands in a fixed order.  dbias: MFMAs of the dy fragments against
//    ones, wave (half, quarter q) on k-chunk q (two per wave and stage), the
//    four k-chunks' partials added through LDS at the end.
#include <algorithm>
#include <cstdlib>
#include "conv_common.h"

namespace {
using namespace vsrk_conv;

constexpr int RW_NW = 8;                               // waves
constexpr int RW_KC = 4;                               // k-chunks of 32 columns per segment
constexpr int RW_SEG = 32 * RW_KC;                     // 128 output columns per segment
constexpr int RW_XV = RW_SEG + 8;                      // x row slot: columns -1 .. 128 (+6 unused)
constexpr int RW_XP = RW_XV / 8;                       // 17 pieces of 1 KB (8 voxels x 64 channels)
constexpr int RW_YP = RW_SEG / 8;                      // 16 dy pieces
constexpr int RW_NP = RW_XP + RW_YP;                   // 33
constexpr int RW_NQ = (RW_NP + RW_NW - 1) / RW_NW;     // 5 piece roles (wave 0 has 5 pieces, the others 4)
constexpr int RW_XSLOT = RW_XP * 1024;                 // 17,408 B
constexpr int RW_YSLOT = RW_YP * 1024;                 // 16,384 B
constexpr int RW_NXS = 4, RW_NYS = 2;                  // ring slots
constexpr int RW_YBASE = RW_NXS * RW_XSLOT;
constexpr int RW_LDS = RW_YBASE + RW_NYS * RW_YSLOT;   // 102,400 B: one workgroup per CU
constexpr int RW_COW = 64;                             // output channels per workgroup
constexpr int RW_SLAB = 9 * RW_COW * 64 + RW_COW;      // floats per (band, chunk) slab
constexpr uint32_t RW_OOB = 0x80000000u;               // buffer offset past the range: reads zero

#ifndef RW_ABL
#define RW_ABL 0  // ablation builds only (wrong results): 1 no per-stage staging / barrier, 2 no MFMA
#endif

__host__ __device__ constexpr int rw_swz(int j) { return 2 * ((j >> 1) & 1) + 4 * ((j >> 3) & 1); }

typedef __amdgpu_buffer_rsrc_t RwRsrc;
__device__ __forceinline__ RwRsrc rw_rsrc(const void* base) {
  const uint64_t b = (uint64_t)base;
  const uint64_t u = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(b >> 32)) << 32) |
                     (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)b);
  return __builtin_amdgcn_make_buffer_rsrc((void*)u, 0, 0x7FFFFFF0, 0x00020000);
}
typedef uint32_t rw_u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void rw_st16(uint32_t addr, uint4 v) {
  *(__attribute__((address_space(3))) rw_u32x4*)(size_t)addr = __builtin_bit_cast(rw_u32x4, v);
}

typedef float f32x4_t __attribute__((ext_vector_type(4)));
template <typename H> struct V8R;
template <> struct V8R<bf16> { typedef bf16x8 type; };
template <> struct V8R<f16> { typedef f16x8 type; };
__device__ __forceinline__ f32x4_t rw_mfma(bf16x8 a, bf16x8 b, f32x4_t c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x4_t rw_mfma(f16x8 a, f16x8 b, f32x4_t c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}
// 8 consecutive voxels (k) of one channel: two transposed 4-row reads (LDS
// byte addresses: no generic-pointer arithmetic or null checks)
__device__ __forceinline__ uint4 rw_frag(uint32_t p0, uint32_t p1) {
  const v4i16 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)(size_t)p0);
  const v4i16 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)(size_t)p1);
  return __builtin_bit_cast(uint4, __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7));
}

constexpr int RW_MAXB = 16;  // 64-channel blocks of a sub-pixel view (1024 logical channels)

struct RowArgs {
  const char* x;   // element (n, d, h, w, c) at x + 2 * (n*xsn + d*xsd + h*xsh + w*xsw + c)
  const char* dy;
  // element offset of 64-channel block b inside its operand: b * 64 for a
  // plain view; for a sub-pixel view (shuffle r: logical channel
  // (i r + j) C' + c' of LR voxel (h, w) at physical (r h + i, r w + j, c'))
  // the block's phase row / column and c' base (its h / w strides above are
  // then r physical rows / columns) -- EDSR's up-sampler and DRF's sub-pixel
  // projections (edsr_net.py:59-62, drf_net.py:81-100)
  int xoff[RW_MAXB], yoff[RW_MAXB];
  // sub-pixel forms (SPM): per block of the shuffled operand, the taps its
  // phase meets (bit kh * 3 + kw); the others are structurally zero in the
  // equivalent weight (drf_net.py:70-102 at k = 2s: 4 of 9) -- their MFMAs
  // are skipped and their slab entries written as zeros
  uint16_t tapm[RW_MAXB];
  int tapm_x;  // the mask belongs to the input block (x shuffled) or the output block
  float* ws;
  int64_t xsn, xsd, xsh, xsw, ysn, ysd, ysh, ysw;
  int xd, H, W;
  int bands, band_h, nseg, ncot, ncic, nsplit;
  int want_bias;
  int prio;  // A/B knob (VSRK_WGRAD_ROW_PRIO=1): s_setprio 1 around each group's MFMAs
};

template <typename H, bool SPM>
__global__ __launch_bounds__(RW_NW * 64, 1) void wgrad_row_kernel(RowArgs a) {
  using V8 = typename V8R<H>::type;
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int coh = wave & 1, cib = wave >> 1;  // output half (32), input quarter (16)

  // ---- which (band, channel chunk) this workgroup is ----
  const int ncombo = a.ncot * a.ncic;
  const int L = xcd_remap(blockIdx.x, a.nsplit * ncombo);
  const int split = L / ncombo;
  const int combo = L - split * ncombo;
  const int cot = combo % a.ncot, cic = combo / a.ncot;
  const int seg = split % a.nseg;
  const int t0 = split / a.nseg;
  const int band = t0 % a.bands, img = t0 / a.bands;
  const int nb = img / a.xd, dd = img - nb * a.xd;
  const int h0 = band * a.band_h;
  const int nst = min(a.H, h0 + a.band_h) - h0;  // output rows (stages)
  const int w0 = seg * RW_SEG;
  const unsigned tapm = SPM ? (unsigned)a.tapm[a.tapm_x ? cic : cot] : 0x1ffu;  // workgroup-uniform
  const char* xim = a.x + 2 * (nb * a.xsn + dd * a.xsd + a.xoff[cic]);
  const char* yim = a.dy + 2 * (nb * a.ysn + dd * a.ysd + a.yoff[cot]);

  // ---- per-lane piece roles (1 KB = 8 voxels x 64 channels), the same kind
  // for every wave at each q: q = 0, 1: x piece wave + 8q; q = 2, 3: dy piece
  // wave + 8(q - 2); q = 4: x piece 16 (wave 0 only).  x piece j: slot voxel
  // v = 8j + l/8 (column w0 - 1 + v); dy piece j: voxel v = 8j + l/8 (column
  // w0 + v); lane l loads chunk l & 7 (linear, coalesced) and stores it at
  // chunk (l & 7) ^ rw_swz(v) of the LDS voxel row.
  static_assert(RW_XP == 2 * RW_NW + 1 && RW_YP == 2 * RW_NW, "piece roles");
  uint32_t goff[RW_NQ], loff[RW_NQ];
#pragma unroll
  for (int q = 0; q < RW_NQ; ++q) {
    const bool isx = q != 2 && q != 3;
    const int j = q == 4 ? 2 * RW_NW : wave + RW_NW * (q & 1);
    if (isx) {
      const int v = 8 * j + (lane >> 3);
      const int col = w0 - 1 + v;
      const bool ok = v < RW_SEG + 2 && col >= 0 && col < a.W;
      goff[q] = ok ? (uint32_t)(2 * (col * (int)a.xsw + 8 * (lane & 7))) : RW_OOB;
      loff[q] = (uint32_t)(j * 1024 + (lane >> 3) * 128 + 16 * ((lane & 7) ^ rw_swz(v)));
    } else {
      const int v = 8 * j + (lane >> 3);
      const int col = w0 + v;
      goff[q] = col < a.W ? (uint32_t)(2 * (col * (int)a.ysw + 8 * (lane & 7))) : RW_OOB;
      loff[q] = (uint32_t)(j * 1024 + (lane >> 3) * 128 + 16 * ((lane & 7) ^ rw_swz(v)));
    }
  }
  const uint32_t lbase = lds_addr(lds);
  // piece set t: x row t (image row h0 - 1 + t) for x slot t % 4 and dy row
  // t - 2 (output row h0 + t - 2) for dy slot (t - 2) % 2
  auto load_set = [&](int t, uint4 (&r)[RW_NQ]) __attribute__((always_inline)) {
    const int xr = h0 - 1 + t;
    const bool xok = xr >= 0 && xr < a.H;
    const int yr = t - 2;
    const bool yok = yr >= 0 && yr < nst;
    const RwRsrc rx = rw_rsrc(xim + 2 * (int64_t)(xok ? xr : 0) * a.xsh);
    const RwRsrc ry = rw_rsrc(yim + 2 * (int64_t)(h0 + (yok ? yr : 0)) * a.ysh);
#pragma unroll
    for (int q = 0; q < RW_NQ; ++q) {
      const bool isx = q != 2 && q != 3;
      if (q == 4 && wave != 0) break;
      r[q] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(
                                           isx ? rx : ry, (int)((isx ? xok : yok) ? goff[q] : RW_OOB), 0, 0));
    }
  };
  auto store_set = [&](int t, const uint4 (&r)[RW_NQ]) __attribute__((always_inline)) {
    const uint32_t xs = lbase + (uint32_t)(t % RW_NXS) * RW_XSLOT;
    const int yr = t - 2;
    const uint32_t ys = lbase + RW_YBASE + (uint32_t)((yr < 0 ? 0 : yr) % RW_NYS) * RW_YSLOT;
#pragma unroll
    for (int q = 0; q < RW_NQ; ++q) {
      const bool isx = q != 2 && q != 3;
      if (q == 4 && wave != 0) break;
      if (isx) rw_st16(xs + loff[q], r[q]);
      else if (yr >= 0) rw_st16(ys + loff[q], r[q]);
    }
  };

  // ---- fragment read offsets (bytes within a slot, k-chunk 0) ----
  // lane (g, q, p) of a transposed read supplies voxel 8g + q (+4 for the
  // second read) of the k-chunk, channels 4p..4p+3 of its 16-channel block.
  const int g = lane >> 4, qq = (lane >> 2) & 3, pp = lane & 3;
  uint32_t xo[3][2];  // [kw][read]: x slot voxel kw + 8g + q + 4h
#pragma unroll
  for (int kw = 0; kw < 3; ++kw)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int v = kw + 8 * g + qq + 4 * h;
      xo[kw][h] = (uint32_t)(v * 128 + 16 * ((2 * cib + (pp >> 1)) ^ rw_swz(v)) + 8 * (pp & 1));
    }
  uint32_t yo[2][2];  // [output block][read]
#pragma unroll
  for (int b = 0; b < 2; ++b)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int v = 8 * g + qq + 4 * h;
      yo[b][h] = (uint32_t)(v * 128 + 16 * ((2 * (2 * coh + b) + (pp >> 1)) ^ rw_swz(v)) + 8 * (pp & 1));
    }

  f32x4_t acc[3][3][2];  // [kh][kw][output block]: co 32 coh + 16 b + 4 (l >> 4) + i, ci 16 cib + (l & 15)
#pragma unroll
  for (int i = 0; i < 18; ++i) acc[i / 6][(i / 2) % 3][i % 2] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  // dbias: wave (coh, cib) takes both output blocks of its half on k-chunk
  // cib: every (block, k-chunk) once, two MFMAs per wave and stage
  f32x4_t bacc[2] = {f32x4_t{0.f, 0.f, 0.f, 0.f}, f32x4_t{0.f, 0.f, 0.f, 0.f}};
  uint4 ones;
  {
    const H one = from_f32<H>(1.f);
    const uint16_t u = __builtin_bit_cast(uint16_t, one);
    const uint32_t w2 = (uint32_t)u | ((uint32_t)u << 16);
    ones = make_uint4(w2, w2, w2, w2);
  }

  // ---- prologue: piece sets 0..2 into LDS, set 3 in registers ----
  const int last = nst + 1;  // the last piece set (x row h0 + nst)
  uint4 stg[RW_NQ], stg2[RW_NQ];
  load_set(0, stg);
  if (1 <= last) load_set(1, stg2);
  store_set(0, stg);
  if (1 <= last) store_set(1, stg2);
  if (2 <= last) {
    load_set(2, stg);
    store_set(2, stg);
  }
  __syncthreads();
  if (3 <= last) load_set(3, stg);
  __builtin_amdgcn_sched_barrier(0);

  // ---- main loop: stage s = output row h0 + s reads sets <= s + 2 ----
  for (int s = 0; s < nst; ++s) {
    // this stage's fragment addresses (k-chunk 0; the k-chunk is the reads'
    // immediate offset), pinned in VGPRs: 22 adds per stage
    uint32_t xa[3][3][2], ya[2][2];
#pragma unroll
    for (int kh = 0; kh < 3; ++kh) {
      const uint32_t xrow = lbase + (uint32_t)((s + kh) % RW_NXS) * RW_XSLOT;
#pragma unroll
      for (int kw = 0; kw < 3; ++kw)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          xa[kh][kw][h] = xrow + xo[kw][h];
          asm volatile("" : "+v"(xa[kh][kw][h]));
        }
    }
    {
      const uint32_t yr = lbase + RW_YBASE + (uint32_t)(s % RW_NYS) * RW_YSLOT;
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          ya[b][h] = yr + yo[b][h];
          asm volatile("" : "+v"(ya[b][h]));
        }
    }
    // 12 groups G = (k-chunk G / 3, kh G % 3): 3 x fragments (+ the k-chunk's
    // 2 dy fragments at kh 0) and 6 MFMAs; group G + 1's reads are issued
    // before group G's MFMAs (a register double buffer; two groups ahead
    // measured no faster), the scheduler kept from sinking them to their use.
    uint4 xf[2][3], yf[2][2];
    auto load_group = [&](int G) __attribute__((always_inline)) {
      const int kc = G / 3, kh = G % 3;
      if (kh == 0) {
#pragma unroll
        for (int b = 0; b < 2; ++b) yf[kc & 1][b] = rw_frag(ya[b][0] + kc * 4096, ya[b][1] + kc * 4096);
      }
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) xf[G & 1][kw] = rw_frag(xa[kh][kw][0] + kc * 4096, xa[kh][kw][1] + kc * 4096);
    };
    load_group(0);
#pragma unroll
    for (int G = 0; G < 3 * RW_KC; ++G) {
      if (G + 1 < 3 * RW_KC) load_group(G + 1);
      __builtin_amdgcn_sched_barrier(0);
      if (a.prio) __builtin_amdgcn_s_setprio(1);
      const int kc = G / 3, kh = G % 3;
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {
        if (SPM && !((tapm >> (kh * 3 + kw)) & 1)) continue;  // workgroup-uniform
#pragma unroll
        for (int b = 0; b < 2; ++b)
          if (RW_ABL & 2) acc[kh][kw][b][0] += __builtin_bit_cast(float, yf[kc & 1][b].x ^ xf[G & 1][kw].y);
          else acc[kh][kw][b] = rw_mfma(__builtin_bit_cast(V8, yf[kc & 1][b]), __builtin_bit_cast(V8, xf[G & 1][kw]),
                                   acc[kh][kw][b]);
      }
      if (kh == 1 && kc == cib) {  // wave-uniform
#pragma unroll
        for (int b = 0; b < 2; ++b)
          bacc[b] = rw_mfma(__builtin_bit_cast(V8, yf[kc & 1][b]), __builtin_bit_cast(V8, ones), bacc[b]);
      }
      if (a.prio) __builtin_amdgcn_s_setprio(0);
      __builtin_amdgcn_sched_barrier(0);
    }
    // set s + 3 (loaded during this stage) into its slots -- x row s - 1's and
    // dy row s - 1's, which every wave left at the previous barrier -- then
    // publish it and start the loads of set s + 4
    if (!(RW_ABL & 1)) {
      if (s + 3 <= last) store_set(s + 3, stg);
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      if (s + 4 <= last) load_set(s + 4, stg);
    }
    __builtin_amdgcn_sched_barrier(0);
  }

  // ---- slab of (split, combo): [tap][co 64][ci 64] + dbias[64] ----
  float* out = a.ws + ((int64_t)split * ncombo + combo) * RW_SLAB;
  const int l15 = lane & 15, lg = lane >> 4;
#pragma unroll
  for (int t9 = 0; t9 < 9; ++t9)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int co = 32 * coh + 16 * b + 4 * lg + i, ci = 16 * cib + l15;
        out[(t9 * RW_COW + co) * 64 + ci] = ((tapm >> t9) & 1) ? acc[t9 / 3][t9 % 3][b][i] : 0.f;
      }
  if (a.want_bias && cic == 0) {  // workgroup-uniform
    // bacc[b][i] = dbias partial (k-chunk cib) of channel 32 coh + 16 b + 4 lg + i
    float* part = reinterpret_cast<float*>(lds);  // [k-chunk][64]; the ring is idle now
    __syncthreads();
    if (l15 == 0) {
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int i = 0; i < 4; ++i) part[cib * 64 + 32 * coh + 16 * b + 4 * lg + i] = bacc[b][i];
    }
    __syncthreads();
    if (threadIdx.x < RW_COW) {
      const int c = threadIdx.x;
      out[9 * RW_COW * 64 + c] = ((part[c] + part[64 + c]) + part[128 + c]) + part[192 + c];
    }
  }
}

int g_wrow_mode = -1;  // -1: VSRK_WGRAD_ROW (unset: on), 0 off, 1 on, 2 on with the sub-pixel tap skip forms

int wrow_num_cus() {
  static int n = 0;
  if (n == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
  }
  return n;
}

}  // namespace

void vsrk_conv_set_wgrad_row_mode(int mode) { g_wrow_mode = mode; }

bool vsrk_wgrad_row_plan(const vsrk_conv_desc* d, const vsrk_tensor5* x, const vsrk_tensor5* dy, VsrkRowPlan* p) {
  if (g_wrow_mode < 0) {
    const char* e = getenv("VSRK_WGRAD_ROW");
    g_wrow_mode = (e && e[0] == '0') ? 0 : 1;
  }
  if (g_wrow_mode == 0) return false;
  if (!vsrk_is16(x->dtype) || dy->dtype != x->dtype) return false;
  if (d->kd != 1 || d->kh != 3 || d->kw != 3 || d->pd != 0 || d->ph != 1 || d->pw != 1) return false;
  // (sub-pixel views: one operand is a shuffle-r view of a high-res buffer;
  // with d->subpixel set, the taps a phase never meets are skipped, see tapm)
  if (d->prologue != VSRK_PRO_NONE) return false;
  if (x->c % 64 || dy->c % 64 || (x->shuffle > 1 && dy->shuffle > 1)) return false;
  // Views with the sub-pixel tap skip (DRF's projections) stay on the
  // pipelined kernel unless forced (mode 2): with 4 of 9 taps per phase the
  // row pipeline is load-bound and its 9-tap slabs double the reduce -- cfg3
  // A/B, same box: projection weight gradients 25.3 ms/step here vs 22.0 on the
  // pipelined kernel (profiles/r5_wgrad_row_subpixel_ab.txt).  Plain
  // shuffled views (EDSR's up-sampler, all taps live) run here.
  if (d->subpixel && (x->shuffle > 1 || dy->shuffle > 1) && g_wrow_mode != 2) return false;
  if (x->c / 64 > RW_MAXB || dy->c / 64 > RW_MAXB) return false;
  for (const vsrk_tensor5* t : {x, dy}) {  // a sub-pixel view: every 64-channel block inside one phase
    if (t->shuffle <= 1) continue;
    const int r = t->shuffle, cph = t->c / (r * r);
    if (cph * r * r != t->c || cph % 64) return false;
  }
  if (x->n != dy->n || x->d != dy->d || x->h != dy->h || x->w != dy->w) return false;
  if (!chunk_ok(x, 2) || !chunk_ok(dy, 2)) return false;
  for (const vsrk_tensor5* t : {x, dy}) {
    const int64_t r = t->shuffle > 1 ? t->shuffle : 1;
    if (t->sn < 0 || t->sd < 0 || t->sh < 0 || t->sw < 0 ||
        (int64_t)(RW_XV + 2) * r * t->sw + (r - 1) * t->sh + t->c >= (1ll << 29))
      return false;
  }
  const int64_t images = (int64_t)x->n * x->d;
  if (images <= 0 || x->h <= 0 || x->w <= 0) return false;
  const int nseg = ceil_div(x->w, RW_SEG);
  const int ncot = dy->c / RW_COW, ncic = x->c / 64;
  const int64_t per_band = images * nseg * ncot * ncic;  // workgroups per band of every image
  // about one workgroup per CU (the ring takes 100 KB): bands of >= 8 rows
  int64_t want = std::max<int64_t>(1, wrow_num_cus());
  if (vsrk_g_grid_cap > 0) want = std::min<int64_t>(want, vsrk_g_grid_cap);
  int bands = (int)std::max<int64_t>(1, std::min<int64_t>((want + per_band / 2) / per_band, ceil_div(x->h, 8)));
  {
    static int ov = -1;  // A/B knob: VSRK_WGRAD_ROW_BANDS=<bands per image column>
    if (ov < 0) {
      const char* e = getenv("VSRK_WGRAD_ROW_BANDS");
      ov = e ? std::max(0, atoi(e)) : 0;
    }
    if (ov > 0) bands = std::min(ov, x->h);
  }
  if (vsrk_g_grid_cap > 0) bands = std::max(1, std::min(bands, x->h));
  p->band_h = ceil_div(x->h, bands);
  p->bands = ceil_div(x->h, p->band_h);
  p->nseg = nseg;
  p->ncot = ncot;
  p->ncic = ncic;
  const int64_t ns = images * p->bands * nseg;
  if (ns * ncot * ncic >= (1ll << 30)) return false;
  p->nsplit = (int)ns;
  p->cot_w = RW_COW;
  p->slab = RW_SLAB;
  p->ws_bytes = (size_t)ns * ncot * ncic * RW_SLAB * sizeof(float);
  return true;
}

int vsrk_conv_wgrad_row(const vsrk_conv_desc* d, const vsrk_tensor5* x, const vsrk_tensor5* dy, int want_bias,
                        float* ws, size_t ws_bytes, VsrkRowPlan* plan, hipStream_t s) {
  VsrkRowPlan p;
  if (!vsrk_wgrad_row_plan(d, x, dy, &p)) return 0;
  if (ws_bytes < p.ws_bytes) return 0;
  RowArgs a;
  a.x = (const char*)x->ptr;
  a.dy = (const char*)dy->ptr;
  a.ws = ws;
  // logical (LR-grid) strides and per-block offsets of the two operands
  auto blocks = [](const vsrk_tensor5* t, int64_t& sh, int64_t& sw, int* off) {
    const int r = t->shuffle > 1 ? t->shuffle : 1;
    sh = (int64_t)r * t->sh;
    sw = (int64_t)r * t->sw;
    const int cph = t->c / (r * r);
    for (int b = 0; b < t->c / 64; ++b) {
      const int c = 64 * b, sub = c / cph, cc = c - sub * cph;
      off[b] = (int)((sub / r) * t->sh + (sub % r) * t->sw + cc);
    }
  };
  a.xsn = x->sn; a.xsd = x->sd;
  a.ysn = dy->sn; a.ysd = dy->sd;
  blocks(x, a.xsh, a.xsw, a.xoff);
  blocks(dy, a.ysh, a.ysw, a.yoff);
  const vsrk_tensor5* spt = x->shuffle > 1 ? x : (dy->shuffle > 1 ? dy : nullptr);
  const bool spm = d->subpixel && spt;
  a.tapm_x = spt == x;
  if (spm) {
    const int r = spt->shuffle, cph = spt->c / (r * r);
    const int32_t code = d->subpixel & ~(1 << 25);  // gradients of the forward (unflipped) taps
    for (int b = 0; b < spt->c / 64; ++b) a.tapm[b] = (uint16_t)subpixel_tapmask(code, r, 64 * b / cph);
  }
  a.xd = x->d;
  a.H = x->h;
  a.W = x->w;
  a.bands = p.bands;
  a.band_h = p.band_h;
  a.nseg = p.nseg;
  a.ncot = p.ncot;
  a.ncic = p.ncic;
  a.nsplit = p.nsplit;
  a.want_bias = want_bias;
  {
    static int prio = -1;
    if (prio < 0) {
      const char* e = getenv("VSRK_WGRAD_ROW_PRIO");
      prio = (e && e[0] == '1') ? 1 : 0;
    }
    a.prio = prio;
  }
  const int grid = p.nsplit * p.ncot * p.ncic;
  vsrk_dispatch16(x->dtype, [&](auto tag) {
    using H = decltype(tag);
    auto kern = spm ? wgrad_row_kernel<H, true> : wgrad_row_kernel<H, false>;
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, RW_LDS);
    kern<<<grid, RW_NW * 64, RW_LDS, s>>>(a);
    return 0;
  });
  *plan = p;
  return 1;
}
