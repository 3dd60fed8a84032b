// Fast path of the implicit-GEMM convolution (forward and data-gradient) for
// bf16 channels-last views on CDNA4 (gfx950).  Same contract as
// conv_fwd_kernel (conv_fwd.hip): nn.Conv2d / nn.Conv3d forward
// (edsr_net.py:28-64, duf_net.py:35-49,116-214) and, with a mode-1 packed
// weight, the data gradient of loss.backward() (base_trainer.py:128).
//
// What is different from conv_fwd_kernel, and why (PMC on the EDSR 64->64
// 3x3 conv: 14 VALU + 8 SALU instructions per MFMA, 43 % of wave time in
// waits):
//  * Both operands are staged by LDS-DMA (global_load_lds_dwordx4, issued as
//    inline asm so hipcc does not drain it before the MFMAs).  Zero padding
//    (halo outside the image, channel chunks beyond cin) is a DMA from a
//    zero page instead of a masked register path: no staging VGPRs, no
//    ds_write pass, no commit barrier.
//  * A two-slot ring with ONE barrier per stage: the DMA of stage g+1 is
//    issued right after the barrier that opens stage g and lands while
//    stage g's MFMAs run.
//  * Unpadded 64-byte LDS rows with the 16-byte pieces XOR-swizzled by the
//    row's halo column (ww >> 2) & 3 (A) or row (B): conflict-free
//    ds_read_b128 for any column shift kw (the 16-lane groups of a b128
//    read touch rows {0-3,12-15,20-27} + v0, whose keys differ within each
//    4-bank class).  Every ds_read address is a per-lane base (6 + 2
//    registers, computed once per launch) plus a compile-time immediate.
//  * Epilogue addresses: one 64-bit row base per (row, tensor), channel
//    offsets are constants; the sub-pixel (PixelShuffle) store resolves its
//    sub-pixel per 32-channel block (wave-uniform).
//
// Tile: NW waves x MS rows x 32 columns of one (n, d) slice, NT output
// channels (NT/32 MFMA column blocks).  Stage: (kd tap, 32 input channels).
// MFMA v_mfma_f32_32x32x16_bf16, operands "weights x voxels": a lane's
// accumulator column is one voxel, its registers 4 consecutive channels.
//
// This header holds the kernel template; conv_fast.hip holds the host entry
// (eligibility, argument set-up) and each conv_fast_*.hip translation unit
// instantiates one family of tile shapes, so the library builds in parallel.
#pragma once
#include "conv_common.h"

namespace vsrk_conv {

struct FastArgs {
  View x, y, res, msk;
  const void* w;  // packed weight, elements of the input's 16-bit type
  const float* bias;
  const float* pro_scale;
  const float* pro_shift;
  int cin, cout, cin_pad, cout_pad;
  int kd, pd, ph, pw;
  int prologue, act, accumulate, has_res, has_mask, bias_r;
  float out_scale;
  const float* act_param;
  const float* mask_slope;
  int tiles_h, tiles_w, ntn, ntiles;
  int ablate;  // diagnostics only (VSRK_FAST_ABLATE): 1 skip DMA after the first stage, 2 skip MFMAs, 4 skip epilogue
};

constexpr int kFastNotEligible = -1000;
// Persistent grid size for `ntiles` output tiles: one workgroup per CU, or the
// test cap set by vsrk_conv_set_grid_cap (so small shapes run many tiles per
// workgroup through the cross-tile pipeline).
int fast_grid(int64_t ntiles);

// Per-family launchers (one translation unit each).  Return VSRK_OK, an error
// status, or kFastNotEligible when the shape does not fit the family's LDS.
int fast_k1(const FastArgs& a, int nt, bool yf, bool h16, hipStream_t s);       // conv_fast_k1.hip
int fast_k3_n32(const FastArgs& a, bool yf, bool h16, hipStream_t s);           // conv_fast_k3_n32.hip
int fast_k3_n64(const FastArgs& a, bool yf, bool h16, hipStream_t s);           // conv_fast_k3_n64.hip
int fast_k3_n64_xs(const FastArgs& a, bool yf, bool h16, hipStream_t s);        // conv_fast_k3_n64_xs.hip
int fast_k3_n64_ys(const FastArgs& a, bool yf, bool h16, hipStream_t s);        // conv_fast_k3_n64_ys.hip

}  // namespace vsrk_conv

#ifdef VSRK_FAST_KERNEL_TU
namespace {
using namespace vsrk_conv;

// s_waitcnt vmcnt(N) (expcnt / lgkmcnt left at their maxima)
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}

// 16 B per lane of zeros: the DMA source of every padding chunk.
__device__ __attribute__((aligned(256))) uint4 g_zero_page[16];



template <int KK, int NT, int MS, int XS, int YS, int PRO, typename YT, int NW, typename H>
__global__ __launch_bounds__(NW * 64, NW == 4 ? 1 : 2) void conv_fast_kernel(FastArgs a) {
  constexpr int NTH = NW * 64;
  constexpr int NS = NT / 32;
  constexpr int FTH = NW * MS;
  constexpr int HWd = TW + KK - 1;
  constexpr int HROWS = (FTH + KK - 1) * HWd;
  // A DMA wave-instructions per stage (16 rows of 64 B each).  With the
  // BN/ReLU prologue the count is padded to a multiple of NW (every wave
  // owns NAW chunks of the A region, the padding ones zero), so that each
  // wave issues the same number of DMAs per stage: the late prologue below
  // waits for its own A chunks with a compile-time vmcnt.
  constexpr int NAI0 = (HROWS + 15) / 16;
  constexpr int NAW = (NAI0 + NW - 1) / NW;
  constexpr int NAI = PRO ? NAW * NW : NAI0;
  constexpr int TAPS = KK * KK;
  constexpr int NBI = TAPS * NT / 16;     // B DMA wave-instructions per stage
  constexpr int ABYTES = NAI * 1024;
  constexpr int BBYTES = NBI * 1024;
  constexpr int SLOT = ABYTES + BBYTES;
  constexpr int NBW = (NBI + NW - 1) / NW;
  static_assert(NAW <= 16 && NBW <= 16, "per-wave DMA count");
  // transposed epilogue (H output): channel block CB and where its
  // per-wave scratch lives -- in the ring slot that is idle at epilogue
  // time, or (small slots) in a region of its own after the ring.
  constexpr bool TRANS = sizeof(YT) == 2;
  constexpr int CB = (!YS && SLOT >= NW * 32 * (NT * 4 + 16)) ? NT : 32;
  constexpr bool SCR_OWN = TRANS && SLOT < NW * 32 * (CB * 4 + 16);
  extern __shared__ __attribute__((aligned(16))) char lds[];

  const int tid = threadIdx.x, lane = tid & 63, r = lane & 31, hf = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: SALU address math
  float* lbias = reinterpret_cast<float*>(lds + 2 * SLOT + (SCR_OWN ? NW * 32 * (CB * 4 + 16) : 0));  // [cout_pad], view order
  const float aslope = a.act == VSRK_ACT_PRELU ? *a.act_param : 0.f;
  const float mslope = a.mask_slope ? *a.mask_slope : 0.f;
  auto SCR_BASE = [&](int sl) __attribute__((always_inline)) { return SCR_OWN ? 2 * SLOT : sl * SLOT; };
  constexpr int NQ = NAW + NBW;  // DMA wave-instructions per stage and wave
  int slot_epi = 0;  // the ring slot free during the deferred epilogue
  float* lsc = lbias + a.cout_pad;
  float* lsh = lsc + a.cin_pad;
  if constexpr (PRO) stage_prologue(lsc, lsh, a.prologue, a.pro_scale, a.pro_shift, a.cin, a.cin_pad, tid, NTH);
  for (int i = tid; i < a.cout_pad; i += NTH) {
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
    lbias[i] = b * a.out_scale;
  }

  // ---- per-lane DMA roles, fixed for the launch ----
  // A: instruction i = wave + NW*k fills LDS rows 16i..16i+15; lane -> row
  // v = 16i + lane/4, position P = lane%4 holding logical piece
  // p = P ^ ((ww >> 2) & 3) (8 channels) of halo voxel (hh, ww).
  const int xr = XS ? a.x.r : 1;
  int a_rel[NAW], a_hw[NAW], a_p8[NAW];
#pragma unroll
  for (int k = 0; k < NAW; ++k) {
    const int i = wave + NW * k;
    const int v = 16 * i + (lane >> 2);
    const int hh = v / HWd, ww = v - (v / HWd) * HWd;
    const int p = (lane & 3) ^ ((ww >> 2) & 3);
    const bool row = i < NAI && v < HROWS;
    a_hw[k] = row ? ((hh << 8) | ww) : -1;
    a_p8[k] = 8 * p;
    a_rel[k] = (int)((int64_t)hh * xr * a.x.sh + (int64_t)ww * xr * a.x.sw) + 8 * p;
  }
  // B: row = tap*NT + n (64 B = 32 input channels), piece swizzle (row>>2)&3.
  int b_rel[NBW];
#pragma unroll
  for (int k = 0; k < NBW; ++k) {
    // (PRO: a wave past the last B instruction repeats it -- the same bytes
    // to the same place -- so every wave issues NBW B DMAs per stage)
    const int i = PRO ? min(wave + NW * k, NBI - 1) : wave + NW * k;
    const int row = 16 * i + (lane >> 2);
    const int tap = row / NT, n = row - (row / NT) * NT;
    const int p = (lane & 3) ^ ((row >> 2) & 3);
    b_rel[k] = (tap * a.cout_pad + n) * a.cin_pad + 8 * p;
  }
  // ds_read bases (bytes within a slot)
  uint32_t aoff[KK][2], boff[2];
#pragma unroll
  for (int kw = 0; kw < KK; ++kw)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
      aoff[kw][ks] = (uint32_t)((wave * MS * HWd + kw + r) * 64 + 16 * ((2 * ks + hf) ^ (((kw + r) >> 2) & 3)));
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) boff[ks] = (uint32_t)(r * 64 + 16 * ((2 * ks + hf) ^ ((r >> 2) & 3)));

  // ---- tiles of this workgroup (XCD group x owns a contiguous range) ----
  const int G = gridDim.x;
  const int xg = blockIdx.x & 7, j = blockIdx.x >> 3;
  const int gx = (G >> 3) + (xg < (G & 7) ? 1 : 0);
  const int cx = xg * (G >> 3) + min(xg, G & 7);
  const int t_lo = (int)((int64_t)a.ntiles * cx / G);
  const int t_hi = (int)((int64_t)a.ntiles * (cx + gx) / G);
  const int nchunk = (a.cin + 31) / 32;

  struct Tile {
    int nb, dz, h0, w0, n0, kd_lo, nst;
  };
  // Tile order: output channel tile fastest, then -- for a depth kernel
  // (kd > 1) -- output depth, then columns, rows, sample.  With depth next,
  // the workgroups of one XCD (a contiguous tile range) walk the depths of a
  // few spatial tiles together, so each staged input slice serves its kd
  // output depths out of that XCD's L2; in the (column, row, depth) order an
  // XCD swept a whole 128 x 128 slice per depth and three F-channel input
  // slices (6-21 MB) overflowed its 4 MB L2: the DUF 3x3x3 conv read 2.15x
  // its algorithmic bytes from HBM (PMC, profiles/traffic_duf_bf16.json).
  const bool depth_major = a.kd > 1;
  auto decode = [&](int t) __attribute__((always_inline)) {
    Tile tl;
    const int tn = t % a.ntn;
    int tm = t / a.ntn;
    int tw_i, th_i;
    if (depth_major) {
      tl.dz = tm % a.y.d;
      tm /= a.y.d;
      tw_i = tm % a.tiles_w;
      tm /= a.tiles_w;
      th_i = tm % a.tiles_h;
      tl.nb = tm / a.tiles_h;
    } else {
      tw_i = tm % a.tiles_w;
      tm /= a.tiles_w;
      th_i = tm % a.tiles_h;
      tm /= a.tiles_h;
      tl.dz = tm % a.y.d;
      tl.nb = tm / a.y.d;
    }
    tl.h0 = th_i * FTH;
    tl.w0 = tw_i * TW;
    tl.n0 = tn * NT;
    tl.kd_lo = max(0, a.pd - tl.dz);
    const int kd_hi = min(a.kd, a.x.d + a.pd - tl.dz);
    tl.nst = max(1, kd_hi - tl.kd_lo) * nchunk;
    return tl;
  };

  const char* zp = reinterpret_cast<const char*>(g_zero_page);
  unsigned tmask = 0;  // spatial validity of this lane's A chunks for the current tile
  // DMA of stage s of tile tl into ring slot `slot`, split so that its
  // wave-instructions can be spread over the MFMAs of the running stage:
  // prep() resolves the stage's base addresses and the lane's chunk
  // validity, dma(q) issues this wave's q-th instruction (A chunks first).
  struct Dma {
    const H* xb;
    const H* wsrc;
    uint32_t sbase;
    unsigned m;  // valid A chunks of this lane (bit k)
    int c0;      // first input channel of the stage
    int slot;
    bool on;
  };
  auto prep = [&](const Tile& tl, int s, int slot) __attribute__((always_inline)) {
    Dma d;
    const int kdi = tl.kd_lo + s / nchunk;
    const int c0 = (s % nchunk) * 32;
    const int di = tl.dz + kdi - a.pd;
    const int hb = tl.h0 - a.ph, wb = tl.w0 - a.pw;
    if (s == 0) {
      tmask = 0;
#pragma unroll
      for (int k = 0; k < NAW; ++k) {
        const int hh = a_hw[k] >> 8, ww = a_hw[k] & 0xff;
        const bool ok = a_hw[k] >= 0 && hb + hh >= 0 && hb + hh < a.x.h && wb + ww >= 0 && wb + ww < a.x.w;
        tmask |= (ok ? 1u : 0u) << k;
      }
    }
    const bool dok = di >= 0 && di < a.x.d;
    int64_t xoff;
    if constexpr (XS) {
      const int sub = c0 / a.x.cphys, cc = c0 - sub * a.x.cphys;
      const int si = sub / xr, sj = sub - si * xr;
      xoff = tl.nb * a.x.sn + (int64_t)(dok ? di : 0) * a.x.sd + (int64_t)(hb * xr + si) * a.x.sh +
             (int64_t)(wb * xr + sj) * a.x.sw + cc;
    } else {
      xoff = tl.nb * a.x.sn + (int64_t)(dok ? di : 0) * a.x.sd + (int64_t)hb * a.x.sh + (int64_t)wb * a.x.sw + c0;
    }
    d.xb = reinterpret_cast<const H*>(a.x.ptr) + xoff;
    d.wsrc = reinterpret_cast<const H*>(a.w) + ((int64_t)kdi * TAPS * a.cout_pad + tl.n0) * a.cin_pad + c0;
    d.sbase = lds_addr(lds) + slot * SLOT;
    d.c0 = c0;
    d.slot = slot;
    d.m = 0;
#pragma unroll
    for (int k = 0; k < NAW; ++k) {
      const bool ok = dok && ((tmask >> k) & 1) && c0 + a_p8[k] < a.cin;
      d.m |= (ok ? 1u : 0u) << k;
    }
    d.on = true;
    return d;
  };
  auto dma = [&](const Dma& d, int q) __attribute__((always_inline)) {
    if (q < NAW) {
      const int i = wave + NW * q;
      if (i < NAI) {
        const void* src = ((d.m >> q) & 1) ? (const void*)(d.xb + a_rel[q]) : (const void*)zp;
        glds16(src, d.sbase + i * 1024);
      }
    } else if (q < NAW + NBW && !(a.ablate & 8)) {
      const int i = PRO ? min(wave + NW * (q - NAW), NBI - 1) : wave + NW * (q - NAW);
      if (i < NBI) glds16(d.wsrc + b_rel[q - NAW], d.sbase + ABYTES + i * 1024);
    }
  };
  auto issue = [&](const Tile& tl, int s, int slot) __attribute__((always_inline)) -> unsigned {
    const Dma d = prep(tl, s, slot);
#pragma unroll
    for (int q = 0; q < NQ; ++q) dma(d, q);
    return d.m;
  };

  // BN-affine/ReLU prologue on this lane's own landed A chunks (valid ones;
  // padding stays zero as in the reference, where the conv pads relu(bn(x))).
  auto transform = [&](int slot, int s, unsigned m) __attribute__((always_inline)) {
    const int c0 = (s % nchunk) * 32;
    const bool relu_in = (a.prologue & VSRK_PRO_RELU) != 0;
#pragma unroll
    for (int k = 0; k < NAW; ++k) {
      if ((m >> k) & 1) {
        uint4* p = reinterpret_cast<uint4*>(lds + slot * SLOT + (wave + NW * k) * 1024 + lane * 16);
        *p = prologue_lds<H>(*p, c0 + a_p8[k], relu_in, lsc, lsh);
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

  // MFMAs of one stage, ordered by (kw, k-step): the MS + KK - 1 halo-row A
  // fragments of a (kw, k-step) serve every (row, kh) pair, so a stage reads
  // (MS + KK - 1) + KK * NS fragments per MS * KK * NS MFMAs (0.5 per MFMA at
  // MS = 4, NS = 2).  The next stage's DMA wave-instructions are spread over
  // the groups so they interleave with the math.
  constexpr int ITERS = KK * 2;
  constexpr int QPG = (NQ + ITERS - 1) / ITERS;  // DMA instructions per group
  // Late prologue (PRO): the BN-affine+ReLU transform of the NEXT stage's A
  // chunks runs inside this stage's MFMA groups, from group TSTART on (one
  // group after the last A DMA was issued), instead of between the DMA wait
  // and the barrier where every wave of the workgroup did it at once.  It is
  // branch-free: a lane's chunk outside the image stays zero, and in the
  // last stage (no next stage) a chunk of the current slot is rewritten
  // unchanged.  Measured: -2 % on the DUF 3x3x3 convs (the transform is
  // issue-bound, ~26 VALU per 8 channels, not latency-bound).
  constexpr int TSTART = ((NAW + QPG - 1) / QPG + 1 < ITERS) ? (NAW + QPG - 1) / QPG + 1 : ITERS - 1;
  constexpr int NB_AFTER = (TSTART * QPG < NQ ? TSTART * QPG : NQ) - NAW;  // DMAs issued after the A chunks
  // (1x1 convs: too few groups per stage -- their prologue stays up front)
  constexpr bool LATE = PRO && NB_AFTER >= 0 && TSTART < ITERS;
  const bool relu_in = (a.prologue & VSRK_PRO_RELU) != 0;
  auto late_chunk = [&](const Dma& d, int k) __attribute__((always_inline)) {
    const int sl = d.on ? d.slot : d.slot ^ 1;  // !on: d.slot is the other slot; rewrite the current one
    uint4* p = reinterpret_cast<uint4*>(lds + sl * SLOT + (wave + NW * k) * 1024 + lane * 16);
    const uint4 v = *p;
    const uint4 t = prologue_lds<H>(v, d.c0 + a_p8[k], relu_in, lsc, lsh);
    const bool ok = (d.m >> k) & 1;
    uint4 o;
    o.x = d.on ? (ok ? t.x : 0u) : v.x;
    o.y = d.on ? (ok ? t.y : 0u) : v.y;
    o.z = d.on ? (ok ? t.z : 0u) : v.z;
    o.w = d.on ? (ok ? t.w : 0u) : v.w;
    *p = o;
  };
  // Software-pipelined by hand: group it+1's fragments are read before group
  // it's MFMAs and DMAs are issued (the DMA asm statements are memory
  // barriers to hipcc, which would otherwise never hoist a ds_read across
  // them and expose the LDS latency at every group).
  struct Frags {
    uint4 ax[MS + KK - 1], bw[KK][NS];
  };
  auto compute = [&](int slot, const Dma& d) __attribute__((always_inline)) {
    const char* sA = lds + slot * SLOT;
    const char* sB = sA + ABYTES;
    auto load = [&](Frags& f, int it) __attribute__((always_inline)) {
      const int kw = it >> 1, ks = it & 1;
      const char* pa = sA + aoff[kw][ks];
      const char* pb = sB + boff[ks];
#pragma unroll
      for (int hr = 0; hr < MS + KK - 1; ++hr) f.ax[hr] = *reinterpret_cast<const uint4*>(pa + hr * HWd * 64);
#pragma unroll
      for (int kh = 0; kh < KK; ++kh)
#pragma unroll
        for (int ns = 0; ns < NS; ++ns)
          f.bw[kh][ns] = *reinterpret_cast<const uint4*>(pb + ((kh * KK + kw) * NT + ns * 32) * 64);
    };
    Frags fr[2];
    load(fr[0], 0);
#pragma unroll
    for (int it = 0; it < ITERS; ++it) {
      if (it + 1 < ITERS) load(fr[(it + 1) & 1], it + 1);
      const Frags& f = fr[it & 1];
      if constexpr (LATE) {
        if (it == TSTART) wait_vmcnt<(NB_AFTER >= 0 ? NB_AFTER : 0)>();
        if (it >= TSTART) {
#pragma unroll
          for (int k = 0; k < NAW; ++k)
            if (TSTART + (k * (ITERS - TSTART)) / NAW == it) late_chunk(d, k);
        }
      }
#pragma unroll
      for (int kh = 0; kh < KK; ++kh)
#pragma unroll
        for (int ms = 0; ms < MS; ++ms)
#pragma unroll
          for (int ns = 0; ns < NS; ++ns) mma<H>(acc[ms][ns], f.bw[kh][ns], f.ax[ms + kh]);
      if (d.on) {
#pragma unroll
        for (int q = it * QPG; q < (it + 1) * QPG; ++q) dma(d, q);
      }
    }
  };

  // Epilogue: acc[ms][ns][4g+e] is output channel n0 + ns*32 + 8g + 4hf + e of
  // voxel (ho = h0 + wave*MS + ms, wo = w0 + r).  out = fma(acc, out_scale,
  // bias*out_scale) [relu] [* (mask > 0)] [+ residual] [+ out].  MODE (bits:
  // 1 residual, 2 mask, 4 accumulate) is compile-time per copy so the common
  // forms carry no dead work; row/channel checks only on partial tiles.
  auto epi_mode = [&](const Tile& tl, auto mode_c) __attribute__((always_inline)) {
    constexpr int MODE = decltype(mode_c)::value;
    // MODE = the forms this copy may apply; the generic copy (7) applies the
    // ones the call asks for (a missing residual/mask view aliases y).
    const bool use_res = (MODE & 1) && a.has_res, use_msk = (MODE & 2) && a.has_mask,
               use_acc = (MODE & 4) && a.accumulate;
    using Pk = typename std::conditional<sizeof(YT) == 4, uint4, uint2>::type;
    const bool full = tl.h0 + FTH <= a.y.h && tl.w0 + TW <= a.y.w && tl.n0 + NT <= a.cout;
    const bool act = a.act != VSRK_ACT_NONE;
    const float osc = a.out_scale;
#pragma unroll
    for (int ms = 0; ms < MS; ++ms) {
      const int ho = tl.h0 + wave * MS + ms, wo = tl.w0 + r;
      const bool row_ok = full || (ho < a.y.h && wo < a.y.w);
      const int yr = YS ? a.y.r : 1;
      const int64_t ybase = tl.nb * a.y.sn + (int64_t)tl.dz * a.y.sd + (int64_t)ho * yr * a.y.sh + (int64_t)wo * yr * a.y.sw;
      const YT* rp = nullptr;
      const YT* mp = nullptr;
      if constexpr (!YS && (MODE & 1))
        rp = reinterpret_cast<const YT*>(a.res.ptr) + (tl.nb * a.res.sn + (int64_t)tl.dz * a.res.sd +
                                                       (int64_t)ho * a.res.sh + (int64_t)wo * a.res.sw);
      if constexpr (!YS && (MODE & 2))
        mp = reinterpret_cast<const YT*>(a.msk.ptr) + (tl.nb * a.msk.sn + (int64_t)tl.dz * a.msk.sd +
                                                       (int64_t)ho * a.msk.sh + (int64_t)wo * a.msk.sw);
#pragma unroll
      for (int ns = 0; ns < NS; ++ns) {
        const int cb = tl.n0 + ns * 32;  // first channel of this 32-channel block (wave-uniform)
        int64_t yb = ybase + cb;
        if constexpr (YS) {
          const int sub = cb / a.y.cphys, cc = cb - sub * a.y.cphys;
          const int si = sub / yr, sj = sub - si * yr;
          yb = ybase + (int64_t)si * a.y.sh + (int64_t)sj * a.y.sw + cc;
        }
        YT* yp = reinterpret_cast<YT*>(a.y.ptr) + yb + 4 * hf;
        Pk mv[4], rv[4], ov[4];
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int co = cb + 8 * g + 4 * hf;
          const bool ok = row_ok && (full || co < a.cout);
          if constexpr (MODE & 1) rv[g] = (ok && use_res) ? *reinterpret_cast<const Pk*>(rp + co) : Pk{};
          if constexpr (MODE & 2) mv[g] = (ok && use_msk) ? *reinterpret_cast<const Pk*>(mp + co) : Pk{};
          if constexpr (MODE & 4) ov[g] = (ok && use_acc) ? *reinterpret_cast<const Pk*>(yp + 8 * g) : Pk{};
        }
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int co = cb + 8 * g + 4 * hf;
          const float4 bs = *reinterpret_cast<const float4*>(lbias + co);
          float v[4] = {fmaf(acc[ms][ns][4 * g + 0], osc, bs.x), fmaf(acc[ms][ns][4 * g + 1], osc, bs.y),
                        fmaf(acc[ms][ns][4 * g + 2], osc, bs.z), fmaf(acc[ms][ns][4 * g + 3], osc, bs.w)};
          if (act) {
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = act_apply(a.act, v[e], aslope);
          }
          if ((MODE & 2) && use_msk) {
            float mm[4];
            unpack_pk<YT>(mv[g], mm);
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = mask_apply(mm[e], v[e], mslope);
          }
          if constexpr (MODE & 1) {
            float rr[4];
            unpack_pk<YT>(rv[g], rr);
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] += rr[e];
          }
          if constexpr (MODE & 4) {
            float o[4];
            unpack_pk<YT>(ov[g], o);
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] += o[e];
          }
          if (full) {
            *reinterpret_cast<Pk*>(yp + 8 * g) = pack_pk<YT, Pk>(v);
          } else if (row_ok && co < a.cout) {
            const int valid = a.cout - co;
            if (valid >= 4) {
              *reinterpret_cast<Pk*>(yp + 8 * g) = pack_pk<YT, Pk>(v);
            } else {
              for (int e = 0; e < valid; ++e) yp[8 * g + e] = from_f32<YT>(v[e]);
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
  // Transposed epilogue (H output): per (row ms, block of CB channels)
  // each wave parks its raw fp32 accumulators in a private LDS scratch
  // [32 voxels][CB] (rows padded 16 B: conflict-free b128 writes), reads
  // them back as (voxel, 8 consecutive channels) per lane and finishes
  // there, so every global access is 16 contiguous bytes and a wave
  // instruction covers 64/(CB/8) whole voxels (1 KiB contiguous for a
  // 64-channel channels-last row) instead of 32 voxels x 8 bytes.
  //
  // Operand prefetch: when the epilogue reads exactly one extra tensor
  // (residual: fwd of the second conv of a residual block and the dgrad
  // that adds the skip gradient; ReLU mask: dgrad through an activation),
  // its 16-byte chunks are loaded into registers at the start of the tile's
  // LAST stage, so they land under that stage's MFMAs.  Without this every
  // wave of the workgroup stalls on them together at epilogue time and the
  // MFMA pipes idle (EDSR 64->64: 120 us plain vs 171 us with a residual).
  constexpr int PLPV = CB / 8, PVPI = 64 / PLPV, PNST = 32 / PVPI;
  constexpr int PNB = NT / CB;
  constexpr bool PREF = TRANS && !YS;
  const int pmode = !PREF ? 0 : (a.has_res && !a.has_mask && !a.accumulate) ? 1
                              : (a.has_mask && !a.has_res && !a.accumulate) ? 2 : 0;
  uint4 pre[MS][PNB][PNST];
  auto prefetch = [&](const Tile& tl) __attribute__((always_inline)) {
    if constexpr (PREF) {
      const View& pv = pmode == 1 ? a.res : a.msk;
#pragma unroll
      for (int ms = 0; ms < MS; ++ms) {
        const int ho = tl.h0 + wave * MS + ms;
#pragma unroll
        for (int cbk = 0; cbk < PNB; ++cbk) {
          const int co = tl.n0 + cbk * CB + (lane % PLPV) * 8;
          const H* rowp = reinterpret_cast<const H*>(pv.ptr) +
                             (tl.nb * pv.sn + (int64_t)tl.dz * pv.sd + (int64_t)ho * pv.sh + co);
#pragma unroll
          for (int st = 0; st < PNST; ++st) {
            const int wo = tl.w0 + st * PVPI + lane / PLPV;
            const bool ok = ho < a.y.h && wo < a.y.w && co < a.cout;
            pre[ms][cbk][st] =
                ok ? *reinterpret_cast<const uint4*>(rowp + (int64_t)wo * pv.sw) : make_uint4(0, 0, 0, 0);
          }
        }
      }
    }
  };
  auto epi_tr = [&](const Tile& tl, auto mode_c) __attribute__((always_inline)) {
    constexpr int MODE = decltype(mode_c)::value;
    // MODE 1 / 2 are exactly pmode 1 / 2 (one extra operand, no accumulate)
    constexpr bool USE_PRE = PREF && (MODE == 1 || MODE == 2);
    const bool use_res = (MODE & 1) && a.has_res, use_msk = (MODE & 2) && a.has_mask,
               use_acc = (MODE & 4) && a.accumulate;
    constexpr int LPV = CB / 8;    // lanes per voxel
    constexpr int VPI = 64 / LPV;  // voxels per wave instruction
    constexpr int RS = CB * 4 + 16;
    char* scr = lds + SCR_BASE(slot_epi) + wave * 32 * RS;
    const bool act = a.act != VSRK_ACT_NONE;
    const float osc = a.out_scale;
    const int c8 = (lane % LPV) * 8;
#pragma unroll
    for (int ms = 0; ms < MS; ++ms) {
      const int ho = tl.h0 + wave * MS + ms;
      if (ho >= a.y.h) continue;  // wave-uniform
      const int yr = YS ? a.y.r : 1;
#pragma unroll
      for (int cbk = 0; cbk < NT / CB; ++cbk) {
        const int cb = tl.n0 + cbk * CB;
        if (cb >= a.cout) continue;  // wave-uniform
#pragma unroll
        for (int nl = 0; nl < CB / 32; ++nl)
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            const f32x16& A = acc[ms][cbk * (CB / 32) + nl];
            *reinterpret_cast<float4*>(scr + r * RS + (nl * 32 + 8 * g + 4 * hf) * 4) =
                make_float4(A[4 * g], A[4 * g + 1], A[4 * g + 2], A[4 * g + 3]);
          }
        const int co = cb + c8;
        const float4 b0 = *reinterpret_cast<const float4*>(lbias + co);
        const float4 b1 = *reinterpret_cast<const float4*>(lbias + co + 4);
        const float bsv[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
        int64_t ych = cb;  // channel part of the output offset
        if constexpr (YS) {
          const int sub = cb / a.y.cphys, cc = cb - sub * a.y.cphys;
          const int si = sub / yr, sj = sub - si * yr;
          ych = (int64_t)si * a.y.sh + (int64_t)sj * a.y.sw + cc;
        }
        const int64_t yrow = tl.nb * a.y.sn + (int64_t)tl.dz * a.y.sd + (int64_t)ho * yr * a.y.sh + ych + c8;
#pragma unroll
        for (int st = 0; st < 32 / VPI; ++st) {
          const int vx = st * VPI + lane / LPV;
          const int wo = tl.w0 + vx;
          const bool ok = wo < a.y.w && co < a.cout;
          const float4 q0 = *reinterpret_cast<const float4*>(scr + vx * RS + c8 * 4);
          const float4 q1 = *reinterpret_cast<const float4*>(scr + vx * RS + c8 * 4 + 16);
          float t[8] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w};
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            t[e] = fmaf(t[e], osc, bsv[e]);
            if (act) t[e] = act_apply(a.act, t[e], aslope);
          }
          H* yp = reinterpret_cast<H*>(a.y.ptr) + yrow + (int64_t)wo * yr * a.y.sw;
          if ((MODE & 2) && use_msk) {
            const H* mp = reinterpret_cast<const H*>(a.msk.ptr) + (tl.nb * a.msk.sn + (int64_t)tl.dz * a.msk.sd +
                                                                           (int64_t)ho * a.msk.sh + (int64_t)wo * a.msk.sw + co);
            uint4 mv;
            if constexpr (USE_PRE) mv = pre[ms][cbk][st];
            else mv = ok ? *reinterpret_cast<const uint4*>(mp) : make_uint4(0, 0, 0, 0);
            float m[8];
            Chunk<H>::unpack(mv, m);
#pragma unroll
            for (int e = 0; e < 8; ++e) t[e] = mask_apply(m[e], t[e], mslope);
          }
          if ((MODE & 1) && use_res) {
            const H* rp = reinterpret_cast<const H*>(a.res.ptr) + (tl.nb * a.res.sn + (int64_t)tl.dz * a.res.sd +
                                                                           (int64_t)ho * a.res.sh + (int64_t)wo * a.res.sw + co);
            uint4 rv;
            if constexpr (USE_PRE) rv = pre[ms][cbk][st];
            else rv = ok ? *reinterpret_cast<const uint4*>(rp) : make_uint4(0, 0, 0, 0);
            float rr[8];
            Chunk<H>::unpack(rv, rr);
#pragma unroll
            for (int e = 0; e < 8; ++e) t[e] += rr[e];
          }
          if ((MODE & 4) && use_acc) {
            const uint4 ov = ok ? *reinterpret_cast<const uint4*>(yp) : make_uint4(0, 0, 0, 0);
            float o[8];
            Chunk<H>::unpack(ov, o);
#pragma unroll
            for (int e = 0; e < 8; ++e) t[e] += o[e];
          }
          if (ok) *reinterpret_cast<uint4*>(yp) = Chunk<H>::pack(t);
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
  const int emode = (a.has_res ? 1 : 0) | (a.has_mask ? 2 : 0) | (a.accumulate ? 4 : 0);
  auto epilogue = [&](const Tile& tl) __attribute__((always_inline)) {
    if constexpr (TRANS) {
      if (emode == 0) epi_tr(tl, std::integral_constant<int, 0>{});
      else if (emode == 1) epi_tr(tl, std::integral_constant<int, 1>{});
      else if (emode == 2) epi_tr(tl, std::integral_constant<int, 2>{});
      else epi_tr(tl, std::integral_constant<int, 7>{});
    } else {
      if (emode == 0) epi_mode(tl, std::integral_constant<int, 0>{});
      else if (emode == 1) epi_mode(tl, std::integral_constant<int, 1>{});
      else if (emode == 2) epi_mode(tl, std::integral_constant<int, 2>{});
      else epi_mode(tl, std::integral_constant<int, 7>{});
    }
  };

  // Main loop, one iteration per stage.  A tile's epilogue is deferred to
  // the next iteration, right after its barrier and before that iteration's
  // DMA is issued: its stores then drain under the MFMAs instead of in front
  // of the next vmcnt wait, and any loads it makes are waited for before a
  // DMA is in flight.
  int t = t_lo + j;
  if (t >= t_hi) return;
  Tile cur = decode(t), prev = cur;
  bool pend = false;
  int s = 0, slot = 0;
  unsigned mcur = issue(cur, 0, 0), mnxt = 0;
  bool pro_done = false;  // stage s's A chunks were transformed by the previous compute (late prologue)
  __syncthreads();  // bias / prologue tables visible
  while (true) {
    // the stage after this one (possibly the first stage of the next tile)
    Tile nxt = cur;
    int ns_ = s + 1;
    bool have_next = true;
    if (ns_ >= cur.nst) {
      ns_ = 0;
      const int tn = t + gx;
      if (tn < t_hi) nxt = decode(tn); else have_next = false;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's DMA of stage s has landed
    if constexpr (PRO) {
      if (!pro_done) transform(slot, s, mcur);  // first stage: no earlier compute transformed it
    }
    __syncthreads();  // every wave's DMA of stage s landed (and transformed); slot^1 is free
    if (pend) {
      slot_epi = slot ^ 1;
      if (!(a.ablate & 4)) epilogue(prev);
      pend = false;
      // the scratch was the slot the next DMA fills: every wave must be done with it
      if constexpr (TRANS && !SCR_OWN) {
        if (have_next) __syncthreads();
      }
    }
    Dma dn;
    dn.on = false;
    dn.slot = slot ^ 1;
    dn.m = 0;
    dn.c0 = 0;
    if (have_next && !(a.ablate & 1)) {
      dn = prep(nxt, ns_, slot ^ 1);
      mnxt = dn.m;
    }
    if (pmode && s + 1 >= cur.nst) prefetch(cur);  // lands under this stage's MFMAs
    if (!(a.ablate & 2)) {
      compute(slot, dn);
      pro_done = LATE && dn.on;
    } else if (dn.on) {
#pragma unroll
      for (int q = 0; q < NQ; ++q) dma(dn, q);
    }
    if (s + 1 >= cur.nst) {
      prev = cur;
      pend = true;
    }
    if (!have_next) break;
    if (ns_ == 0) t += gx;
    cur = nxt;
    s = ns_;
    slot ^= 1;
    mcur = mnxt;
  }
  if (pend) {
    slot_epi = slot ^ 1;
    epilogue(prev);
  }
}


template <int KK, int NT, int MS, int XS, int YS, int PRO, typename YT, int NW, typename H>
int launch_fast(FastArgs a, hipStream_t s) {
  constexpr int FTH = NW * MS;
  constexpr int HWd = TW + KK - 1;
  constexpr int NAI0 = ((FTH + KK - 1) * HWd + 15) / 16;
  constexpr int NAI = PRO ? (NAI0 + NW - 1) / NW * NW : NAI0;  // as in the kernel
  constexpr int SLOT = NAI * 1024 + KK * KK * NT * 64;
  constexpr bool TRANS = sizeof(YT) == 2;
  constexpr int CB = (!YS && SLOT >= NW * 32 * (NT * 4 + 16)) ? NT : 32;
  constexpr bool SCR_OWN = TRANS && SLOT < NW * 32 * (CB * 4 + 16);
  a.tiles_h = ceil_div(a.y.h, FTH);
  const int64_t ntiles = (int64_t)a.y.n * a.y.d * a.tiles_h * a.tiles_w * a.ntn;
  VSRK_CHECK(ntiles < (1ll << 31), "conv_fwd: too many tiles");
  a.ntiles = (int)ntiles;
  if (a.ntiles == 0) return VSRK_OK;
  const size_t lds = 2 * (size_t)SLOT + (SCR_OWN ? NW * 32 * (CB * 4 + 16) : 0) + (size_t)a.cout_pad * 4 +
                     (PRO ? 2 * (size_t)a.cin_pad * 4 : 0);
  if (lds > 160 * 1024) return kFastNotEligible;  // e.g. a 4096-entry bias table: generic kernel
  auto kern = conv_fast_kernel<KK, NT, MS, XS, YS, PRO, YT, NW, H>;
  (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  const int grid = fast_grid(ntiles);
  kern<<<grid, NW * 64, lds, s>>>(a);
  VSRK_LAUNCH_CHECK("conv_fwd(fast)");
  return VSRK_OK;
}

template <int KK, int NT, int MS, int XS, int YS, typename YT, typename H, int NW = 8>
int fast_pro(const FastArgs& a, hipStream_t s) {
  if (a.prologue) return launch_fast<KK, NT, MS, XS, YS, 1, YT, NW, H>(a, s);
  return launch_fast<KK, NT, MS, XS, YS, 0, YT, NW, H>(a, s);
}

// y in fp32 or in the input's 16-bit type H (bf16 / fp16)
template <int KK, int NT, int MS, int XS, int YS>
int fast_y(const FastArgs& a, bool yf, bool h16, hipStream_t s) {
  if (h16) return yf ? fast_pro<KK, NT, MS, XS, YS, float, f16>(a, s) : fast_pro<KK, NT, MS, XS, YS, f16, f16>(a, s);
  return yf ? fast_pro<KK, NT, MS, XS, YS, float, bf16>(a, s) : fast_pro<KK, NT, MS, XS, YS, bf16, bf16>(a, s);
}
}  // namespace
#endif  // VSRK_FAST_KERNEL_TU
