// Rolling-depth weight/bias gradient of a 16-bit Conv3d 3x3x3: the autograd
// of DUF's dense-unit convs nn.Conv3d(F, 32, 3, padding=(p, 1, 1)).weight /
// .bias in loss.backward() (duf_net.py:203,214; base_trainer.py:128).
//
// What bounded conv_wgrad_pipe (PMC, DUF 64->32: 9.3 VALU per MFMA, MFMA
// pipes 28 % busy): a workgroup owned ONE kd tap, so every input slice was
// staged, BN-affine+ReLU-transformed and read three times (once per kd), and
// the staging went through registers.  Here:
//  * A workgroup owns a 32 (output) x 32 (input) channel block and all 27
//    taps, and walks the input depth slices di of its tiles once.  Stage di
//    brings x slice di and output-gradient slice dz = di + pd; the three
//    output-gradient slices di + pd - kd that slice di meets (kd = 0, 1, 2)
//    sit in a five-slot LDS ring, so every x slice and every dy slice is
//    staged and transformed once.
//  * Both operands arrive by LDS-DMA (global_load_lds_dwordx4), three stages
//    in flight; the BN/ReLU prologue is applied in LDS by the wave that
//    issued a piece, one stage early, beside the MFMAs.
//  * v_mfma_f32_16x16x32_{bf16,f16} on ds_read_b64_tr_b16 operands: a wave
//    holds all 27 taps of a 16 x 16 (output x input) channel block in 108
//    accumulator registers; 8 waves = 2 output halves x 2 input halves x 2
//    row halves of the tile.  LDS images are voxel-major rows of 32 channels
//    (64 B) with the two 32-byte halves XOR-swizzled by bit 3 of the voxel
//    index; x halo rows are 40 voxels long (34 used) so that bit depends on
//    the halo row and column separately and every fragment address is a
//    per-lane base plus a compile-time offset.  Transposed reads are
//    conflict-free.
//  * Deterministic: per-(split, row half) fp32 slabs in conv_wgrad.hip's
//    layout ([9 taps][32 co][32 ci] + dbias per kd "combo"), summed in a
//    fixed order by wgrad_reduce_kernel.  dbias: an MFMA against ones on each
//    dy slice once (workgroups of input chunk 0).
#include <cstdlib>
#include "conv_common.h"

namespace {
using namespace vsrk_conv;

constexpr int WNW = 8;                    // waves
constexpr int WTH = 8;                    // dy tile rows
constexpr int WHR = WTH + 2;              // 10 halo rows
constexpr int WHS = 40;                   // halo row stride in voxels (34 used)
constexpr int WXV = WHR * WHS;            // 400 x voxels per slot
constexpr int WNXP = WXV / 16;            // 25 x pieces (16 voxels x 64 B)
constexpr int WDV = WTH * TW;             // 256 dy voxels
constexpr int WNDP = WDV / 16;            // 16 dy pieces
constexpr int WNP = WNXP + WNDP;          // 41
constexpr int WNQ = (WNP + WNW - 1) / WNW;  // 6 pieces per wave and stage
constexpr int WXSLOT = WNXP * 1024;       // 25,600 B
constexpr int WDSLOT = WNDP * 1024;       // 16,384 B
constexpr int WNXS = 3, WNDS = 5;         // ring slots
constexpr int WDBASE = WNXS * WXSLOT;     // dy ring base
constexpr int WJUNK = WDBASE + WNDS * WDSLOT;
constexpr int WLDS = WJUNK + 1024;        // + prologue tables (2 x 32 floats)

struct RDivW {
  uint32_t d, mul, p;
};
RDivW make_rdivw(int d) {
  int l = 0;
  while ((1u << l) < (uint32_t)d) ++l;
  const uint32_t p = 31 + l;
  return RDivW{(uint32_t)d, (uint32_t)(((1ull << p) + (uint64_t)d - 1) / (uint64_t)d), p};
}
__device__ __forceinline__ int rdivw(int x, const RDivW& f) { return (int)(((uint64_t)(uint32_t)x * f.mul) >> f.p); }

struct WRArgs {
  const char* x;   // element (nb, di, h, w, c) at x + 2 * (nb*xsn + di*xsd + h*xsh + w*xsw + c)
  const char* dy;
  const float* pro_scale;
  const float* pro_shift;
  float* ws;
  int xsn, xsd, xsh, xsw, ysn, ysd, ysh, ysw;
  int xd, xh, xw, yd, yh, yw;
  int pd, ph, pw;
  int cin, cout, prologue, want_bias;
  int dzc, ntiles, tps, nsplit, nci_chunks, nco_tiles, slab, kd_bias;
  RDivW tiles_w, tiles_h, nzc;
  int prio;  // A/B knob (VSRK_ROLL_PRIO=1): s_setprio 1 for waves 4-7
};

__device__ __attribute__((aligned(256))) uint4 g_wroll_zero[16];
#ifdef ROLL_STAMP
// Diagnostic builds only (tools/conv_microbench.py --stamps): s_memtime
// stamps of waves 0 and 4 (one SIMD) of workgroups 0-15 kept in VGPR lanes,
// stored at exit: per step [after the stage wait, after the barrier, after
// compute]
#ifndef ROLL_STAMP_SKIP
#define ROLL_STAMP_SKIP 8
#endif
__device__ unsigned g_wroll_stamp[16 * 2 * 128];
#endif

#ifndef WR_XWIN
#define WR_XWIN 1
#endif

template <int N>
__device__ __forceinline__ void wr_wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}

typedef float f32x4_t __attribute__((ext_vector_type(4)));
template <typename H> struct V8W;
template <> struct V8W<bf16> { typedef bf16x8 type; };
template <> struct V8W<f16> { typedef f16x8 type; };
__device__ __forceinline__ f32x4_t mfma16(bf16x8 a, bf16x8 b, f32x4_t c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x4_t mfma16(f16x8 a, f16x8 b, f32x4_t c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}
// 8 consecutive voxels (k) of one channel: two transposed 4-row reads
__device__ __forceinline__ uint4 tr_frag(const char* p0, const char* p1) {
  const v4i16 a = ds_read_tr(p0);
  const v4i16 b = ds_read_tr(p1);
  return __builtin_bit_cast(uint4, __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7));
}

struct WTile {
  int nb, h0, w0, z0, z1, di_s, nst;
};

template <int PRO, typename H>
__global__ __launch_bounds__(WNW * 64, 2) void wgrad_roll_kernel(WRArgs a) {
  using V8 = typename V8W<H>::type;
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  if (a.prio && wave >= 4) __builtin_amdgcn_s_setprio(1);
  const int coh = wave & 1, cih = (wave >> 1) & 1, vh = wave >> 2;  // output half, input half, row half

  // ---- which (channel block, split) this workgroup is ----
  const int L = xcd_remap(blockIdx.x, a.nsplit * a.nci_chunks * a.nco_tiles);
  const int split = L / (a.nci_chunks * a.nco_tiles);
  const int combo = L - split * (a.nci_chunks * a.nco_tiles);
  const int cot = combo % a.nco_tiles, cic = combo / a.nco_tiles;
  const int co0 = cot * 32, ci0 = cic * 32;
  const bool do_bias = a.want_bias && cic == 0;
  float* lsc = reinterpret_cast<float*>(lds + WLDS);  // prologue scale / shift of the block's 32 channels
  float* lsh = lsc + 32;
  if constexpr (PRO) {
    if (tid < 32) {
      const int c = ci0 + tid;
      const bool ok = c < a.cin;
      const bool aff = (a.prologue & VSRK_PRO_AFFINE) != 0;
      lsc[tid] = ok ? (aff ? a.pro_scale[c] : 1.f) : 0.f;
      lsh[tid] = ok ? (aff ? a.pro_shift[c] : 0.f) : 0.f;
    }
  }

  // ---- per-lane DMA roles: piece j = wave + 8q fills 1 KB ----
  //  j < 25: x voxel v = 16 j + l/4 of the 10 x 40 halo image (row v/40, col
  //  v%40 < 34), j < 41: dy voxel v = 16 (j - 25) + l/4 of the 8 x 32 tile;
  //  16-byte position l & 3 holds logical piece (l & 3) ^ 2*bit3(v) (8 channels).
  int rel[WNQ], hwv[WNQ];
  unsigned qx = 0, qy = 0;
#pragma unroll
  for (int q = 0; q < WNQ; ++q) {
    const int j = wave + WNW * q;
    rel[q] = 0;
    hwv[q] = -1;
    if (j < WNXP) {
      const int v = 16 * j + (lane >> 2);
      const int hh = v / WHS, ww = v - (v / WHS) * WHS;
      const int p = (lane & 3) ^ (2 * ((v >> 3) & 1));
      rel[q] = hh * a.xsh + ww * a.xsw + 8 * p;
      hwv[q] = ww < TW + 2 ? ((hh << 8) | ww) : -1;
      qx |= 1u << q;
    } else if (j < WNP) {
      const int v = 16 * (j - WNXP) + (lane >> 2);
      const int hr = v / TW, wc = v - (v / TW) * TW;
      const int p = (lane & 3) ^ (2 * ((v >> 3) & 1));
      rel[q] = hr * a.ysh + wc * a.ysw + 8 * p;
      hwv[q] = (hr << 8) | wc;
      qy |= 1u << q;
    }
  }
  // ---- fragment read bases (bytes within a slot) ----
  // lane (g, q, p) of a transposed read supplies voxel (block row) q of the
  // 16-lane group g's 4-voxel block, channels 4p..4p+3 of its 16-channel half.
  const int g = lane >> 4, qq = (lane >> 2) & 3, pp = lane & 3;
  // x: voxel v = 40 R + kw + 8 g + q + 4 h: the swizzle bit is bit 3 of v =
  // (R & 1) ^ bit3(kw + 8g + q + 4h) (40 R is a multiple of 8, 5 R has R's parity)
  // (even R; an odd R flips the 32-byte half: byte address ^ 32)
  uint32_t xb[3][2];  // [kw][h]
#pragma unroll
  for (int kw = 0; kw < 3; ++kw)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int c = kw + 8 * g + qq + 4 * h;
      xb[kw][h] = (uint32_t)((vh * 4 * WHS + c) * 64 + 32 * (cih ^ ((c >> 3) & 1)) + 8 * pp);
    }
  // dy: voxel v = 32 hr + 8 g + q + 4 h: bit 3 of v = g & 1
  uint32_t yb[2];
#pragma unroll
  for (int h = 0; h < 2; ++h)
    yb[h] = (uint32_t)((vh * 4 * TW + 8 * g + qq + 4 * h) * 64 + 32 * (coh ^ (g & 1)) + 8 * pp);

  // ---- tiles: this split's contiguous range ----
  const int t_begin = split * a.tps;
  const int t_end = min(a.ntiles, t_begin + a.tps);
  auto decode = [&](int t) __attribute__((always_inline)) {
    WTile tl;
    int u = rdivw(t, a.nzc);
    tl.z0 = (t - u * (int)a.nzc.d) * a.dzc;
    int v = rdivw(u, a.tiles_w);
    tl.w0 = (u - v * (int)a.tiles_w.d) * TW;
    tl.nb = rdivw(v, a.tiles_h);
    tl.h0 = (v - tl.nb * (int)a.tiles_h.d) * WTH;
    tl.z1 = min(tl.z0 + a.dzc, a.yd);
    tl.di_s = tl.z0 - a.pd;
    tl.nst = min(a.xd - 1, tl.z1 + 1 - a.pd) - tl.di_s + 1;
    return tl;
  };
  // spatial validity of this lane's pieces for a tile (bit q)
  auto tile_mask = [&](const WTile& tl) __attribute__((always_inline)) {
    unsigned m = 0;
#pragma unroll
    for (int q = 0; q < WNQ; ++q) {
      const int hh = hwv[q] >> 8, ww = hwv[q] & 0xff;
      bool ok;
      if ((qx >> q) & 1)
        ok = hwv[q] >= 0 && (unsigned)(tl.h0 - a.ph + hh) < (unsigned)a.xh && (unsigned)(tl.w0 - a.pw + ww) < (unsigned)a.xw;
      else
        ok = ((qy >> q) & 1) && tl.h0 + hh < a.yh && tl.w0 + ww < a.yw;
      m |= (ok ? 1u : 0u) << q;
    }
    return m;
  };

  struct Walk {
    int t, k;  // tile, stage within it
    WTile tl;
    unsigned m;
  };
  auto advance = [&](Walk& w) __attribute__((always_inline)) -> bool {
    if (++w.k < w.tl.nst) return true;
    w.k = 0;
    if (++w.t >= t_end) return false;
    w.tl = decode(w.t);
    w.m = tile_mask(w.tl);
    return true;
  };
  const char* zp = reinterpret_cast<const char*>(g_wroll_zero);
  asm volatile("" : "+v"(zp));  // the zero page address in a VGPR pair, not re-materialised per piece
  // DMA of walk w's stage into x slot xs / dy slot ys
  struct Dma {
    const H* xb;
    const H* yb;
    unsigned use;
  };
  auto prep = [&](const Walk& w) __attribute__((always_inline)) {
    Dma d;
    const int di = w.tl.di_s + w.k, dz = di + a.pd;
    const bool xok = di >= 0, yok = dz >= w.tl.z0 && dz < w.tl.z1;
    d.xb = reinterpret_cast<const H*>(a.x) +
           (w.tl.nb * a.xsn + (xok ? di : 0) * a.xsd + (w.tl.h0 - a.ph) * a.xsh + (w.tl.w0 - a.pw) * a.xsw + ci0);
    d.yb = reinterpret_cast<const H*>(a.dy) +
           (w.tl.nb * a.ysn + (yok ? dz : w.tl.z0) * a.ysd + w.tl.h0 * a.ysh + w.tl.w0 * a.ysw + co0);
    d.use = w.m & ((xok ? qx : 0u) | (yok ? qy : 0u));
    return d;
  };
  auto dma = [&](Dma d, int q, int xs, int ys) __attribute__((always_inline)) {
    const int j = wave + WNW * q;
    const H* base = ((qx >> q) & 1) ? d.xb : d.yb;
    const void* src = ((d.use >> q) & 1) ? (const void*)(base + rel[q]) : (const void*)zp;
    const int off = j < WNXP ? xs * WXSLOT + j * 1024 : j < WNP ? WDBASE + ys * WDSLOT + (j - WNXP) * 1024 : WJUNK;
    glds16_m0(src, (uint32_t)__builtin_amdgcn_readfirstlane((int)(lds_addr(lds) + off)));
  };
  // BN-affine/ReLU prologue on this lane's own landed x piece q (in-image
  // pieces only: the halo stays zero, the conv pads relu(bn(x)))
  auto transform_piece = [&](int xs, int q, unsigned m) __attribute__((always_inline)) {
    if (((qx & m) >> q) & 1) {
      const int j = wave + WNW * q;
      uint4* p = reinterpret_cast<uint4*>(lds + xs * WXSLOT + j * 1024 + lane * 16);
      const int v = 16 * j + (lane >> 2);
      *p = prologue_lds<H>(*p, 8 * ((lane & 3) ^ (2 * ((v >> 3) & 1))), (a.prologue & VSRK_PRO_RELU) != 0, lsc, lsh);
    }
  };

  f32x4_t acc[3][3][3];  // [kd][kh][kw]: output ch 16 coh + 4 (l >> 4) + i, input ch 16 cih + (l & 15)
#pragma unroll
  for (int i = 0; i < 27; ++i) acc[i / 9][(i / 3) % 3][i % 3] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  f32x4_t bacc = f32x4_t{0.f, 0.f, 0.f, 0.f};  // dbias (MFMA against ones)
  uint4 ones;
  {
    const H one = from_f32<H>(1.f);
    const uint16_t u = __builtin_bit_cast(uint16_t, one);
    const uint32_t w2 = (uint32_t)u | ((uint32_t)u << 16);
    ones = make_uint4(w2, w2, w2, w2);
  }

  // One stage: x slot XS (compile time), dy slots of kd = 0, 1, 2 (runtime
  // byte offsets).  Per dy row r of the wave (4): the 3 dy fragments (one
  // per kd), then per kh the 3 kw fragments of x row r + kh and 3 x 3 MFMAs
  // (kd active x kw).  DMA pieces of the stage two ahead: 2 per row; the late
  // prologue of the next stage: in the last row.
  auto compute = [&](auto xs_c, const uint32_t* yoff, unsigned km, bool newy, Dma dn, bool don, int xs2,
                     int ys2, bool tnext, unsigned tm) __attribute__((always_inline)) {
    constexpr int XS = decltype(xs_c)::value;
    const char* xsl = lds + XS * WXSLOT;
    auto load_x = [&](uint4* f, int R) __attribute__((always_inline)) {
      const uint32_t flip = (R & 1) ? 32u : 0u;
#pragma unroll
      for (int kw = 0; kw < 3; ++kw)
        f[kw] = tr_frag(xsl + ((xb[kw][0] + R * WHS * 64) ^ flip), xsl + ((xb[kw][1] + R * WHS * 64) ^ flip));
    };
    int qi = 0;
    // x rows R = r + kh: each halo row feeds three (r, kh) pairs, so the
    // three rows a dy row meets stay in registers (a sliding window of
    // 3 rows x 3 kw fragments) and each row is read from LDS once per stage:
    // 6 instead of 12 row reads (36 instead of 72 transposed reads per stage;
    // the weight gradient is LDS-read bound).  WR_XWIN=0: the old form.
#if WR_XWIN
    uint4 xw[3][3];
    load_x(xw[0], 0);
    load_x(xw[1], 1);
#endif
#pragma unroll
    for (int r = 0; r < 4; ++r) {
#if WR_XWIN
      load_x(xw[(r + 2) % 3], r + 2);
#endif
      uint4 yf[3];
#pragma unroll
      for (int kd = 0; kd < 3; ++kd) {
        const char* ys = lds + yoff[kd] + r * TW * 64;
        yf[kd] = tr_frag(ys + yb[0], ys + yb[1]);
      }
#pragma unroll
      for (int k = 0; k < 2; ++k, ++qi) {
        if (qi < WNQ && don) dma(dn, qi, xs2, ys2);
      }
      if constexpr (PRO) {
        // the next stage's x pieces: waited for once this stage's pieces are
        // all issued (row 2), transformed two per row over rows 2 and 3
        // (one burst in row 3 cost ~30 % of the kernel beside the prologue-free form)
        if (r >= 2 && tnext) {
          if (r == 2) {
            if (don) wr_wait_vmcnt<WNQ>();
            else wr_wait_vmcnt<0>();
          }
#pragma unroll
          for (int q = 2 * (r - 2); q < 2 * (r - 1); ++q) transform_piece((XS + 1) % 3, q, tm);
        }
      }
#if WR_XWIN
      // kd outermost: one branch per (row, kd) for the inactive taps of a
      // slice near the tile's depth ends (12 per stage; per (row, kh, kd)
      // there were 36, each a scalar test and branch between MFMA groups)
#pragma unroll
      for (int kd = 0; kd < 3; ++kd) {
        if ((km >> kd) & 1) {
#pragma unroll
          for (int kh = 0; kh < 3; ++kh) {
            const uint4* xf = xw[(r + kh) % 3];
#pragma unroll
            for (int kw = 0; kw < 3; ++kw)
              acc[kd][kh][kw] = mfma16(__builtin_bit_cast(V8, yf[kd]), __builtin_bit_cast(V8, xf[kw]), acc[kd][kh][kw]);
          }
        }
      }
#else
#pragma unroll
      for (int kh = 0; kh < 3; ++kh) {
        uint4 xf[3];
        load_x(xf, r + kh);
#pragma unroll
        for (int kd = 0; kd < 3; ++kd) {
          if ((km >> kd) & 1) {
#pragma unroll
            for (int kw = 0; kw < 3; ++kw)
              acc[kd][kh][kw] = mfma16(__builtin_bit_cast(V8, yf[kd]), __builtin_bit_cast(V8, xf[kw]), acc[kd][kh][kw]);
          }
        }
      }
#endif
      if (do_bias && cih == 0 && newy)
        bacc = mfma16(__builtin_bit_cast(V8, yf[0]), __builtin_bit_cast(V8, ones), bacc);
    }
  };

  // ---- main loop ----
  Walk cur;
  cur.t = t_begin;
  cur.k = 0;
  const bool any = t_begin < t_end;
  if (any) {
    cur.tl = decode(t_begin);
    cur.m = tile_mask(cur.tl);
  }
  Walk nx = cur;
  bool vn = any;
  int stage = 0;  // global stage index: x slot stage % 3, dy slot stage % 5
  if (any) {
    const Dma d0 = prep(nx);
#pragma unroll
    for (int q = 0; q < WNQ; ++q) dma(d0, q, 0, 0);
    vn = advance(nx);
    if (vn) {
      const Dma d1 = prep(nx);
#pragma unroll
      for (int q = 0; q < WNQ; ++q) dma(d1, q, 1, 1);
      vn = advance(nx);
    }
  }
  bool tnext = false;  // the stage after the current one exists
  unsigned tm = 0;     // its lane mask
  {
    Walk k1 = cur;
    tnext = any && advance(k1);
    tm = k1.m;
  }
  __syncthreads();  // prologue tables visible
  if constexpr (PRO) {
    if (any) {
      if (tnext) wr_wait_vmcnt<WNQ>();
      else wr_wait_vmcnt<0>();
#pragma unroll
      for (int q = 0; q < 4; ++q) transform_piece(0, q, cur.m);
    }
  }
#ifdef ROLL_STAMP
  unsigned stv0 = 0, stv1 = 0;
  int stc = -3 * ROLL_STAMP_SKIP;
  auto stamp = [&]() __attribute__((always_inline)) {
    if (stc >= 0 && stc < 128) {
      const unsigned tv = (unsigned)__builtin_amdgcn_s_memtime();
      if (stc < 64) stv0 = lane == stc ? tv : stv0;
      else stv1 = lane == stc - 64 ? tv : stv1;
    }
    ++stc;
  };
#else
  auto stamp = [&]() __attribute__((always_inline)) {};
#endif
  auto step = [&](auto xs_c) __attribute__((always_inline)) -> bool {
    constexpr int XS = decltype(xs_c)::value;
    if (tnext) wr_wait_vmcnt<WNQ>();
    else wr_wait_vmcnt<0>();
    stamp();
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    stamp();
    const int di = cur.tl.di_s + cur.k, P = di + a.pd;
    unsigned km = 0;
    if (di >= 0) {
#pragma unroll
      for (int kd = 0; kd < 3; ++kd) km |= (P - kd >= cur.tl.z0 && P - kd < cur.tl.z1 ? 1u : 0u) << kd;
    }
    const bool newy = P >= cur.tl.z0 && P < cur.tl.z1;
    uint32_t yoff[3];
#pragma unroll
    for (int kd = 0; kd < 3; ++kd) yoff[kd] = WDBASE + ((stage + 5 - kd) % 5) * WDSLOT;
    Dma dn;
    dn.xb = nullptr;
    dn.yb = nullptr;
    dn.use = 0;
    if (vn) dn = prep(nx);
    compute(xs_c, yoff, km, newy, dn, vn, (XS + 2) % 3, (stage + 2) % 5, tnext, tm);
    stamp();
    // the stage just issued (nx) is the next one's successor
    tnext = vn;
    tm = nx.m;
    if (vn) vn = advance(nx);
    ++stage;
    return advance(cur);
  };
  if (any) {
    while (step(std::integral_constant<int, 0>{}) && step(std::integral_constant<int, 1>{}) &&
           step(std::integral_constant<int, 2>{})) {
    }
  }

#ifdef ROLL_STAMP
  if (blockIdx.x < 16 && (wave == 0 || wave == 4)) {
    unsigned* o = g_wroll_stamp + (blockIdx.x * 2 + (wave >> 2)) * 128;
    o[lane] = stv0;
    o[64 + lane] = stv1;
  }
#endif
  // ---- slabs: split index 2 * split + row half, combo (kd, ci chunk, co tile) ----
  const int ncombo = 3 * a.nci_chunks * a.nco_tiles;
  const int l15 = lane & 15, lg = lane >> 4;
#pragma unroll
  for (int kd = 0; kd < 3; ++kd) {
    const int vc = (kd * a.nci_chunks + cic) * a.nco_tiles + cot;
    float* out = a.ws + ((int64_t)(2 * split + vh) * ncombo + vc) * a.slab;
#pragma unroll
    for (int t9 = 0; t9 < 9; ++t9)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int co = 16 * coh + 4 * lg + i, ci = 16 * cih + l15;
        out[(t9 * 32 + co) * 32 + ci] = acc[kd][t9 / 3][t9 % 3][i];
      }
  }
  if (do_bias && cih == 0) {
    const int vc = (a.kd_bias * a.nci_chunks + 0) * a.nco_tiles + cot;
    float* out = a.ws + ((int64_t)(2 * split + vh) * ncombo + vc) * a.slab + 9 * 1024;
    if (l15 == 0) {
#pragma unroll
      for (int i = 0; i < 4; ++i) out[16 * coh + 4 * lg + i] = bacc[i];
    }
  }
}

#ifdef ROLL_STAMP
}  // namespace
extern "C" int vsrk_wroll_stamps(unsigned* dst) {
  return hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_wroll_stamp), sizeof(g_wroll_stamp)) == hipSuccess ? 0 : 1;
}
namespace {
#endif

int g_wroll_mode = -1;  // -1: VSRK_WGRAD_ROLL (unset: 2), 0 off, 1 forced on, 2 automatic

int wroll_num_cus() {
  static int n = 0;
  if (n == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
  }
  return n;
}

}  // namespace

void vsrk_conv_set_wgrad_roll_mode(int mode) { g_wroll_mode = mode; }

// The plan of the rolling weight gradient for a request, or false when the
// request is not eligible.  Workspace: nsplit*2 x (3 * nci * nco) slabs of
// (9 * 1024 + 32) floats.
bool vsrk_wgrad_roll_plan(const vsrk_conv_desc* d, const vsrk_tensor5* x, const vsrk_tensor5* dy, int* nsplit,
                          int* tps, int* ntiles, int* dzc, size_t* ws_bytes) {
  if (g_wroll_mode < 0) {
    const char* e = getenv("VSRK_WGRAD_ROLL");
    g_wroll_mode = !e ? 2 : (e[0] == '0' ? 0 : 1);
  }
  if (g_wroll_mode == 0) return false;
  // automatic mode: with a single output depth the kd-tap reuse of the
  // rolling walk does not pay for its ring (DUF's last unit, 3 -> 1: 812 vs
  // 982 us for the pipelined kernel); at 3 output depths it does since the
  // round-5 loop order (DUF unit 5 at F = 192, 5 -> 3: 1495 vs 1703 us; it
  // lost, 1764 vs 1619, in round 3)
  if (g_wroll_mode == 2 && dy->d <= 1 && vsrk_g_roll_dz == 0) return false;
  if (!vsrk_is16(x->dtype) || dy->dtype != x->dtype) return false;
  if (d->kd != 3 || d->kh != 3 || d->kw != 3 || d->pd < 0 || d->pd > 2 || d->ph < 0 || d->ph > 2 || d->pw < 0 ||
      d->pw > 2)
    return false;
  if (x->shuffle > 1 || dy->shuffle > 1 || x->c % 32 || dy->c % 32) return false;
  if (!chunk_ok(x, 2) || !chunk_ok(dy, 2)) return false;
  if (dy->d != x->d + 2 * d->pd - 2 || dy->h != x->h + 2 * d->ph - 2 || dy->w != x->w + 2 * d->pw - 2) return false;
  for (const vsrk_tensor5* t : {x, dy}) {
    const int64_t span = (int64_t)(t->n - 1) * t->sn + (int64_t)(t->d - 1) * t->sd + (int64_t)(t->h + WHR) * t->sh +
                         (int64_t)(t->w + WHS) * t->sw + t->c;
    if (span >= (1ll << 31) || t->sn < 0 || t->sd < 0 || t->sh < 0 || t->sw < 0) return false;
  }
  const int nco = dy->c / 32, nci = x->c / 32;
  const int tiles_h = ceil_div(dy->h, WTH), tiles_w = ceil_div(dy->w, TW);
  const int64_t spatial = (int64_t)dy->n * tiles_h * tiles_w;
  // depth runs: whole depth unless the grid would have < 1 tile per workgroup
  int z = dy->d;
  const int combos = nco * nci;
  const int64_t want_wg = std::max<int64_t>(1, wroll_num_cus());
  if (spatial * combos < want_wg) {
    const int64_t runs = std::min<int64_t>(ceil_div64(want_wg, spatial * combos), dy->d);
    z = (int)ceil_div64(dy->d, runs);
  }
  if (vsrk_g_roll_dz > 0) z = std::min(vsrk_g_roll_dz, dy->d);
  const int nz = ceil_div(dy->d, z);
  const int64_t nt = spatial * nz;
  if (nt >= (1ll << 30)) return false;
  // one workgroup per CU (the ring takes the whole LDS): the grid must not
  // spill a few workgroups into a second wave (224 -> 32 with 37 x 7 = 259
  // workgroups on 256 CUs: 6.0 ms, r3e microbench)
  int splits = (int)std::max<int64_t>(1, std::min<int64_t>(nt, want_wg / combos));
  if (vsrk_g_grid_cap > 0) splits = std::max(1, std::min(splits, vsrk_g_grid_cap));
  const int t = (int)ceil_div64(nt, splits);
  splits = (int)ceil_div64(nt, t);
  *nsplit = splits;
  *tps = t;
  *ntiles = (int)nt;
  *dzc = z;
  *ws_bytes = (size_t)2 * splits * 3 * combos * (9 * 1024 + 32) * sizeof(float);
  return true;
}

// 1 = launched the slab kernel (the caller reduces with nsplit * 2 splits,
// 3 * nci * nco combos of 32 x 32 channels, slab 9 * 1024 + 32); 0 = not eligible.
int vsrk_conv_wgrad_roll(const vsrk_conv_desc* d, const vsrk_tensor5* x, const vsrk_tensor5* dy,
                         const float* pro_scale, const float* pro_shift, int want_bias, float* ws, size_t ws_bytes,
                         int* nsplit_out, hipStream_t s) {
  int nsplit, tps, ntiles, dzc;
  size_t need;
  if (!vsrk_wgrad_roll_plan(d, x, dy, &nsplit, &tps, &ntiles, &dzc, &need)) return 0;
  if (ws_bytes < need) return 0;
  const int pro = d->prologue & (VSRK_PRO_AFFINE | VSRK_PRO_RELU);
  WRArgs a;
  a.x = (const char*)x->ptr;
  a.dy = (const char*)dy->ptr;
  a.pro_scale = pro_scale;
  a.pro_shift = pro_shift;
  a.ws = ws;
  a.xsn = (int)x->sn; a.xsd = (int)x->sd; a.xsh = (int)x->sh; a.xsw = (int)x->sw;
  a.ysn = (int)dy->sn; a.ysd = (int)dy->sd; a.ysh = (int)dy->sh; a.ysw = (int)dy->sw;
  a.xd = x->d; a.xh = x->h; a.xw = x->w;
  a.yd = dy->d; a.yh = dy->h; a.yw = dy->w;
  a.pd = d->pd; a.ph = d->ph; a.pw = d->pw;
  a.cin = x->c;
  a.cout = dy->c;
  a.prologue = pro;
  a.want_bias = want_bias;
  a.dzc = dzc;
  a.ntiles = ntiles;
  a.tps = tps;
  a.nsplit = nsplit;
  a.nci_chunks = x->c / 32;
  a.nco_tiles = dy->c / 32;
  a.slab = 9 * 1024 + 32;
  a.kd_bias = std::min(d->pd, 2);
  {
    static int prio = -1;
    if (prio < 0) {
      const char* e = getenv("VSRK_ROLL_PRIO");
      prio = (e && e[0] == '1') ? 1 : 0;
    }
    a.prio = prio;
  }
  a.tiles_w = make_rdivw(ceil_div(dy->w, TW));
  a.tiles_h = make_rdivw(ceil_div(dy->h, WTH));
  a.nzc = make_rdivw(ceil_div(dy->d, dzc));
  const int grid = nsplit * a.nci_chunks * a.nco_tiles;
  const size_t lds = WLDS + 2 * 32 * sizeof(float);
  vsrk_dispatch16(x->dtype, [&](auto tag) {
    using H = decltype(tag);
    auto kern = pro ? wgrad_roll_kernel<1, H> : wgrad_roll_kernel<0, H>;
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    kern<<<grid, WNW * 64, lds, s>>>(a);
    return 0;
  });
  *nsplit_out = nsplit;
  return 1;
}
