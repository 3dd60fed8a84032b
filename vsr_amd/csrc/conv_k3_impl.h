// 3x3 / 3x3x3 implicit-GEMM convolution, second generation (bf16 in, bf16
// out, fp32 accumulate) on CDNA4 -- the EDSR body conv (edsr_net.py:41-53),
// the DUF Conv3d 3x3x3 units (duf_net.py:203,214) and their data gradients
// (base_trainer.py:128), the sub-pixel up-sampler convs (edsr_net.py:61-62)
// and DRF's projections.  Same contract as conv_fast_kernel (conv_fast_impl.h).
//
// Why a second kernel: conv_fast_kernel runs one 8-wave workgroup per CU,
// so every barrier and every tile epilogue stalls all four SIMDs at once,
// and its per-DMA zero-page selects and M0 juggling cost ~20 instructions
// (plus SGPR spills) per 1 KiB piece.  Here:
//  * Two 4-wave workgroups per CU (one wave per SIMD each): one workgroup's
//    epilogue and barrier waits overlap the other's MFMAs.
//  * Register tile of 4 rows x 32 columns x NT output channels per wave
//    (acc 128 VGPRs at NT = 64): per (kw, 16-channel k-step) a wave reads
//    4 + 2 halo-row A fragments and 3 kh x NT/32 B fragments for 12 (NT 32)
//    or 24 (NT 64) v_mfma_f32_32x32x16_bf16: 0.5 ds_read_b128 per MFMA at
//    NT = 64 (the LDS array sustains 2 per MFMA gap).
//  * Stage = (kd tap, 16 input channels), stored as two 8-channel planes of
//    16-byte entries: A [plane][18 halo rows x 34 columns], B [plane][9 taps
//    x NT].  A fragment is 32 consecutive entries of one plane per lane half,
//    so every ds_read_b128 lane group of 16 touches 16 distinct 4-bank sets
//    for any column shift kw: conflict-free without swizzles.
//  * Staging by LDS-DMA from buffer loads (buffer_load_dwordx4 ... lds):
//    each lane's byte offset within the tile is fixed per tile, the stage
//    (kd tap, channel block, sub-pixel) is one scalar offset, and padding
//    (halo outside the image, unused entries) is an out-of-range offset the
//    buffer unit returns as zeros -- no selects, no zero page.
//  * Double-buffered 38 KiB stages (2 x 78 KiB per CU), one barrier per
//    stage; the next stage's DMA (possibly the next tile's first) is issued
//    after that barrier and lands under the current stage's MFMAs.
//  * Epilogue without LDS: v_permlane32_swap gives each lane 8 consecutive
//    output channels of one voxel, so every store / residual / mask access
//    is 16 contiguous bytes.
#pragma once
#include "conv_common.h"

namespace vsrk_conv {

struct K3Args {
  View x, y, res, msk;
  const bf16* w;
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
};

constexpr int K3_R = 4;                  // output rows per wave
constexpr int K3_NW = 4;                 // waves per workgroup
constexpr int K3_FTH = K3_R * K3_NW;     // tile rows (16)
constexpr int K3_HR = K3_FTH + 2;        // halo rows (18)
constexpr int K3_HC = TW + 2;            // halo columns (34)
constexpr int K3_NV = K3_HR * K3_HC;     // halo entries per plane (612)
constexpr int K3_NVP = 640;              // padded to whole 64-entry DMA pieces
constexpr int K3_AI = 2 * K3_NVP / 64;   // A DMA wave-instructions per stage (20)
constexpr int K3_ABYTES = 2 * K3_NVP * 16;

template <int NT>
struct K3Geom {
  static constexpr int BENT = 9 * NT;                   // B entries per plane
  static constexpr int BI = (2 * BENT + 63) / 64;       // B DMA wave-instructions per stage
  static constexpr int BBYTES = BI * 1024;
  static constexpr int SLOT = K3_ABYTES + BBYTES;
  static constexpr int NAW = (K3_AI + K3_NW - 1) / K3_NW;
  static constexpr int NBW = (BI + K3_NW - 1) / K3_NW;
  static size_t lds_bytes(int cout_pad, int cin_pad, bool pro) {
    return 2 * (size_t)SLOT + (size_t)cout_pad * 4 + (pro ? 2 * (size_t)cin_pad * 4 : 0);
  }
};

constexpr int kK3NotEligible = -1001;
// persistent grid: two workgroups per CU (or the vsrk_conv_set_grid_cap test cap)
int k3_grid(int64_t ntiles);

// per-family launchers (one translation unit each): VSRK_OK, an error status
// or kK3NotEligible
int k3_n32(const K3Args& a, bool pro, hipStream_t s);          // conv_k3_n32.hip
int k3_n64(const K3Args& a, bool pro, hipStream_t s);          // conv_k3_n64.hip
int k3_n64_sub(const K3Args& a, int xs, int ys, hipStream_t s);  // conv_k3_n64_sub.hip

}  // namespace vsrk_conv

#ifdef VSRK_K3_KERNEL_TU
namespace {
using namespace vsrk_conv;

typedef int32_t i32x4 __attribute__((ext_vector_type(4)));

// raw buffer resource over [base, base + 2 GiB): an offset at or beyond
// 0x7FFFFFF0 reads as zeros (the padding convention of this kernel)
__device__ __forceinline__ i32x4 make_rsrc(const void* base) {
  const uint64_t b = (uint64_t)base;
  i32x4 r;
  r[0] = __builtin_amdgcn_readfirstlane((int)(uint32_t)b);
  r[1] = __builtin_amdgcn_readfirstlane((int)(uint32_t)(b >> 32) & 0xffff);
  r[2] = 0x7FFFFFF0;
  r[3] = 0x00020000;
  return r;
}
constexpr uint32_t K3_OOB = 0x80000000u;

// lane l's 16 bytes from rsrc[voff + soff] land at LDS byte lds_base + 16 l.
// Inline asm so hipcc neither drains it before unrelated LDS reads nor
// schedules around it; M0 is saved and restored inside the statement.
__device__ __forceinline__ void bdma16(i32x4 rsrc, uint32_t voff, uint32_t soff, uint32_t lds_base) {
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %4\n\t"
      "s_nop 0\n\t"
      "buffer_load_dwordx4 %1, %2, %3 offen lds\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(rsrc), "s"(__builtin_amdgcn_readfirstlane(soff)),
        "s"(__builtin_amdgcn_readfirstlane(lds_base)));
}

// N LDS-DMA pieces in one statement (one M0 save / restore): piece k loads
// rsrc[v[k] + soff] into LDS at m0_base + k * STEP.
template <int N, int STEP>
__device__ __forceinline__ void bdma16xN(i32x4 rsrc, const uint32_t* v, uint32_t soff, uint32_t m0_base) {
  static_assert(N >= 1 && N <= 5, "1..5 pieces");
  unsigned keep;
  const uint32_t so = __builtin_amdgcn_readfirstlane(soff), mb = __builtin_amdgcn_readfirstlane(m0_base);
  if constexpr (N == 1) {
    asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %4\n\ts_nop 0\n\t"
      "buffer_load_dwordx4 %1, %2, %3 offen lds\n\t"
      "s_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(v[0]), "s"(rsrc), "s"(so), "s"(mb), "n"(STEP));
  }
  if constexpr (N == 2) {
    asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %5\n\ts_nop 0\n\t"
      "buffer_load_dwordx4 %1, %3, %4 offen lds\n\t"
      "s_add_u32 m0, m0, %6\n\ts_nop 0\n\t"
      "buffer_load_dwordx4 %2, %3, %4 offen lds\n\t"
      "s_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(v[0]), "v"(v[1]), "s"(rsrc), "s"(so), "s"(mb), "n"(STEP));
  }
  if constexpr (N == 3) {
    asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %6\n\ts_nop 0\n\t"
      "buffer_load_dwordx4 %1, %4, %5 offen lds\n\t"
      "s_add_u32 m0, m0, %7\n\ts_nop 0\n\t"
      "buffer_load_dwordx4 %2, %4, %5 offen lds\n\t"
      "s_add_u32 m0, m0, %7\n\ts_nop 0\n\t"
      "buffer_load_dwordx4 %3, %4, %5 offen lds\n\t"
      "s_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(v[0]), "v"(v[1]), "v"(v[2]), "s"(rsrc), "s"(so), "s"(mb), "n"(STEP));
  }
  if constexpr (N == 4) {
    asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %7\n\ts_nop 0\n\t"
      "buffer_load_dwordx4 %1, %5, %6 offen lds\n\t"
      "s_add_u32 m0, m0, %8\n\ts_nop 0\n\t"
      "buffer_load_dwordx4 %2, %5, %6 offen lds\n\t"
      "s_add_u32 m0, m0, %8\n\ts_nop 0\n\t"
      "buffer_load_dwordx4 %3, %5, %6 offen lds\n\t"
      "s_add_u32 m0, m0, %8\n\ts_nop 0\n\t"
      "buffer_load_dwordx4 %4, %5, %6 offen lds\n\t"
      "s_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]), "s"(rsrc), "s"(so), "s"(mb), "n"(STEP));
  }
  if constexpr (N == 5) {
    asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %8\n\ts_nop 0\n\t"
      "buffer_load_dwordx4 %1, %6, %7 offen lds\n\t"
      "s_add_u32 m0, m0, %9\n\ts_nop 0\n\t"
      "buffer_load_dwordx4 %2, %6, %7 offen lds\n\t"
      "s_add_u32 m0, m0, %9\n\ts_nop 0\n\t"
      "buffer_load_dwordx4 %3, %6, %7 offen lds\n\t"
      "s_add_u32 m0, m0, %9\n\ts_nop 0\n\t"
      "buffer_load_dwordx4 %4, %6, %7 offen lds\n\t"
      "s_add_u32 m0, m0, %9\n\ts_nop 0\n\t"
      "buffer_load_dwordx4 %5, %6, %7 offen lds\n\t"
      "s_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]), "v"(v[4]), "s"(rsrc), "s"(so), "s"(mb), "n"(STEP));
  }
}

// 8 consecutive channels per lane after the permlane32 swap
__device__ __forceinline__ void unpack8(uint4 v, float* f) { Chunk<bf16>::unpack(v, f); }

template <int NT, int XS, int YS, int PRO>
__global__ __launch_bounds__(K3_NW * 64, 2) void conv_k3_kernel(K3Args a) {
  using G = K3Geom<NT>;
  constexpr int NS = NT / 32;
  constexpr int SLOT = G::SLOT, NAW = G::NAW, NBW = G::NBW, BI = G::BI, BENT = G::BENT;
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int tid = threadIdx.x, lane = tid & 63, l32 = lane & 31, hf = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  float* lbias = reinterpret_cast<float*>(lds + 2 * SLOT);
  float* lsc = lbias + a.cout_pad;
  float* lsh = lsc + a.cin_pad;
  for (int i = tid; i < a.cout_pad; i += K3_NW * 64) {
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
  if constexpr (PRO) stage_prologue(lsc, lsh, a.prologue, a.pro_scale, a.pro_shift, a.cin, a.cin_pad, tid, K3_NW * 64);

  // B DMA roles, fixed: instruction j = wave + 4k holds entries j*64 + lane
  // -> (plane, tap, co) of the packed weight [tap][cout_pad][cin_pad]; waves
  // below BI % 4 issue NBW pieces, the others NBW - 1
  uint32_t b_off[NBW];
#pragma unroll
  for (int k = 0; k < NBW; ++k) {
    const int e = (wave + K3_NW * k) * 64 + lane;
    const int pl = e / BENT, rem = e - (e / BENT) * BENT;
    const int tap = rem / NT, co = rem - (rem / NT) * NT;
    b_off[k] = pl < 2 ? (uint32_t)(2 * ((tap * a.cout_pad + co) * a.cin_pad + 8 * pl)) : K3_OOB;
  }
  const bool b_full = (BI % K3_NW) == 0 || wave < (BI % K3_NW);
  const i32x4 wrsrc = make_rsrc(a.w);
  const uint32_t lds0 = lds_addr(lds);
  const uint32_t a_rd = (uint32_t)(((hf * K3_NVP) + wave * K3_R * K3_HC + l32) * 16);
  const uint32_t b_rd = (uint32_t)(K3_ABYTES + ((hf * BENT) + l32) * 16);
  const int xr = XS ? a.x.r : 1;
  const int64_t xsh = (int64_t)xr * a.x.sh, xsw = (int64_t)xr * a.x.sw;
  const int nchunk = a.cin / 16;

  // tiles of this workgroup: XCD group xg owns a contiguous range
  const int Gd = gridDim.x;
  const int xg = blockIdx.x & 7, jx = blockIdx.x >> 3;
  const int gx = (Gd >> 3) + (xg < (Gd & 7) ? 1 : 0);
  const int cx = xg * (Gd >> 3) + min(xg, Gd & 7);
  const int t_lo = (int)((int64_t)a.ntiles * cx / Gd);
  const int t_hi = (int)((int64_t)a.ntiles * (cx + gx) / Gd);

  // per-tile A state: buffer resource at the tile's halo origin (scalar) and
  // each lane's byte offset per A instruction, out of range where the halo
  // leaves the image (the DMA then writes zeros)
  uint32_t voff[NAW];
  i32x4 xrsrc;
  int nb = 0, dz = 0, h0 = 0, w0 = 0, n0 = 0, kd_lo = 0, nst = 1;
  auto set_tile = [&](int t) __attribute__((always_inline)) {
    const int tn = t % a.ntn;
    int tm = t / a.ntn;
    const int tw_i = tm % a.tiles_w;
    tm /= a.tiles_w;
    const int th_i = tm % a.tiles_h;
    tm /= a.tiles_h;
    dz = tm % a.y.d;
    nb = tm / a.y.d;
    h0 = th_i * K3_FTH;
    w0 = tw_i * TW;
    n0 = tn * NT;
    kd_lo = max(0, a.pd - dz);
    nst = max(1, min(a.kd, a.x.d + a.pd - dz) - kd_lo) * nchunk;
    const int hb = h0 - a.ph, wb = w0 - a.pw;
    xrsrc = make_rsrc(a.x.ptr + 2 * (nb * a.x.sn + (int64_t)hb * xsh + (int64_t)wb * xsw));
#pragma unroll
    for (int k = 0; k < NAW; ++k) {
      const int i = wave + K3_NW * k;
      const int v = (i % (K3_NVP / 64)) * 64 + lane;
      const int hh = v / K3_HC, ww = v - (v / K3_HC) * K3_HC;
      const bool ok = v < K3_NV && hb + hh >= 0 && hb + hh < a.x.h && wb + ww >= 0 && wb + ww < a.x.w;
      voff[k] = ok ? (uint32_t)(2 * ((int64_t)hh * xsh + (int64_t)ww * xsw + 8 * (i / (K3_NVP / 64)))) : K3_OOB;
    }
  };
  // issue stage s of the current tile into `slot`; returns its channel base
  auto issue = [&](int s, int slot) __attribute__((always_inline)) -> int {
    const int kdi = kd_lo + s / nchunk;
    const int c0 = (s - (s / nchunk) * nchunk) * 16;
    int64_t xo = (int64_t)(dz + kdi - a.pd) * a.x.sd;
    if constexpr (XS) {
      const int sub = c0 / a.x.cphys, cc = c0 - sub * a.x.cphys;
      const int si = sub / xr, sj = sub - si * xr;
      xo += (int64_t)si * a.x.sh + (int64_t)sj * a.x.sw + cc;
    } else {
      xo += c0;
    }
    const uint32_t soa = (uint32_t)(2 * xo);
    const uint32_t sob = (uint32_t)(2 * (((int64_t)kdi * 9 * a.cout_pad + n0) * a.cin_pad + c0));
    const uint32_t base = lds0 + slot * SLOT + wave * 1024;
    static_assert(NAW == 5 && K3_AI == 20, "A staging: five pieces per wave");
    bdma16xN<5, K3_NW * 1024>(xrsrc, voff, soa, base);
    if (b_full) bdma16xN<NBW, K3_NW * 1024>(wrsrc, b_off, sob, base + K3_ABYTES);
    else bdma16xN<NBW - 1, K3_NW * 1024>(wrsrc, b_off, sob, base + K3_ABYTES);
    return c0;
  };

  f32x16 acc[K3_R][NS];
#pragma unroll
  for (int r = 0; r < K3_R; ++r)
#pragma unroll
    for (int n = 0; n < NS; ++n)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[r][n][i] = 0.f;

  const float aslope = a.act == VSRK_ACT_PRELU ? *a.act_param : 0.f;
  const float mslope = a.mask_slope ? *a.mask_slope : 0.f;
  const bool use_res = a.has_res, use_msk = a.has_mask, use_acc = a.accumulate, act = a.act != VSRK_ACT_NONE;
  const bool relu_in = (a.prologue & VSRK_PRO_RELU) != 0;
  const int yr = YS ? a.y.r : 1;

  // ---- main loop: one iteration per stage ----
  // Stage s's DMA was issued one iteration earlier into `slot`.  Wait for
  // this wave's part, apply the prologue to it, barrier (every wave's part
  // landed; every wave is done reading slot ^ 1), issue stage s + 1 (maybe
  // the next tile's first) into slot ^ 1, then the MFMAs of stage s, then the
  // tile's epilogue after its last stage.
  int t = t_lo + jx;
  if (t >= t_hi) return;
  set_tile(t);
  __syncthreads();  // bias / prologue tables
  int s = 0, slot = 0;
  int c0 = issue(0, 0);
  while (true) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's DMA of stage s landed
    if constexpr (PRO) {
      if (a.prologue) {
#pragma unroll
        for (int k = 0; k < NAW; ++k) {
          const int i = wave + K3_NW * k;
          if (i < K3_AI && voff[k] != K3_OOB) {
            uint4* p = reinterpret_cast<uint4*>(lds + slot * SLOT + i * 1024 + lane * 16);
            *p = prologue_lds<bf16>(*p, c0 + 8 * (i / (K3_NVP / 64)), relu_in, lsc, lsh);
          }
        }
      }
    }
    __syncthreads();
#ifdef VSRK_K3_DEBUG_DUMP
    if (blockIdx.x == 0 && t == t_lo + jx && s == 0) {  // probe build only: the first landed stage
      for (int i = tid; i < SLOT / 16; i += K3_NW * 64)
        reinterpret_cast<uint4*>(VSRK_K3_DEBUG_DUMP)[i] = reinterpret_cast<const uint4*>(lds)[i];
    }
#endif
    const bool last = s + 1 >= nst;
    // epilogue coordinates of the current tile (set_tile below moves on)
    const int e_nb = nb, e_dz = dz, e_h0 = h0, e_w0 = w0, e_n0 = n0;
    const int tn = t + gx;
    const bool more = !last || tn < t_hi;
    int c0n = 0;
    if (more) {
      if (last) set_tile(tn);
      c0n = issue(last ? 0 : s + 1, slot ^ 1);
    }
    // MFMAs of stage s: per kw, 6 halo-row A fragments and 3 x NS B fragments
    // (raised issue priority: the other workgroup's wave on this SIMD takes
    // the gaps for its DMA / epilogue instructions)
    __builtin_amdgcn_s_setprio(1);
    {
      const char* sA = lds + slot * SLOT;
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {
        uint4 af[K3_R + 2], bw[3][NS];
#pragma unroll
        for (int rr = 0; rr < K3_R + 2; ++rr)
          af[rr] = *reinterpret_cast<const uint4*>(sA + a_rd + (rr * K3_HC + kw) * 16);
#pragma unroll
        for (int kh = 0; kh < 3; ++kh)
#pragma unroll
          for (int ns = 0; ns < NS; ++ns)
            bw[kh][ns] = *reinterpret_cast<const uint4*>(sA + b_rd + ((kh * 3 + kw) * NT + ns * 32) * 16);
#pragma unroll
        for (int kh = 0; kh < 3; ++kh)
#pragma unroll
          for (int r = 0; r < K3_R; ++r)
#pragma unroll
            for (int ns = 0; ns < NS; ++ns) mma<bf16>(acc[r][ns], bw[kh][ns], af[r + kh]);
      }
    }
    __builtin_amdgcn_s_setprio(0);
    if (last) {
      // Epilogue.  Per register: bias (pre-scaled), out_scale, activation
      // (register 4g + e is channel 8g + 4hf + e); then v_permlane32_swap
      // vdst, src -- it exchanges lanes 32-63 of vdst with lanes 0-31 of src --
      // with vdst = group 2q, src = group 2q+1: the low half ends up with
      // channels 16q .. 16q+7 (own 2q | upper's 2q), the high half with
      // 16q+8 .. 16q+15 (lower's 2q+1 | own 2q+1), so each lane finishes 8
      // consecutive channels of its voxel with 16-byte accesses at a per-row
      // base + immediate offsets.  (Inline asm: hipcc's builtin lowering fed
      // both operands from one register here.)
      const int wo = e_w0 + l32;
      const bool ok_w = wo < a.y.w;
      int64_t ybase, rbase = 0, mbase = 0;
      if constexpr (YS) {  // sub-pixel store: the tile's 64 channels are one sub-pixel (cphys % 64 == 0)
        const int sub = e_n0 / a.y.cphys, cc0 = e_n0 - sub * a.y.cphys;
        const int si = sub / yr, sj = sub - si * yr;
        ybase = e_nb * a.y.sn + (int64_t)e_dz * a.y.sd + (int64_t)si * a.y.sh + (int64_t)(wo * yr + sj) * a.y.sw + cc0;
      } else {
        ybase = e_nb * a.y.sn + (int64_t)e_dz * a.y.sd + (int64_t)wo * a.y.sw + e_n0;
        rbase = e_nb * a.res.sn + (int64_t)e_dz * a.res.sd + (int64_t)wo * a.res.sw + e_n0;
        mbase = e_nb * a.msk.sn + (int64_t)e_dz * a.msk.sd + (int64_t)wo * a.msk.sw + e_n0;
      }
      const int64_t ysh = (int64_t)yr * a.y.sh;
#pragma unroll
      for (int r = 0; r < K3_R; ++r) {
        const int ho = e_h0 + wave * K3_R + r;
        if (ho >= a.y.h) {  // wave-uniform
#pragma unroll
          for (int ns = 0; ns < NS; ++ns)
#pragma unroll
            for (int i = 0; i < 16; ++i) acc[r][ns][i] = 0.f;
          continue;
        }
        bf16* yrow = reinterpret_cast<bf16*>(a.y.ptr) + ybase + ho * ysh + hf * 8;
        const bf16* rrow = reinterpret_cast<const bf16*>(a.res.ptr) + rbase + (int64_t)ho * a.res.sh + hf * 8;
        const bf16* mrow = reinterpret_cast<const bf16*>(a.msk.ptr) + mbase + (int64_t)ho * a.msk.sh + hf * 8;
#pragma unroll
        for (int ns = 0; ns < NS; ++ns) {
          f32x16& A = acc[r][ns];
          float v[16];
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            const float4 bq = *reinterpret_cast<const float4*>(lbias + e_n0 + ns * 32 + 8 * g + 4 * hf);
            const float bb[4] = {bq.x, bq.y, bq.z, bq.w};
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const float tq = fmaf(A[4 * g + e], a.out_scale, bb[e]);
              v[4 * g + e] = act ? act_apply(a.act, tq, aslope) : tq;
            }
            }
          asm volatile(
              "s_nop 1\n\t"
              "v_permlane32_swap_b32 %0, %4\n\tv_permlane32_swap_b32 %1, %5\n\t"
              "v_permlane32_swap_b32 %2, %6\n\tv_permlane32_swap_b32 %3, %7\n\t"
              "v_permlane32_swap_b32 %8, %12\n\tv_permlane32_swap_b32 %9, %13\n\t"
              "v_permlane32_swap_b32 %10, %14\n\tv_permlane32_swap_b32 %11, %15"
              : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]), "+v"(v[4]), "+v"(v[5]), "+v"(v[6]), "+v"(v[7]),
                "+v"(v[8]), "+v"(v[9]), "+v"(v[10]), "+v"(v[11]), "+v"(v[12]), "+v"(v[13]), "+v"(v[14]),
                "+v"(v[15]));
#pragma unroll
          for (int q = 0; q < 2; ++q) {
            const int cl = ns * 32 + q * 16;  // channel offset within the tile (lane half adds 8)
            const bool ok = ok_w && e_n0 + cl + hf * 8 < a.cout;
            float* tv = v + q * 8;
            if (use_msk) {
              float m[8];
              unpack8(ok ? *reinterpret_cast<const uint4*>(mrow + cl) : make_uint4(0, 0, 0, 0), m);
#pragma unroll
              for (int e = 0; e < 8; ++e) tv[e] = mask_apply(m[e], tv[e], mslope);
            }
            if (use_res) {
              float rr[8];
              unpack8(ok ? *reinterpret_cast<const uint4*>(rrow + cl) : make_uint4(0, 0, 0, 0), rr);
#pragma unroll
              for (int e = 0; e < 8; ++e) tv[e] += rr[e];
            }
            if (use_acc) {
              float o[8];
              unpack8(ok ? *reinterpret_cast<const uint4*>(yrow + cl) : make_uint4(0, 0, 0, 0), o);
#pragma unroll
              for (int e = 0; e < 8; ++e) tv[e] += o[e];
            }
            if (ok) *reinterpret_cast<uint4*>(yrow + cl) = Chunk<bf16>::pack(tv);
          }
#pragma unroll
          for (int i = 0; i < 16; ++i) A[i] = 0.f;
        }
      }
    }
    if (!more) break;
    if (last) t = tn;
    s = last ? 0 : s + 1;
    slot ^= 1;
    c0 = c0n;
  }
}

template <int NT, int XS, int YS, int PRO>
int launch_k3(K3Args a, hipStream_t s) {
  using G = K3Geom<NT>;
  a.tiles_h = ceil_div(a.y.h, K3_FTH);
  const int64_t ntiles = (int64_t)a.y.n * a.y.d * a.tiles_h * a.tiles_w * a.ntn;
  VSRK_CHECK(ntiles < (1ll << 31), "conv_fwd(k3): too many tiles");
  a.ntiles = (int)ntiles;
  if (a.ntiles == 0) return VSRK_OK;
  const size_t lds = G::lds_bytes(a.cout_pad, a.cin_pad, PRO);
  if (lds > 80 * 1024) return kK3NotEligible;  // two workgroups per CU
  auto kern = conv_k3_kernel<NT, XS, YS, PRO>;
  (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  const int grid = k3_grid(ntiles);
  kern<<<grid, K3_NW * 64, lds, s>>>(a);
  VSRK_LAUNCH_CHECK("conv_fwd(k3)");
  return VSRK_OK;
}
}  // namespace
#endif  // VSRK_K3_KERNEL_TU
