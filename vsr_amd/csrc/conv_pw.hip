// Pointwise (1x1x1) convolution on CDNA4 for 16-bit (bf16 / fp16) channels-last activations:
// forward / data-gradient (pw_fwd) and weight gradient (pw_wgrad).
//
// DUF's dense-unit bottlenecks (BN3d-ReLU-Conv1x1x1, duf_net.py:198-200,
// cin = cout = 64..224 at up to 7 x 128 x 128 voxels per sample) and its
// 256-channel heads (duf_net.py:40-49) move (cin + cout) * 2 bytes per voxel
// for 2 * cin * cout flops: <= 256 flop/B at cin = cout <= 256, under the
// MI355X ridge (2.5 PF / 8 TB/s ~ 312 flop/B).  They are HBM-bound, so the
// design goal is ONE pass over x and y at full HBM rate (the 3x3 tile kernels
// re-read x once per 128-channel output tile and stage it through LDS with a
// barrier per tile):
//
//  * pw_fwd: the weight chunk (<= 256 x 256 bf16 = 128 KiB) is staged into LDS
//    once per workgroup.  Each wave then streams its own 32*M-voxel tiles
//    straight from HBM into registers as the MFMA B operand (x^T: lane l holds
//    voxel l&31, 8 channels), applies the BatchNorm+ReLU prologue in
//    registers, runs all output-channel blocks against the resident weights
//    (A operand, one conflict-free ds_read_b128 per MFMA) and stores: no
//    barrier after the weight load, the next tile's loads in flight during
//    the current tile's MFMAs and stores.
//  * pw_wgrad: dW = dY^T X reduces over voxels.  Each workgroup owns a
//    contiguous voxel range and a (cout chunk x cin chunk) of <= 256 x 256,
//    stages 64 voxels of dY and X per step (register-staged double buffer,
//    planar 64-byte rows read transposed with ds_read_b64_tr_b16), and writes
//    one fp32 partial slab; pw_wgrad_reduce sums the slabs in split order
//    (deterministic).  One pass over dY and X per cin/cout chunk.
#include <algorithm>
#include <cstdlib>
#include <type_traits>
#include "conv_common.h"

int vsrk_g_pw_mode = -1;  // -1: from VSRK_CONV_PW (default on), 0 off, 1 on

namespace {
using namespace vsrk_conv;

constexpr int PW_THR = 256;  // 4 waves, one per SIMD
#ifndef PW_EIN_EARLY
#define PW_EIN_EARLY 1
#endif
enum { EIN_GEN = 1, EIN_ACC = 2, EIN_PB = 3, EIN_PBACC = 4 };  // staged kernel store-pass forms
constexpr int PW_KP = 64;    // wgrad voxels per stage
#ifndef PW_NT
#define PW_NT 2  // non-temporal output stores of the staged kernel (DUF 75.8 -> 75.4 ms, profiles/r4_pw_nt_ab.txt); 0 for A/B
#endif
#ifndef PW_BXPRE
#define PW_BXPRE 1  // fused BN-backward reduce: BN input rows loaded ahead of the MFMAs (0: in the store pass)
#endif

static bool pw_enabled() {
  if (vsrk_g_pw_mode < 0) {
    const char* e = getenv("VSRK_CONV_PW");
    vsrk_g_pw_mode = (e && e[0] == '0') ? 0 : 1;
  }
  return vsrk_g_pw_mode == 1;
}

static int pw_num_cus() {
  static int n = 0;
  if (n == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
  }
  return n;
}

// Division by a launch constant d (dividends < 2^31), branch-free:
// q = (x * mul) >> p with p = 31 + ceil(log2 d), mul = ceil(2^p / d) < 2^32.
struct FastDiv {
  uint32_t d, mul, p;
};
static FastDiv make_fastdiv(int d) {
  int l = 0;
  while ((1u << l) < (uint32_t)d) ++l;
  const uint32_t p = 31 + l;
  return FastDiv{(uint32_t)d, (uint32_t)(((1ull << p) + (uint64_t)d - 1) / (uint64_t)d), p};
}
__device__ __forceinline__ uint32_t fdiv(uint32_t x, const FastDiv& f) {
  return (uint32_t)(((uint64_t)x * f.mul) >> f.p);
}

// Raw buffer resource over [base, base + 2 GiB) (wave-uniform base): offsets
// at or beyond 0x7FFFFFF0 read as zero and drop stores -- the out-of-range
// voxels and channels of a tile, without branches.
typedef __amdgpu_buffer_rsrc_t Rsrc;
constexpr uint32_t PW_OOB = 0x80000000u;
__device__ __forceinline__ Rsrc rsrc_at(const void* base) {
  const uint64_t b = (uint64_t)base;
  const uint64_t u = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(b >> 32)) << 32) |
                     (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)b);
  return __builtin_amdgcn_make_buffer_rsrc((void*)u, 0, 0x7FFFFFF0, 0x00020000);
}
typedef int v4i_t __attribute__((ext_vector_type(4)));
// LDS access by 32-bit byte address (plain vector types: HIP's uint4 class has
// no address-space-qualified copy)
typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2_t __attribute__((ext_vector_type(2)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 lds_ld16(uint32_t addr) {
  return __builtin_bit_cast(uint4, *(const __attribute__((address_space(3))) u32x4_t*)(size_t)addr);
}
__device__ __forceinline__ float4 lds_ldf4(uint32_t addr) {
  return __builtin_bit_cast(float4, *(const __attribute__((address_space(3))) f32x4_t*)(size_t)addr);
}
__device__ __forceinline__ void lds_st8(uint32_t addr, uint2 v) {
  *(__attribute__((address_space(3))) u32x2_t*)(size_t)addr = __builtin_bit_cast(u32x2_t, v);
}
typedef int v2i_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint4 bload16(Rsrc r, uint32_t off) {
  return __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 0));
}
__device__ __forceinline__ uint2 bload8(Rsrc r, uint32_t off) {
  return __builtin_bit_cast(uint2, __builtin_amdgcn_raw_buffer_load_b64(r, (int)off, 0, 0));
}
__device__ __forceinline__ void bstore8(Rsrc r, uint32_t off, uint2 v) {
  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(v2i_t, v), r, (int)off, 0, 0);
}

template <typename H>
__device__ __forceinline__ uint4 h8_affine(uint4 v, const float4& s0, const float4& s1, const float4& h0,
                                          const float4& h1, bool relu) {
  float f[8];
  Chunk<H>::unpack(v, f);
  const float sc[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
  const float sh[8] = {h0.x, h0.y, h0.z, h0.w, h1.x, h1.y, h1.z, h1.w};
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const float t = fmaf(f[e], sc[e], sh[e]);
    f[e] = relu ? fmaxf(t, 0.f) : t;
  }
  return Chunk<H>::pack(f);
}

struct PwArgs {  // 16-bit tensors of one type H (bf16 / fp16)
  const void* x;
  void* y;
  const void* msk;
  const void* w;  // packed [round_up(cout,128)][ci_pad] (vsrk_conv_pack_weight)
  const float* bias;
  const float* pro_scale;
  const float* pro_shift;
  const float* mask_slope;
  const float* act_param;                 // PReLU slope (device scalar)
  // fused per-channel reduction of the stored output (RED 1: BatchNorm
  // statistics sum y, sum y^2; RED 2: BatchNorm+ReLU backward sum dy',
  // sum dy' xhat with dy' = y * (bnx * scale + shift > 0), xhat =
  // (bnx - mean) * invstd): per-lane partials, slab [block][wave][lane][16]
  const void* bnx;
  int64_t bsn, bsw;
  const float *bsc, *bsh, *bmu, *bis;
  float* red_ws;
  // BNB: the conv input is a BatchNorm+ReLU backward applied on the fly
  // (x = dz, the BN's output gradient; qx = the BN's input): the applied
  // gradient feeds the MFMAs and is stored to xo (the weight gradient's dY)
  const void* qx;
  void* xo;
  int64_t qsn, qsw, osn, osw;
  const float *qsh, *qmu, *qis, *qgm, *qsdy, *qsdyx;
  float qinv_count;
  int64_t xsn, xsw, ysn, ysw, msn, msw;  // element strides
  int nvox, dhw;
  FastDiv fd;                             // division by dhw
  int cin, cout, ci_pad, co_rows;
  int prologue, act, accumulate, has_mask;
  // PBWD (EIN form): the PReLU backward of the output's consumer applied
  // after the accumulate, on output channels >= pm_lo (a consumer that
  // owns the tail slice of a concat gradient): dy' = (conv [+ dy]) *
  // (msk > 0 ? 1 : slope), msk = that PReLU's output; the slope gradient
  // sum_{msk<0} dy' msk as per-lane partials, slab [block y][block x][wave][lane]
  int pbwd, pm_lo;
  double* slope_part;  // [block y][block x][wave] partials of the slope gradient
  float out_scale;
  int ntiles;  // tiles of 32*M voxels
  int ablate;  // A/B knob (VSRK_PW_ABLATE): 1 = no stores, 2 = no MFMA, 4 = no loads (staged)
};

// Byte offsets of a tile's voxels relative to the sample that holds its first
// voxel: lane voxel v = v0 + k (k < 32*M) -> (n - n0) * sn + r * sw.
struct TileBase {
  int n0, r0;
};
__device__ __forceinline__ TileBase tile_base(int v0, const FastDiv& fd) {
  const int n0 = (int)fdiv((uint32_t)v0, fd);
  return {n0, v0 - n0 * (int)fd.d};
}
__device__ __forceinline__ uint32_t lane_off(const TileBase& tb, int k, int v, int nvox, const FastDiv& fd,
                                             int64_t sn, int64_t sw) {
  // the host guarantees these offsets fit 31 bits: 32-bit arithmetic
  const uint32_t rel = (uint32_t)(tb.r0 + k);
  const uint32_t dn = fdiv(rel, fd);
  const uint32_t r = rel - dn * fd.d;
  const uint32_t off = 2u * (dn * (uint32_t)sn + r * (uint32_t)sw);
  return v < nvox ? off : PW_OOB;
}

// ---------------------------------------------------------------------------
// forward / data gradient: y[v][co] = epi(sum_ci W[co][ci] * pro(x[v][ci]))
// NCB output blocks of 32 channels per workgroup (blockIdx.y picks the chunk),
// KS = 2*NCB k-steps of 16 input channels (cin_pad == 32*NCB), M tiles of 32
// voxels per wave step.
// ---------------------------------------------------------------------------
template <int NCB, int M, bool PRO, bool EIN, typename H>
__global__ __launch_bounds__(PW_THR, 1) void pw_fwd_kernel(PwArgs a) {
  const H* aX = reinterpret_cast<const H*>(a.x);
  H* aY = reinterpret_cast<H*>(a.y);
  const H* aM = reinterpret_cast<const H*>(a.msk);
  const H* aW = reinterpret_cast<const H*>(a.w);
  constexpr int KS = 2 * NCB;
  constexpr int COP = 32 * NCB;
  constexpr int CIP = 16 * KS;
  extern __shared__ __attribute__((aligned(16))) char lds[];
  char* lw = lds;                                        // [KS][2][COP] x 16 B
  float* lsc = reinterpret_cast<float*>(lds + KS * 2 * COP * 16);  // [CIP]
  float* lsh = lsc + CIP;                                // [CIP]
  float* lb = lsh + CIP;                                 // [COP]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int hf = lane >> 5, col = lane & 31;
  const int co0 = blockIdx.y * COP;

  for (int i = tid; i < KS * 2 * COP; i += PW_THR) {
    const int co = i % COP, t = i / COP, h = t & 1, s = t >> 1;
    const int ci = 16 * s + 8 * h;
    uint4 v = make_uint4(0, 0, 0, 0);
    if (ci < a.ci_pad && co0 + co < a.co_rows)
      v = *reinterpret_cast<const uint4*>(aW + (int64_t)(co0 + co) * a.ci_pad + ci);
    *reinterpret_cast<uint4*>(lw + i * 16) = v;
  }
  if (PRO) stage_prologue(lsc, lsh, a.prologue, a.pro_scale, a.pro_shift, a.cin, CIP, tid, PW_THR);
  for (int i = tid; i < COP; i += PW_THR) lb[i] = (a.bias && co0 + i < a.cout) ? a.bias[co0 + i] : 0.f;
  __syncthreads();

  const bool relu_in = (a.prologue & VSRK_PRO_RELU) != 0;
  const float mslope = a.mask_slope ? *a.mask_slope : 0.f;
  const int nwaves = gridDim.x * (PW_THR / 64);
  const int wv = __builtin_amdgcn_readfirstlane(wave);

  // B operand of k-step s: 8 channels 16s + 8hf of voxel col (zero outside)
  auto load = [&](int tile, uint4 (&b)[M][KS]) __attribute__((always_inline)) {
    const int v0 = tile * 32 * M;
    const TileBase tb = tile_base(v0, a.fd);
    const Rsrc r = rsrc_at(aX + (int64_t)tb.n0 * a.xsn);
#pragma unroll
    for (int m = 0; m < M; ++m) {
      const uint32_t off = lane_off(tb, m * 32 + col, v0 + m * 32 + col, a.nvox, a.fd, a.xsn, a.xsw);
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        const int c = 16 * s + 8 * hf;
        b[m][s] = bload16(r, c < a.cin ? off + 2 * c : PW_OOB);
      }
    }
  };

  uint4 bc[M][KS];
  int t = blockIdx.x * (PW_THR / 64) + wv;
  if (t < a.ntiles) load(t, bc);
  while (t < a.ntiles) {
    const int tn = t + nwaves;
    const int v0 = t * 32 * M;
    const TileBase tb = tile_base(v0, a.fd);
    const Rsrc ry = rsrc_at(aY + (int64_t)tb.n0 * a.ysn);
    // epilogue inputs of this tile first, then the next tile's operands: the
    // epilogue's wait (vmcnt) then leaves the prefetch in flight
    uint2 ein[EIN ? M : 1][NCB][4];
    if constexpr (EIN) {
      const Rsrc rm = a.has_mask ? rsrc_at(aM + (int64_t)tb.n0 * a.msn) : ry;
#pragma unroll
      for (int m = 0; m < M; ++m) {
        const uint32_t off = a.has_mask
                                 ? lane_off(tb, m * 32 + col, v0 + m * 32 + col, a.nvox, a.fd, a.msn, a.msw)
                                 : lane_off(tb, m * 32 + col, v0 + m * 32 + col, a.nvox, a.fd, a.ysn, a.ysw);
#pragma unroll
        for (int cb = 0; cb < NCB; ++cb)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int gco = co0 + cb * 32 + 8 * j + 4 * hf;
            ein[m][cb][j] = bload8(rm, gco < a.cout ? off + 2 * gco : PW_OOB);
          }
      }
    }
    uint4 bn[M][KS];
    if (tn < a.ntiles) load(tn, bn);

    f32x16 acc[M][NCB];
#pragma unroll
    for (int m = 0; m < M; ++m)
#pragma unroll
      for (int cb = 0; cb < NCB; ++cb)
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[m][cb][i] = 0.f;
    if (!(a.ablate & 2)) {
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        if (PRO) {
          const int c = 16 * s + 8 * hf;
          const float4 s0 = *reinterpret_cast<const float4*>(lsc + c), s1 = *reinterpret_cast<const float4*>(lsc + c + 4);
          const float4 h0 = *reinterpret_cast<const float4*>(lsh + c), h1 = *reinterpret_cast<const float4*>(lsh + c + 4);
#pragma unroll
          for (int m = 0; m < M; ++m) bc[m][s] = h8_affine<H>(bc[m][s], s0, s1, h0, h1, relu_in);
        }
#pragma unroll
        for (int cb = 0; cb < NCB; ++cb) {
          const uint4 af = *reinterpret_cast<const uint4*>(lw + ((s * 2 + hf) * COP + cb * 32 + col) * 16);
#pragma unroll
          for (int m = 0; m < M; ++m) mma<H>(acc[m][cb], af, bc[m][s]);
        }
        // keep the scheduler from hoisting every k-step's weight reads (register pressure)
        __builtin_amdgcn_sched_barrier(0);
      }
    } else {
#pragma unroll
      for (int m = 0; m < M; ++m) acc[m][0][0] = __builtin_bit_cast(float, bc[m][0].x ^ bc[m][KS - 1].w);
    }

    // epilogue: lane holds voxel col, channels cb*32 + 8j + 4hf + (0..3)
#pragma unroll
    for (int m = 0; m < M; ++m) {
      const uint32_t yoff = lane_off(tb, m * 32 + col, v0 + m * 32 + col, a.nvox, a.fd, a.ysn, a.ysw);
#pragma unroll
      for (int cb = 0; cb < NCB; ++cb) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int co = cb * 32 + 8 * j + 4 * hf;
          const float4 bb = *reinterpret_cast<const float4*>(lb + co);
          float o[4] = {acc[m][cb][4 * j] + bb.x, acc[m][cb][4 * j + 1] + bb.y, acc[m][cb][4 * j + 2] + bb.z,
                        acc[m][cb][4 * j + 3] + bb.w};
          float e4[4] = {0.f, 0.f, 0.f, 0.f};
          if constexpr (EIN) unpack_pk<H>(ein[m][cb][j], e4);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            float rr = act_apply(a.act, o[e] * a.out_scale, 0.f);
            if (a.has_mask) rr = mask_apply(e4[e], rr, mslope);
            o[e] = rr;
          }
          const uint32_t so = co0 + co < a.cout ? yoff + 2 * (co0 + co) : PW_OOB;
          if (a.accumulate) {
            if (a.has_mask) {
              float y4[4];
              unpack_pk<H>(bload8(ry, so), y4);
#pragma unroll
              for (int e = 0; e < 4; ++e) o[e] += y4[e];
            } else {
#pragma unroll
              for (int e = 0; e < 4; ++e) o[e] += e4[e];
            }
          }
          if (!(a.ablate & 1)) bstore8(ry, so, pack_pk<H, uint2>(o));
        }
      }
    }
    if (tn < a.ntiles) {
#pragma unroll
      for (int m = 0; m < M; ++m)
#pragma unroll
        for (int s = 0; s < KS; ++s) bc[m][s] = bn[m][s];
    }
    t = tn;
  }
}

// Staged variant (NCB <= 7 output blocks, NKB <= 8 input blocks; NCB < NKB
// for the narrowing 1x1 convs, e.g. DRF's 256 -> 64): each wave owns an LDS
// tile buffer [32*M voxels][CIP + 8 pad] H.  The next tile is fetched with
// coalesced 16-byte loads (consecutive lanes -> consecutive bytes of a voxel
// row, then the next row) into registers while the current tile computes; the
// B fragments are read back from LDS (row pad: conflict-free ds_read_b128).
// The outputs take the same way back: H-packed accumulators to the buffer,
// then coalesced 16-byte row stores.  Wave-private buffer: no barriers.
// AL: every tile lies inside one sample (d*h*w % (32*M) == 0), so a voxel
// row's offset is row * sw from the tile's base -- the common, cheap case;
// otherwise rows are placed with a division per row.  ACT: VSRK_ACT_NONE /
// VSRK_ACT_RELU at compile time (the epilogue is most of the VALU work).
// EIN: the ReLU/PReLU mask and / or accumulate of a data gradient
// (dx = mask(conv) [+ dx]) applied on the 16-byte row chunks of the store
// pass, their operands loaded as coalesced rows like the output (the tile
// kernel read them 8 bytes per lane across 32 voxel rows).  The buffered
// value is rounded to H before the accumulate: one extra rounding of the new
// term against the tile kernel.
// BNB (with RED 2, no PRO / bias): the input is the BN+ReLU backward of the
// previous BatchNorm, x' = k1 * (qx * k1 + sh > 0 ? x : 0) + k2 * qx + k3
// per channel (bn_relu_bwd_apply_kernel's arithmetic, so x' is bitwise the
// separate apply's; k1 = gamma * invstd is bn_finalize's scale, bn.hip:193),
// computed on the 16-byte row chunks between the coalesced loads and the LDS
// put, and stored once to xo for the weight gradient.
template <int NCB, int NKB, int M, bool PRO, bool AL, int ACT, int EIN, typename H, int RED = 0, bool BNB = false>
__global__ __launch_bounds__(PW_THR, 1) void pw_fwd_staged_kernel(PwArgs a) {
  const H* aX = reinterpret_cast<const H*>(a.x);
  H* aY = reinterpret_cast<H*>(a.y);
  const H* aW = reinterpret_cast<const H*>(a.w);
  constexpr int KS = 2 * NKB;
  constexpr int COP = 32 * NCB;
  constexpr int CIP = 16 * KS;
  constexpr int RS = 2 * (CIP > COP ? CIP : COP) + 16;  // buffer row stride (bytes): input or output row
  constexpr int CPR = CIP / 8;               // 16-byte chunks per row
  constexpr int ROWS = 32 * M;
  constexpr int NCK = ROWS * CPR / 64;       // chunks per lane per tile (= M*KS)
  constexpr int WBYTES = KS * 2 * COP * 16;
  extern __shared__ __attribute__((aligned(16))) char lds[];
  char* lw = lds;                                         // [KS][2][COP] x 16 B
  float* lsc = reinterpret_cast<float*>(lds + WBYTES);    // [CIP]
  float* lsh = lsc + CIP;                                 // [CIP]
  static_assert(!BNB || (RED == 2 && !PRO && !EIN && ACT == 0), "BNB: the data-gradient reduce form only");
  constexpr int OFF_LB = WBYTES + (PRO ? 2 * CIP * 4 : 0);
  constexpr int OFF_Q = OFF_LB + (BNB ? 0 : COP * 4);    // BNB: no bias (a data gradient)
  constexpr int OFF_BUF = OFF_Q + (BNB ? 4 * CIP * 4 : 0);
  float* lb = reinterpret_cast<float*>(lds + OFF_LB);     // [COP]
  float* lq = reinterpret_cast<float*>(lds + OFF_Q);      // BNB: [4][CIP] sh, k1, k2, k3
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int hf = lane >> 5, col = lane & 31;
  const int co0 = blockIdx.y * COP;
  char* buf = lds + OFF_BUF + wave * (ROWS * RS);

  for (int i = tid; i < KS * 2 * COP; i += PW_THR) {
    const int co = i % COP, t = i / COP, h = t & 1, s = t >> 1;
    const int ci = 16 * s + 8 * h;
    uint4 v = make_uint4(0, 0, 0, 0);
    if (ci < a.ci_pad && co0 + co < a.co_rows)
      v = *reinterpret_cast<const uint4*>(aW + (int64_t)(co0 + co) * a.ci_pad + ci);
    *reinterpret_cast<uint4*>(lw + i * 16) = v;
  }
  if (PRO) stage_prologue(lsc, lsh, a.prologue, a.pro_scale, a.pro_shift, a.cin, CIP, tid, PW_THR);
  if constexpr (BNB) {
    for (int c = tid; c < CIP; c += PW_THR) {
      float sh = 0.f, k1 = 0.f, k2 = 0.f, k3 = 0.f;
      if (c < a.cin) {  // bn_relu_bwd_apply_kernel's constants, the same fp32 operations
        const float is = a.qis[c], gm = a.qgm ? a.qgm[c] : 1.f;
        const float aa = gm * is, bb = is * a.qsdyx[c] * a.qinv_count;
        sh = a.qsh[c];
        k1 = aa;
        k2 = -aa * bb;
        k3 = aa * (a.qmu[c] * bb - a.qsdy[c] * a.qinv_count);
      }
      lq[c] = sh;
      lq[CIP + c] = k1;
      lq[2 * CIP + c] = k2;
      lq[3 * CIP + c] = k3;
    }
  } else {
    for (int i = tid; i < COP; i += PW_THR) lb[i] = (a.bias && co0 + i < a.cout) ? a.bias[co0 + i] : 0.f;
  }
  __syncthreads();

  const bool relu_in = (a.prologue & VSRK_PRO_RELU) != 0;
  const int nwaves = gridDim.x * (PW_THR / 64);
  const int wv = __builtin_amdgcn_readfirstlane(wave);
  const float osc = a.out_scale;
  const float pslope = ACT == VSRK_ACT_PRELU ? *a.act_param : 0.f;
  float sacc = 0.f;  // PBWD: this lane's slope-gradient partial
  // fused reduction: this lane's fixed 8-channel column and its constants
  constexpr int ROCPR = COP / 8;
  constexpr int RSTEP = 64 / ROCPR > 0 ? 64 / ROCPR : 1;
  constexpr int RNIT = RED ? (ROWS + RSTEP - 1) / RSTEP : 1;
  const int rcol = lane % ROCPR, rrow0 = lane / ROCPR;
  const bool rch_ok = co0 + 8 * rcol < a.cout;
  float rs1[8], rs2[8], rsc[8], rsh[8], rmu[8], ris[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    rs1[e] = rs2[e] = 0.f;
    rsc[e] = rsh[e] = rmu[e] = ris[e] = 0.f;
    if constexpr (RED == 2) {
      const int c = min(co0 + 8 * rcol + e, a.cout - 1);
      rsc[e] = a.bsc[c];
      rsh[e] = a.bsh[c];
      rmu[e] = a.bmu[c];
      ris[e] = a.bis[c];
    }
  }

  // byte offset of tile row `row` (voxel v0 + row) from the tile's sample base
  auto row_off = [&](const TileBase& tb, int row, int v0, int64_t sn, int64_t sw) __attribute__((always_inline)) {
    if constexpr (AL) {
      return (uint32_t)(2 * (tb.r0 + row) * (uint32_t)sw);
    } else {
      return lane_off(tb, row, v0 + row, a.nvox, a.fd, sn, sw);
    }
  };

  // fixed chunk roles: chunk k of a lane = row (lane + 64k) / CPR, column % CPR.
  // `ln` = lane through an opaque copy per use site: the per-chunk offsets
  // derived from it are recomputed (a few VALU) instead of held in VGPRs.
  constexpr int NQK = BNB ? NCK : 1;
  auto load = [&](int tile, uint4 (&r)[NCK], uint4 (&rq)[NQK]) __attribute__((always_inline)) {
    int ln = lane;
    asm volatile("" : "+v"(ln));
    const int v0 = tile * ROWS;
    const TileBase tb = tile_base(v0, a.fd);
    const Rsrc rs = rsrc_at(aX + (int64_t)tb.n0 * a.xsn);
#pragma unroll
    for (int k = 0; k < NCK; ++k) {
      const int i = ln + 64 * k, row = i / CPR, c = 8 * (i % CPR);
      const uint32_t off = row_off(tb, row, v0, a.xsn, a.xsw);
      r[k] = bload16(rs, c < a.cin ? off + 2 * c : PW_OOB);
    }
    if constexpr (BNB) {
      const Rsrc rq_ = rsrc_at(reinterpret_cast<const H*>(a.qx) + (int64_t)tb.n0 * a.qsn);
#pragma unroll
      for (int k = 0; k < NCK; ++k) {
        const int i = ln + 64 * k, row = i / CPR, c = 8 * (i % CPR);
        const uint32_t off = row_off(tb, row, v0, a.qsn, a.qsw);
        rq[k] = bload16(rq_, c < a.cin ? off + 2 * c : PW_OOB);
      }
    }
  };
  auto put = [&](int tile, const uint4 (&r)[NCK], const uint4 (&rq)[NQK]) __attribute__((always_inline)) {
    int ln = lane;
    asm volatile("" : "+v"(ln));
    if constexpr (BNB) {
      const int v0 = tile * ROWS;
      const TileBase tb = tile_base(v0, a.fd);
      const Rsrc ro = rsrc_at(reinterpret_cast<H*>(a.xo) + (int64_t)tb.n0 * a.osn);
      const uint32_t qb = lds_addr(lq);
#pragma unroll
      for (int k = 0; k < NCK; ++k) {
        const int i = ln + 64 * k, row = i / CPR, c = i % CPR;
        float g[8], f[8], o[8], sh[8], k1[8], k2[8], k3[8];
        Chunk<H>::unpack(r[k], g);
        Chunk<H>::unpack(rq[k], f);
        const uint32_t qa = qb + c * 32;
        *reinterpret_cast<float4*>(sh) = lds_ldf4(qa);
        *reinterpret_cast<float4*>(sh + 4) = lds_ldf4(qa + 16);
        *reinterpret_cast<float4*>(k1) = lds_ldf4(qa + CIP * 4);
        *reinterpret_cast<float4*>(k1 + 4) = lds_ldf4(qa + CIP * 4 + 16);
        *reinterpret_cast<float4*>(k2) = lds_ldf4(qa + CIP * 8);
        *reinterpret_cast<float4*>(k2 + 4) = lds_ldf4(qa + CIP * 8 + 16);
        *reinterpret_cast<float4*>(k3) = lds_ldf4(qa + CIP * 12);
        *reinterpret_cast<float4*>(k3 + 4) = lds_ldf4(qa + CIP * 12 + 16);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float dy = fmaf(f[e], k1[e], sh[e]) > 0.f ? g[e] : 0.f;
          o[e] = fmaf(k1[e], dy, fmaf(k2[e], f[e], k3[e]));
        }
        const uint4 v = Chunk<H>::pack(o);
        *reinterpret_cast<uint4*>(buf + row * RS + c * 16) = v;
        const uint32_t off = row_off(tb, row, v0, a.osn, a.osw);
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4i_t, v), ro,
                                               (int)(8 * c < a.cin ? off + 16 * c : PW_OOB), 0, PW_NT);
      }
    } else {
#pragma unroll
      for (int k = 0; k < NCK; ++k) {
        const int i = ln + 64 * k, row = i / CPR, c = i % CPR;
        *reinterpret_cast<uint4*>(buf + row * RS + c * 16) = r[k];
      }
    }
  };

  constexpr int EIN_NOK = ROWS * (COP / 8) / 64;  // store-pass row chunks per lane
  // EIN forms: 1 = generic (runtime flags: mask, accumulate, PBWD on the
  // channels >= pm_lo); compile-time and branch-free: EIN_ACC (accumulate),
  // EIN_PB (PBWD), EIN_PBACC (both).  The generic store pass carried ~3.5 K
  // extra instructions per tile (divergent per-chunk branches): 2.2x the plain
  // kernel's time at DRF's 64 -> 256 data gradients.
  const bool f_mask = EIN == 1 ? a.has_mask != 0 : false;
  const bool f_acc = EIN == 1 ? a.accumulate != 0 : (EIN == EIN_ACC || EIN == EIN_PBACC);
  const bool f_pb = EIN == 1 ? a.pbwd != 0 : (EIN == EIN_PB || EIN == EIN_PBACC);
  // Store-pass chunk k of a lane: row-major (2 rows of every column per k),
  // or, in the compile-time forms with whole 64-channel column groups, 8 rows
  // x one 64-channel group per k -- so "is this chunk on the PReLU tail" is
  // the same for the whole wave and the tail work is a scalar branch
  constexpr int OCPR_ = COP / 8;
  constexpr bool BLK = EIN >= 2 && OCPR_ % 8 == 0;
  constexpr int NGRP = OCPR_ / 8;
  auto chunk_rc = [&](int ln, int k, int& row, int& c) __attribute__((always_inline)) {
    if constexpr (BLK) {
      row = 8 * (k / NGRP) + (ln >> 3);
      c = 8 * (8 * (k % NGRP) + (ln & 7));
    } else {
      const int i = ln + 64 * k;
      row = i / OCPR_;
      c = 8 * (i % OCPR_);
    }
  };
  auto on_tail = [&](int k, int c) __attribute__((always_inline)) {  // BLK: wave-uniform
    return BLK ? co0 + 64 * (k % NGRP) >= a.pm_lo : co0 + c >= a.pm_lo;
  };
  auto ein_load = [&](int tile, uint4 (&em)[EIN ? EIN_NOK : 1], uint4 (&ey)[EIN ? EIN_NOK : 1])
                      __attribute__((always_inline)) {
    if constexpr (EIN) {
      constexpr int OCPR = COP / 8;
      int ln = lane;
      asm volatile("" : "+v"(ln));
      const int v0 = tile * ROWS;
      const TileBase tb = tile_base(v0, a.fd);
      const Rsrc ry = rsrc_at(aY + (int64_t)tb.n0 * a.ysn);
      const Rsrc rm = rsrc_at(reinterpret_cast<const H*>(a.msk ? a.msk : a.y) + (int64_t)tb.n0 * a.msn);
#pragma unroll
      for (int k = 0; k < EIN_NOK; ++k) {
        int row, c;
        chunk_rc(ln, k, row, c);
        const bool ok = co0 + c < a.cout;
        if (EIN == 1) {
          if (f_mask || (f_pb && co0 + c >= a.pm_lo))
            em[k] = bload16(rm, ok ? row_off(tb, row, v0, a.msn, a.msw) + 2 * (co0 + c) : PW_OOB);
        } else if (f_pb) {
          if (BLK) {
            if (on_tail(k, c)) em[k] = bload16(rm, ok ? row_off(tb, row, v0, a.msn, a.msw) + 2 * (co0 + c) : PW_OOB);
          } else {  // branch-free: chunks below pm_lo read nothing (out-of-range offset) and see m = 0
            em[k] = bload16(rm, ok && on_tail(k, c) ? row_off(tb, row, v0, a.msn, a.msw) + 2 * (co0 + c) : PW_OOB);
          }
        }
        if (f_acc) ey[k] = bload16(ry, ok ? row_off(tb, row, v0, a.ysn, a.ysw) + 2 * (co0 + c) : PW_OOB);
      }
    }
  };
  uint4 rg[NCK], rgq[NQK];
  int t = blockIdx.x * (PW_THR / 64) + wv;
  if (t < a.ntiles) load(t, rg, rgq);
  while (t < a.ntiles) {
    const int tn = t + nwaves;
    put(t, rg, rgq);
    // RED 2: the BN input rows of this tile's reduce, issued before the next
    // tile's operands so the epilogue's wait on them leaves those in flight
    uint4 bx[RED == 2 ? RNIT : 1];
    const bool lane_ok = lane < ROCPR * RSTEP;
    auto load_bx = [&]() __attribute__((always_inline)) {
      const int v0 = t * ROWS;
      const TileBase tb = tile_base(v0, a.fd);
      const Rsrc rb = rsrc_at(reinterpret_cast<const H*>(a.bnx) + (int64_t)tb.n0 * a.bsn);
#pragma unroll
      for (int j = 0; j < RNIT; ++j) {
        const int row = rrow0 + RSTEP * j;
        const bool ok = lane_ok && row < ROWS && rch_ok;
        bx[j] = bload16(rb, ok ? row_off(tb, row, v0, a.bsn, a.bsw) + 2 * (co0 + 8 * rcol) : PW_OOB);
      }
    };
    if constexpr (RED == 2 && PW_BXPRE) load_bx();
    if (tn < a.ntiles) load(tn, rg, rgq);  // in flight during this tile's MFMAs and stores
    // EIN: the store pass's mask / accumulate operands of this tile, issued
    // before its MFMAs (PW_EIN_EARLY) so their latency hides under them; issued
    // at the store pass they made an accumulate data gradient 2.2x the plain one
    // (DRF 64 -> 256 at 512^2: 312 vs 143 us, r5 tools/diag/pw_pbwd_micro.py)
    uint4 em[EIN ? EIN_NOK : 1], ey[EIN ? EIN_NOK : 1];
    if constexpr (EIN && PW_EIN_EARLY) ein_load(t, em, ey);

    f32x16 acc[M][NCB];
#pragma unroll
    for (int m = 0; m < M; ++m)
#pragma unroll
      for (int cb = 0; cb < NCB; ++cb)
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[m][cb][i] = 0.f;
    // k-step s+1's fragments (and prologue constants) are read while step s's MFMAs run
    struct Frag {
      uint4 a[NCB], b[M];
      float4 s0, s1, h0, h1;
    };
    // LDS byte addresses from opaque per-tile bases: the compiler would otherwise
    // hoist one VGPR per (k-step, block) address out of the tile loop (offsets
    // past the 64 KiB immediate range) and starve the fragment pipeline
    uint32_t abase = lds_addr(lw) + (hf * COP + col) * 16;
    uint32_t bbase = lds_addr(buf) + col * RS + hf * 16;
    asm volatile("" : "+v"(abase), "+v"(bbase));
    auto rd = [&](int s, Frag& f) __attribute__((always_inline)) {
#pragma unroll
      for (int m = 0; m < M; ++m) f.b[m] = lds_ld16(bbase + m * 32 * RS + 32 * s);
      const uint32_t as = abase + s * 2 * COP * 16;
#pragma unroll
      for (int cb = 0; cb < NCB; ++cb) f.a[cb] = lds_ld16(as + cb * 32 * 16);
      if (PRO) {
        const int c = 16 * s + 8 * hf;
        f.s0 = *reinterpret_cast<const float4*>(lsc + c);
        f.s1 = *reinterpret_cast<const float4*>(lsc + c + 4);
        f.h0 = *reinterpret_cast<const float4*>(lsh + c);
        f.h1 = *reinterpret_cast<const float4*>(lsh + c + 4);
      }
    };
    Frag fr[2];
    rd(0, fr[0]);
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      Frag& f = fr[s & 1];
      if (s + 1 < KS) rd(s + 1, fr[(s + 1) & 1]);
      if (PRO) {
#pragma unroll
        for (int m = 0; m < M; ++m) f.b[m] = h8_affine<H>(f.b[m], f.s0, f.s1, f.h0, f.h1, relu_in);
      }
#pragma unroll
      for (int cb = 0; cb < NCB; ++cb)
#pragma unroll
        for (int m = 0; m < M; ++m) mma<H>(acc[m][cb], f.a[cb], f.b[m]);
    }

    // epilogue into the buffer (row = voxel, COP H channels), then row stores
    {
      uint32_t ebase = lds_addr(buf) + col * RS + hf * 8;
      uint32_t bias_b = lds_addr(lb) + hf * 16;
      asm volatile("" : "+v"(ebase), "+v"(bias_b));
#pragma unroll
      for (int cb = 0; cb < NCB; ++cb)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          float4 bb = make_float4(0.f, 0.f, 0.f, 0.f);
          if constexpr (!BNB) bb = lds_ldf4(bias_b + (cb * 32 + 8 * j) * 4);
#pragma unroll
          for (int m = 0; m < M; ++m) {
            float o[4] = {acc[m][cb][4 * j] + bb.x, acc[m][cb][4 * j + 1] + bb.y, acc[m][cb][4 * j + 2] + bb.z,
                          acc[m][cb][4 * j + 3] + bb.w};
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              o[e] *= osc;
              if constexpr (ACT == VSRK_ACT_RELU) o[e] = fmaxf(o[e], 0.f);
              if constexpr (ACT == VSRK_ACT_PRELU) o[e] = o[e] > 0.f ? o[e] : pslope * o[e];
            }
            lds_st8(ebase + m * 32 * RS + (cb * 32 + 8 * j) * 2, pack_pk<H, uint2>(o));
          }
        }
    }
    if constexpr (RED != 0) {
      // reduce form of the store pass: lane l keeps ONE 8-channel column
      // (l % OCPR) and walks rows l / OCPR + RSTEP j, so its partial sums
      // are per channel; the lanes past OCPR * RSTEP idle
      const int v0 = t * ROWS;
      const TileBase tb = tile_base(v0, a.fd);
      const Rsrc ry = rsrc_at(aY + (int64_t)tb.n0 * a.ysn);
      if constexpr (RED == 2 && !PW_BXPRE) load_bx();
#pragma unroll
      for (int j = 0; j < RNIT; ++j) {
        const int row = rrow0 + RSTEP * j;
        if (lane_ok && row < ROWS) {
          const uint4 v = *reinterpret_cast<const uint4*>(buf + row * RS + 16 * rcol);
          const uint32_t off = row_off(tb, row, v0, a.ysn, a.ysw);
          const bool vox_ok = AL || v0 + row < a.nvox;
          if (!(a.ablate & 1))
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4i_t, v), ry,
                                                   (int)(rch_ok ? off + 2 * (co0 + 8 * rcol) : PW_OOB), 0, PW_NT);
          if (vox_ok && rch_ok) {
            float o[8];
            Chunk<H>::unpack(v, o);  // the stored (rounded) values, as the separate pass reads them
            if constexpr (RED == 1) {
#pragma unroll
              for (int e = 0; e < 8; ++e) {
                rs1[e] += o[e];
                rs2[e] = fmaf(o[e], o[e], rs2[e]);
              }
            } else {
              float xb[8];
              Chunk<H>::unpack(bx[j], xb);
#pragma unroll
              for (int e = 0; e < 8; ++e) {
                const float dy = fmaf(xb[e], rsc[e], rsh[e]) > 0.f ? o[e] : 0.f;
                rs1[e] += dy;
                rs2[e] = fmaf(dy, (xb[e] - rmu[e]) * ris[e], rs2[e]);
              }
            }
          }
        }
      }
    } else {
      const int v0 = t * ROWS;
      const TileBase tb = tile_base(v0, a.fd);
      const Rsrc ry = rsrc_at(aY + (int64_t)tb.n0 * a.ysn);
      constexpr int OCPR = COP / 8;
      constexpr int NOK = ROWS * OCPR / 64;
      static_assert(NOK >= 1 && ROWS * OCPR % 64 == 0, "whole row chunks per lane");
      int ln = lane;
      asm volatile("" : "+v"(ln));
      if constexpr (EIN && !PW_EIN_EARLY) ein_load(t, em, ey);  // every chunk's operands in flight together
      const float mslope = (EIN && a.mask_slope) ? *a.mask_slope : 0.f;
#pragma unroll
      for (int k = 0; k < NOK; ++k) {
        int row, c;
        chunk_rc(ln, k, row, c);
        uint4 v = *reinterpret_cast<const uint4*>(buf + row * RS + c * 2);
        if constexpr (EIN) {
          float o[8];
          Chunk<H>::unpack(v, o);
          if (f_mask) {
            float m[8];
            Chunk<H>::unpack(em[k], m);
#pragma unroll
            for (int e = 0; e < 8; ++e) o[e] = mask_apply(m[e], o[e], mslope);
          }
          if (f_acc) {
            float yo[8];
            Chunk<H>::unpack(ey[k], yo);
#pragma unroll
            for (int e = 0; e < 8; ++e) o[e] += yo[e];
          }
          v = Chunk<H>::pack(o);
          if (EIN != 1 && f_pb && (!BLK || on_tail(k, c))) {
            const bool tail = BLK || on_tail(k, c);
            float m[8], tr[8];
            Chunk<H>::unpack(em[k], m);
#pragma unroll
            for (int e = 0; e < 8; ++e) o[e] = (tail && !(m[e] > 0.f)) ? mslope * o[e] : o[e];
            v = Chunk<H>::pack(o);
            Chunk<H>::unpack(v, tr);  // the stored (rounded) values, as prelu_bwd reads them
#pragma unroll
            for (int e = 0; e < 8; ++e) sacc = fmaf(m[e] < 0.f ? tr[e] : 0.f, m[e], sacc);  // m = 0 off the tail
          } else if (f_pb && co0 + c >= a.pm_lo) {
            float m[8];
            Chunk<H>::unpack(em[k], m);
#pragma unroll
            for (int e = 0; e < 8; ++e) o[e] = m[e] > 0.f ? o[e] : mslope * o[e];
            v = Chunk<H>::pack(o);
            float tr[8];
            Chunk<H>::unpack(v, tr);  // the stored (rounded) values, as prelu_bwd reads them
            // (out-of-range rows load zeros: m = 0 adds nothing)
#pragma unroll
            for (int e = 0; e < 8; ++e)
              if (m[e] < 0.f) sacc = fmaf(tr[e], m[e], sacc);
          }
        }
        const uint32_t off = row_off(tb, row, v0, a.ysn, a.ysw);
        if (!(a.ablate & 1))
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4i_t, v), ry,
                                                 (int)(co0 + c < a.cout ? off + 2 * (co0 + c) : PW_OOB), 0, PW_NT);
      }
    }
    t = tn;
  }
  if constexpr (EIN) {
    if (f_pb) {
      const double wsum = vsrk_wave_sum((double)sacc);
      if (lane == 0) a.slope_part[(blockIdx.y * gridDim.x + blockIdx.x) * (PW_THR / 64) + wave] = wsum;
      return;
    }
  }
  if constexpr (RED != 0) {
    float* o = a.red_ws + ((((int64_t)blockIdx.y * gridDim.x + blockIdx.x) * (PW_THR / 64) + wave) * 64 + lane) * 16;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      o[e] = rs1[e];
      o[8 + e] = rs2[e];
    }
  }
}

// Channel c of a fused reduction: sum of the lane partials that hold its
// column, over (block, wave, lane) in a fixed order, in double.
__global__ __launch_bounds__(256) void pw_red_final_kernel(const float* __restrict__ ws, int nbx, int cop, int ocpr,
                                                           int rstep, int cout, float* __restrict__ o1,
                                                           float* __restrict__ o2) {
  const int c = blockIdx.x;
  if (c >= cout) return;
  const int yc = c / cop, cc = c - yc * cop, col = cc >> 3, e = cc & 7;
  const int nlane = rstep;            // lanes of column col: col + ocpr * k, k < rstep
  const int nitems = nbx * (PW_THR / 64) * nlane;
  double s1 = 0.0, s2 = 0.0;
  constexpr int U = 8;  // loads in flight per lane before the adds (the partials are latency-bound)
  for (int i0 = threadIdx.x; i0 < nitems; i0 += 256 * U) {
    float v1[U], v2[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = i0 + 256 * u;
      v1[u] = v2[u] = 0.f;
      if (i < nitems) {
        const int k = i % nlane, bw = i / nlane;  // bw = block * waves + wave
        const float* p = ws + (((int64_t)yc * nbx * (PW_THR / 64) + bw) * 64 + col + ocpr * k) * 16;
        v1[u] = p[e];
        v2[u] = p[8 + e];
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      s1 += v1[u];
      s2 += v2[u];
    }
  }
  __shared__ double r1[256], r2[256];
  r1[threadIdx.x] = s1;
  r2[threadIdx.x] = s2;
  __syncthreads();
  for (int k = 128; k > 0; k >>= 1) {
    if (threadIdx.x < k) {
      r1[threadIdx.x] += r1[threadIdx.x + k];
      r2[threadIdx.x] += r2[threadIdx.x + k];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    o1[c] = (float)r1[0];
    o2[c] = (float)r2[0];
  }
}

// Staged launch with the fused per-channel reduction (square f -> f convs,
// one output chunk): RED 1 with the BN prologue (a BatchNorm's input
// statistics, duf_net.py:198-201), RED 2 without (the data gradient that
// feeds a BN+ReLU backward, duf_net.py:198-200).
template <int NCB, int M, int RED, typename H, bool BNB = false>
static bool launch_fwd_reduce(const PwArgs& a, int grid, hipStream_t s) {
  constexpr int KS = 2 * NCB, COP = 32 * NCB, CIP = 16 * KS;
  const size_t lds = (size_t)KS * 2 * COP * 16 + (RED == 1 ? 2 * CIP * 4 : 0) + (BNB ? 4 * CIP * 4 : COP * 4) +
                     4 * (32 * M) * (2 * CIP + 16);
  const bool al = a.dhw % (32 * M) == 0;
  auto kern = al ? pw_fwd_staged_kernel<NCB, NCB, M, RED == 1, true, 0, false, H, RED, BNB>
                 : pw_fwd_staged_kernel<NCB, NCB, M, RED == 1, false, 0, false, H, RED, BNB>;
  (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  kern<<<dim3(grid, 1), PW_THR, lds, s>>>(a);
  return true;
}

// ---------------------------------------------------------------------------
// weight gradient
// ---------------------------------------------------------------------------
struct PwWArgs {
  const void* x;
  const void* dy;
  const float* pro_scale;
  const float* pro_shift;
  float* ws;
  int64_t xsn, xsw, dsn, dsw;  // element strides
  int nvox, vox_per_split, dhw;
  FastDiv fd;
  int cin, cout, prologue;
  int ncit;                  // ci blocks in this launch's chunks (<= 4*NCIW)
  int ci_chunks, nchunks;    // blockIdx.y = co_chunk * ci_chunks + ci_chunk
  int slab;                  // floats per (split, chunk): 32*NCO * 32*ncit + 32*NCO
  int want_bias;
};

// NCO dY channel blocks per chunk; NW waves (4 or 8), wave w owns X blocks
// w, w + NW, ... (NCIW of them).  NW = 8 takes the wide chunks (5-8 X
// blocks) with one block per wave: one pass over dY at 160-256 channels and
// half the accumulators per wave of the 4-wave form's two blocks.
// DEPTH register-staged stages in flight: 1 = the next stage's loads overlap
// the current stage's MFMAs only; 2 = two stages ahead (twice the staging
// registers).  A stage is 64 voxels, a few microseconds of HBM latency
// against well under one of MFMA work at these channel counts, so one
// stage in flight leaves the workgroup waiting on its loads (2.4-3 TB/s at
// 160-224 channels).
template <int NCO, int NCIW, typename H, int DEPTH = 1, int NW = 4>
__global__ __launch_bounds__(NW * 64, 1) void pw_wgrad_kernel(PwWArgs a) {
  const H* aX = reinterpret_cast<const H*>(a.x);
  const H* aD = reinterpret_cast<const H*>(a.dy);
  constexpr int THR = NW * 64;
  constexpr int NCIMAX = NW * NCIW;
  constexpr int DK = (PW_KP * 4 * NCO + THR - 1) / THR;     // dY pieces per thread
  constexpr int XK = (PW_KP * 4 * NCIMAX + THR - 1) / THR;  // X pieces per thread (max)
  constexpr int PLMAX = NCO + NCIMAX;   // 32-channel planes per stage (max)
  constexpr int PSZ = PW_KP * 64;       // bytes per plane: 64 voxel rows of 32 H
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int split = blockIdx.x, chunk = blockIdx.y;
  const int co_chunk = chunk / a.ci_chunks, ci_chunk = chunk - co_chunk * a.ci_chunks;
  const int co0 = co_chunk * 32 * NCO, ci0 = ci_chunk * 32 * a.ncit;
  const int vbeg = split * a.vox_per_split;
  const int vend = min(a.nvox, vbeg + a.vox_per_split);
  const int nst = vend > vbeg ? (vend - vbeg + PW_KP - 1) / PW_KP : 0;
  const bool relu_in = (a.prologue & VSRK_PRO_RELU) != 0;
  const bool aff = (a.prologue & VSRK_PRO_AFFINE) != 0;
  const bool do_bias = a.want_bias && ci_chunk == 0 && wave == 0;

  // Per-thread chunk roles, fixed for the whole loop: dY piece k (i < 256 NCO)
  // and X piece k (i < 256 ncit) are 16-byte pieces i = tid + THR k of the
  // stage's [voxel][plane][4 x 16 B] image; every load instruction reads one
  // tensor.  (Piece validity is wave-uniform: the bounds are multiples of 256.)
  int dvox[DK], dch[DK], dlds[DK];
#pragma unroll
  for (int k = 0; k < DK; ++k) {
    const int i = tid + k * THR;
    const int vox = i / (4 * NCO), within = i - vox * (4 * NCO);
    const int plane = within >> 2, q = within & 3;
    dvox[k] = vox;
    const int c = co0 + plane * 32 + q * 8;
    dch[k] = (i < PW_KP * 4 * NCO && c < a.cout) ? 2 * c : -1;
    dlds[k] = i < PW_KP * 4 * NCO ? plane * PSZ + vox * 64 + q * 16 : -1;
  }
  int xvox[XK], xch[XK], xlds[XK];
  const int nxc = 4 * a.ncit;
#pragma unroll
  for (int k = 0; k < XK; ++k) {
    const int i = tid + k * THR;
    const int vox = i / nxc, within = i - vox * nxc;
    const int plane = within >> 2, q = within & 3;
    xvox[k] = vox;
    const int c = ci0 + plane * 32 + q * 8;
    const bool ok = i < PW_KP * nxc;
    xch[k] = (ok && c < a.cin) ? 2 * c : -1;
    xlds[k] = ok ? (NCO + plane) * PSZ + vox * 64 + q * 16 : -1;
  }

  uint4 ry[DEPTH][DK], rx[DEPTH][XK];
  auto issue = [&](int st, auto S) __attribute__((always_inline)) {
    constexpr int R = decltype(S)::value;
    const int v0 = vbeg + st * PW_KP;
    const TileBase tb = tile_base(v0, a.fd);
    const Rsrc rdy = rsrc_at(aD + (int64_t)tb.n0 * a.dsn);
    const Rsrc rxx = rsrc_at(aX + (int64_t)tb.n0 * a.xsn);
#pragma unroll
    for (int k = 0; k < DK; ++k) {
      const uint32_t off = lane_off(tb, dvox[k], v0 + dvox[k], vend, a.fd, a.dsn, a.dsw);
      ry[R][k] = bload16(rdy, dch[k] >= 0 ? off + dch[k] : PW_OOB);
    }
#pragma unroll
    for (int k = 0; k < XK; ++k) {
      if (xlds[k] >= 0) {
        const uint32_t off = lane_off(tb, xvox[k], v0 + xvox[k], vend, a.fd, a.xsn, a.xsw);
        rx[R][k] = bload16(rxx, xch[k] >= 0 ? off + xch[k] : PW_OOB);
      }
    }
  };
  auto commit = [&](int buf, auto S) __attribute__((always_inline)) {
    constexpr int R = decltype(S)::value;
    char* base = lds + buf * (PLMAX * PSZ);
#pragma unroll
    for (int k = 0; k < DK; ++k)
      if (DK * THR == PW_KP * 4 * NCO || dlds[k] >= 0) *reinterpret_cast<uint4*>(base + dlds[k]) = ry[R][k];
#pragma unroll
    for (int k = 0; k < XK; ++k)
      if (xlds[k] >= 0) *reinterpret_cast<uint4*>(base + xlds[k]) = rx[R][k];
  };
  const std::integral_constant<int, 0> I0{};
  const std::integral_constant<int, DEPTH - 1> I1{};

  // prologue scale/shift of the lane's X channel in each owned block
  float psc[NCIW], psh[NCIW];
#pragma unroll
  for (int b = 0; b < NCIW; ++b) {
    const int c = ci0 + (wave + NW * b) * 32 + (lane & 31);
    const bool ok = c < a.cin;
    psc[b] = ok ? (aff ? a.pro_scale[c] : 1.f) : 0.f;
    psh[b] = ok ? (aff ? a.pro_shift[c] : 0.f) : 0.f;
  }

  f32x16 acc[NCO][NCIW];
#pragma unroll
  for (int i = 0; i < NCO; ++i)
#pragma unroll
    for (int b = 0; b < NCIW; ++b)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][b][e] = 0.f;
  float bsum[NCO];
#pragma unroll
  for (int i = 0; i < NCO; ++i) bsum[i] = 0.f;

  // ds_read_b64_tr_b16: group g = lane>>4 reads a 4-voxel x 16-channel block;
  // lane 4q+p addresses voxel row q, channels 4p..4p+3, and receives channel
  // lane&15 of the group's 16: lane l ends up with channel l&31 of the plane
  // for voxels 8*(l>>5) .. +7 of the k-step.
  const int g = lane >> 4, i16 = lane & 15, q = i16 >> 2, p = i16 & 3;
  const int colb = ((g & 1) * 16 + 4 * p) * 2;
  const int rowk = 8 * (g >> 1) + q;

  auto compute = [&](int buf) __attribute__((always_inline)) {
    const char* base = lds + buf * (PLMAX * PSZ);
#pragma unroll
    for (int kk = 0; kk < PW_KP / 16; ++kk) {
      const int row = kk * 16 + rowk;
      uint4 bfr[NCIW];
#pragma unroll
      for (int b = 0; b < NCIW; ++b) {
        const int blk = wave + NW * b;
        if (blk < a.ncit) {
          const char* px = base + (NCO + blk) * PSZ + row * 64 + colb;
          const v4i16 x0 = ds_read_tr(px), x1 = ds_read_tr(px + 4 * 64);
          uint4 xv = __builtin_bit_cast(uint4, __builtin_shufflevector(x0, x1, 0, 1, 2, 3, 4, 5, 6, 7));
          if (a.prologue) {
            float f[8];
            Chunk<H>::unpack(xv, f);
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              const float tt = fmaf(f[e], psc[b], psh[b]);
              f[e] = relu_in ? fmaxf(tt, 0.f) : tt;
            }
            xv = Chunk<H>::pack(f);
          }
          bfr[b] = xv;
        }
      }
#pragma unroll
      for (int cb = 0; cb < NCO; ++cb) {
        const char* py = base + cb * PSZ + row * 64 + colb;
        const v4i16 y0 = ds_read_tr(py), y1 = ds_read_tr(py + 4 * 64);
        const uint4 af = __builtin_bit_cast(uint4, __builtin_shufflevector(y0, y1, 0, 1, 2, 3, 4, 5, 6, 7));
        if (do_bias) {
          float fa[8];
          Chunk<H>::unpack(af, fa);
#pragma unroll
          for (int e = 0; e < 8; ++e) bsum[cb] += fa[e];
        }
#pragma unroll
        for (int b = 0; b < NCIW; ++b)
          if (wave + NW * b < a.ncit)
            mma<H>(acc[cb][b], af, bfr[b]);
      }
    }
  };

  if constexpr (DEPTH == 1) {
    if (nst > 0) {
      issue(0, I0);
      commit(0, I0);
      __syncthreads();
    }
    for (int st = 0; st < nst; ++st) {
      if (st + 1 < nst) issue(st + 1, I0);
      compute(st & 1);
      if (st + 1 < nst) commit((st + 1) & 1, I0);
      __syncthreads();
    }
  } else {
    // stage s lives in register set s & 1 and LDS buffer s & 1.  Issues run
    // past the end unconditionally (every voxel out of range: zero loads, no
    // memory traffic), so the compiler's in-order vmcnt waits stay exact.
    if (nst > 0) {
      issue(0, I0);
      issue(1, I1);
      commit(0, I0);
      __syncthreads();
      issue(2, I0);
      for (int st = 0; st < nst; st += 2) {
        compute(0);
        commit(1, I1);  // stage st + 1
        __syncthreads();
        issue(st + 3, I1);
        if (st + 1 >= nst) break;
        compute(1);
        commit(0, I0);  // stage st + 2
        __syncthreads();
        issue(st + 4, I0);
      }
    }
  }

  // slab: [co (32*NCO)][ci (32*ncit)] then dbias[32*NCO]
  const int cic = 32 * a.ncit;
  float* out = a.ws + ((int64_t)split * a.nchunks + chunk) * a.slab;
  const int hf = lane >> 5, col = lane & 31;
#pragma unroll
  for (int cb = 0; cb < NCO; ++cb)
#pragma unroll
    for (int b = 0; b < NCIW; ++b) {
      const int blk = wave + NW * b;
      if (blk < a.ncit) {
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int co = cb * 32 + 8 * (e >> 2) + 4 * hf + (e & 3);
          out[co * cic + blk * 32 + col] = acc[cb][b][e];
        }
      }
    }
  if (a.want_bias && ci_chunk == 0 && wave == 0) {
#pragma unroll
    for (int cb = 0; cb < NCO; ++cb) {
      const float tot = bsum[cb] + __shfl_xor(bsum[cb], 32);
      if (hf == 0) out[32 * NCO * cic + cb * 32 + col] = tot;
    }
  }
}

// dw[co][ci] (torch layout of a 1x1x1 weight, fp32) [+]= scale * sum over
// splits of the slabs; then dbias.  A block = 32 consecutive outputs x 8 split
// groups; group g sums splits g, g+8, ... in order (4 loads in flight), the 8
// partials are added in a fixed order: deterministic.
__global__ __launch_bounds__(256) void pw_wgrad_reduce(const float* __restrict__ ws, float* __restrict__ dw,
                                                      float* __restrict__ db, int nsplit, int nchunks, int slab,
                                                      int cout, int cin, int cop, int cic, int ci_chunks,
                                                      float scale, int accumulate) {
  __shared__ float part[8][32];
  const int l = threadIdx.x & 31, grp = threadIdx.x >> 5;
  const int64_t idx = (int64_t)blockIdx.x * 32 + l;
  const int64_t nw = (int64_t)cout * cin;
  const int64_t total = nw + (db ? cout : 0);
  const float* p = nullptr;
  int co = 0;
  if (idx < nw) {
    co = (int)(idx / cin);
    const int ci = (int)(idx - (int64_t)co * cin);
    const int chunk = (co / cop) * ci_chunks + ci / cic;
    p = ws + (int64_t)chunk * slab + (int64_t)(co % cop) * cic + (ci % cic);
  } else if (idx < total) {
    co = (int)(idx - nw);
    const int chunk = (co / cop) * ci_chunks;
    p = ws + (int64_t)chunk * slab + (int64_t)cop * cic + (co % cop);
  }
  float s = 0.f;
  if (p) {
    const int64_t ss = (int64_t)nchunks * slab;
    int k = grp;
    for (; k + 24 < nsplit; k += 32) {
      const float a0 = p[k * ss], a1 = p[(k + 8) * ss], a2 = p[(k + 16) * ss], a3 = p[(k + 24) * ss];
      s += a0;
      s += a1;
      s += a2;
      s += a3;
    }
    for (; k < nsplit; k += 8) s += p[k * ss];
  }
  part[grp][l] = s;
  __syncthreads();
  if (grp != 0 || idx >= total) return;
  float t = part[0][l];
#pragma unroll
  for (int g = 1; g < 8; ++g) t += part[g][l];
  t *= scale;
  if (idx < nw) {
    float* d = dw + idx;
    *d = accumulate ? *d + t : t;
  } else {
    db[co] = accumulate ? db[co] + t : t;
  }
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
static bool dhw_dense(const vsrk_tensor5* t) {
  return t->shuffle <= 1 && t->sw >= t->c && (t->h == 1 || t->sh == (int64_t)t->w * t->sw) &&
         (t->d == 1 || t->sd == (int64_t)t->h * t->sh);
}

// Staged launch (LDS row buffers) of (NCB output blocks, NKB input blocks);
// false when the staged kernel is off (VSRK_PW_STAGED=0) or the output is
// not 8-channel aligned.
template <int NCB, int NKB, int M, typename H>
static bool launch_fwd_staged(const PwArgs& a, int grid, int nchunk, bool pro, hipStream_t s) {
  constexpr int KS = 2 * NKB, COP = 32 * NCB, CIP = 16 * KS;
  static int staged = -1;
  if (staged < 0) {
    const char* e = getenv("VSRK_PW_STAGED");
    staged = (e && e[0] == '0') ? 0 : 1;
  }
  if (!staged || a.cout % 8 != 0) return false;
  const bool ein = a.has_mask || a.accumulate || a.pbwd;
  if (ein && (pro || a.act != VSRK_ACT_NONE)) return false;  // data gradients: no prologue / activation
  if (pro && a.act == VSRK_ACT_PRELU) return false;
  constexpr int RW = CIP > COP ? CIP : COP;
  const size_t lds = (size_t)KS * 2 * COP * 16 + (pro ? 2 * CIP * 4 : 0) + COP * 4 + 4 * (32 * M) * (2 * RW + 16);
  const bool al = a.dhw % (32 * M) == 0;
  const bool relu = a.act == VSRK_ACT_RELU;
  using K = void (*)(PwArgs);
  K kern;
  if (ein) {
    kern = al ? pw_fwd_staged_kernel<NCB, NKB, M, false, true, 0, EIN_GEN, H>
              : pw_fwd_staged_kernel<NCB, NKB, M, false, false, 0, EIN_GEN, H>;
    if constexpr (NKB == 2) {  // DRF's 64-input-channel data gradients: the branch-free forms
      // (with whole 64-channel store groups (COP % 64 == 0) the PReLU tail is
      // decided per group, so it must start on a group boundary; any other
      // c_lo -- e.g. num_features 48: c_lo = 144 of 192 -- takes the generic
      // per-chunk form)
      constexpr bool GROUPED = (COP / 8) % 8 == 0;
      const bool tail_ok = !a.pbwd || !GROUPED || a.pm_lo % 64 == 0;
      if (!a.has_mask && (a.accumulate || a.pbwd) && tail_ok) {
        const int mode = a.pbwd ? (a.accumulate ? EIN_PBACC : EIN_PB) : EIN_ACC;
        if (mode == EIN_ACC)
          kern = al ? pw_fwd_staged_kernel<NCB, NKB, M, false, true, 0, EIN_ACC, H>
                    : pw_fwd_staged_kernel<NCB, NKB, M, false, false, 0, EIN_ACC, H>;
        else if (mode == EIN_PB)
          kern = al ? pw_fwd_staged_kernel<NCB, NKB, M, false, true, 0, EIN_PB, H>
                    : pw_fwd_staged_kernel<NCB, NKB, M, false, false, 0, EIN_PB, H>;
        else
          kern = al ? pw_fwd_staged_kernel<NCB, NKB, M, false, true, 0, EIN_PBACC, H>
                    : pw_fwd_staged_kernel<NCB, NKB, M, false, false, 0, EIN_PBACC, H>;
      }
    }
  } else if (a.act == VSRK_ACT_PRELU) {
    kern = al ? pw_fwd_staged_kernel<NCB, NKB, M, false, true, VSRK_ACT_PRELU, false, H>
              : pw_fwd_staged_kernel<NCB, NKB, M, false, false, VSRK_ACT_PRELU, false, H>;
  } else if (pro) {
    if (al) kern = relu ? pw_fwd_staged_kernel<NCB, NKB, M, true, true, 1, false, H>
                        : pw_fwd_staged_kernel<NCB, NKB, M, true, true, 0, false, H>;
    else kern = relu ? pw_fwd_staged_kernel<NCB, NKB, M, true, false, 1, false, H>
                     : pw_fwd_staged_kernel<NCB, NKB, M, true, false, 0, false, H>;
  } else {
    if (al) kern = relu ? pw_fwd_staged_kernel<NCB, NKB, M, false, true, 1, false, H>
                        : pw_fwd_staged_kernel<NCB, NKB, M, false, true, 0, false, H>;
    else kern = relu ? pw_fwd_staged_kernel<NCB, NKB, M, false, false, 1, false, H>
                     : pw_fwd_staged_kernel<NCB, NKB, M, false, false, 0, false, H>;
  }
  (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  kern<<<dim3(grid, nchunk), PW_THR, lds, s>>>(a);
  return true;
}

static int pw_grid(int64_t ntiles) {
  int grid = (int)std::min<int64_t>(pw_num_cus(), ceil_div64(ntiles, PW_THR / 64));
  if (vsrk_g_grid_cap > 0) grid = std::min(grid, vsrk_g_grid_cap);
  return std::max(grid, 1);
}

// false: not launched (a PReLU activation needs the staged kernel)
template <int NCB, int M, typename H>
static bool launch_fwd(const PwArgs& a, int nchunk, bool pro, hipStream_t s) {
  constexpr int KS = 2 * NCB, COP = 32 * NCB, CIP = 16 * KS;
  const int grid = pw_grid(a.ntiles);
  if constexpr (NCB <= 7) {
    if (launch_fwd_staged<NCB, NCB, M, H>(a, grid, nchunk, pro, s)) return true;
  }
  if constexpr (NCB == 8) {
    // 256 input channels: the staged kernel in two 128-channel output chunks
    // per 256 (x read twice, once per chunk, at the staged kernel's rate; the
    // tile kernel below ran DUF's 256 -> 256 / 512 heads at 1.5-2 TB/s)
    static int st8 = -1;  // A/B knob VSRK_PW_STAGED8=0
    if (st8 < 0) {
      const char* e = getenv("VSRK_PW_STAGED8");
      st8 = (e && e[0] == '0') ? 0 : 1;
    }
    if (st8 && M == 1 && launch_fwd_staged<4, 8, 1, H>(a, grid, 2 * nchunk, pro, s)) return true;
  }
  if (a.act == VSRK_ACT_PRELU) return false;
  const bool ein = a.has_mask || a.accumulate;
  const size_t lds = (size_t)KS * 2 * COP * 16 + (2 * CIP + COP) * sizeof(float);
  auto kern = pro ? (ein ? pw_fwd_kernel<NCB, M, true, true, H> : pw_fwd_kernel<NCB, M, true, false, H>)
                  : (ein ? pw_fwd_kernel<NCB, M, false, true, H> : pw_fwd_kernel<NCB, M, false, false, H>);
  (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  kern<<<dim3(grid, nchunk), PW_THR, lds, s>>>(a);
  return true;
}

// tiles of 32*M voxels, M chosen so one wave step loads ~16 KiB
template <int NCB>
constexpr int pw_m() { return NCB <= 2 ? 4 : (NCB <= 4 ? 2 : 1); }

}  // namespace

// The forward / data-gradient arguments common to every staged and tile
// pointwise launch; false when a lane offset could pass 2 GiB.
static bool pw_fill_args(PwArgs& a, const vsrk_conv_desc* d, const vsrk_tensor5* x, const void* w_packed,
                         const float* bias, const float* pro_scale, const float* pro_shift, const vsrk_tensor5* mask,
                         const vsrk_tensor5* y, int cip) {
  a = PwArgs{};
  a.x = x->ptr;
  a.y = y->ptr;
  a.msk = mask ? mask->ptr : nullptr;
  a.w = w_packed;
  a.bias = bias;
  a.pro_scale = pro_scale;
  a.pro_shift = pro_shift;
  a.mask_slope = d->mask_slope;
  a.act_param = d->act_param;
  a.xsn = x->sn; a.xsw = x->sw;
  a.ysn = y->sn; a.ysw = y->sw;
  a.msn = mask ? mask->sn : 0;
  a.msw = mask ? mask->sw : 0;
  a.dhw = x->d * x->h * x->w;
  const int64_t nvox = (int64_t)x->n * a.dhw;
  if (nvox >= (1ll << 31) - 4096) return false;
  a.nvox = (int)nvox;
  a.fd = make_fastdiv(std::max(a.dhw, 1));
  {
    // lane offsets relative to a tile's first sample stay below 2 GiB
    const int64_t span_n = 32 * 4 / std::max(a.dhw, 1) + 2;
    for (const vsrk_tensor5* t : {x, y, mask}) {
      if (t && 2 * (span_n * t->sn + (int64_t)a.dhw * t->sw + t->c) >= 0x7FFFFFF0ll) return false;
    }
  }
  static int ablate = -1;
  if (ablate < 0) {
    const char* e = getenv("VSRK_PW_ABLATE");
    ablate = e ? atoi(e) : 0;
  }
  a.ablate = ablate;
  a.cin = x->c;
  a.cout = y->c;
  a.ci_pad = cip;
  a.co_rows = round_up(y->c, 128);
  a.prologue = d->prologue;
  a.act = d->act;
  a.accumulate = d->accumulate;
  a.has_mask = mask != nullptr;
  a.out_scale = d->out_scale;
  return true;
}

namespace {
struct PwPbwd {  // the PBWD form (see PwArgs::pbwd)
  int c_lo;
  const vsrk_slope_out* out;
};
}  // namespace

static int fwd_pw_impl(const vsrk_conv_desc* d, const vsrk_tensor5* x, const void* w_packed, const float* bias,
                       const float* pro_scale, const float* pro_shift, const vsrk_tensor5* residual,
                       const vsrk_tensor5* mask, const vsrk_tensor5* y, hipStream_t s, const PwPbwd* pb);

// 1 = launched, 0 = not eligible (caller uses the tile kernels), <0 = -status.
int vsrk_conv_fwd_pw(const vsrk_conv_desc* d, const vsrk_tensor5* x, const void* w_packed, const float* bias,
                     const float* pro_scale, const float* pro_shift, const vsrk_tensor5* residual,
                     const vsrk_tensor5* mask, const vsrk_tensor5* y, hipStream_t s) {
  return fwd_pw_impl(d, x, w_packed, bias, pro_scale, pro_shift, residual, mask, y, s, nullptr);
}

// The data gradient of a pointwise conv with its consumer's PReLU backward
// after the accumulate on output channels >= c_lo (mask = that PReLU's output,
// y's geometry): 1 = launched (*nparts slope partials in ws), 0 = not eligible.
int vsrk_conv_fwd_pw_pbwd(const vsrk_conv_desc* d, const vsrk_tensor5* x, const void* w_packed,
                          const vsrk_tensor5* mask, const vsrk_tensor5* y, int c_lo, const vsrk_slope_out* slope,
                          hipStream_t s) {
  if (!mask || !d->mask_slope || d->prologue || d->act != VSRK_ACT_NONE || d->out_scale != 1.f) return 0;
  if (c_lo < 0 || c_lo >= y->c || c_lo % 8) return 0;
  if (mask->shuffle > 1 || y->shuffle > 1) return 0;
  vsrk_conv_desc dd = *d;
  PwPbwd pb{c_lo, slope};
  return fwd_pw_impl(&dd, x, w_packed, nullptr, nullptr, nullptr, nullptr, mask, y, s, &pb);
}

// grid <= CUs, <= 2 output chunks, one partial per wave
size_t vsrk_pw_pbwd_ws_bytes() { return (size_t)pw_num_cus() * 2 * (PW_THR / 64) * sizeof(double); }

static int fwd_pw_impl(const vsrk_conv_desc* d, const vsrk_tensor5* x, const void* w_packed, const float* bias,
                       const float* pro_scale, const float* pro_shift, const vsrk_tensor5* residual,
                       const vsrk_tensor5* mask, const vsrk_tensor5* y, hipStream_t s, const PwPbwd* pb) {
  if (!pw_enabled()) return 0;
  if (!vsrk_is16(x->dtype) || y->dtype != x->dtype) return 0;
  if (d->kd != 1 || d->kh != 1 || d->kw != 1 || d->pd || d->ph || d->pw) return 0;
  if (residual || d->bias_perm_r > 1) return 0;
  if (d->act == VSRK_ACT_PRELU && !d->act_param) return 0;
  if (x->n != y->n || x->d != y->d || x->h != y->h || x->w != y->w) return 0;
  if (!dhw_dense(x) || !dhw_dense(y) || (mask && (!dhw_dense(mask) || mask->dtype != x->dtype))) return 0;
  if (mask && (mask->n != y->n || mask->d != y->d || mask->h != y->h || mask->w != y->w || mask->c != y->c)) return 0;
  if (x->c % 8 || y->c % 4 || !chunk_ok(x, 2)) return 0;
  if (((uintptr_t)y->ptr) % 8 || y->sn % 4 || y->sw % 4) return 0;
  if (mask && (((uintptr_t)mask->ptr) % 8 || mask->sn % 4 || mask->sw % 4)) return 0;
  const int cip = round_up(x->c, 32);
  const int ncb = cip / 32;  // square kernels: COP = CIP
  if (ncb < 2 || ncb > 8) return 0;
  const int cop_total = round_up(y->c, 32);
  // narrowing convs (DRF's 128..256 -> 64 projections, DUF's 256 -> 16
  // residual head) and the widening data gradients of DRF's 64 -> 128..256
  // projections: one output chunk of cop_total != cip channels (one pass
  // over x instead of cop_total / cip)
  const bool wide_ok = ncb == 2 && (cop_total == 128 || cop_total == 192 || cop_total == 256);
  const int narrow = (cop_total < cip || wide_ok) ? cop_total / 32 : 0;
  if (!narrow && cop_total % cip != 0) return 0;  // output handled in chunks of CIP channels
  const int nchunk = narrow ? 1 : cop_total / cip;
  PwArgs a;
  if (!pw_fill_args(a, d, x, w_packed, bias, pro_scale, pro_shift, mask, y, cip)) return 0;
  if (pb) {  // the mask operand is the PReLU output read after the accumulate
    a.has_mask = 0;
    a.pbwd = 1;
    a.pm_lo = pb->c_lo;
    a.slope_part = pb->out->part;
    *pb->out->nparts = 0;
  }
  if (a.nvox == 0) return 1;
  const bool pro = d->prologue != VSRK_PRO_NONE;
  // PBWD: the staged kernel only, its grid's partials must fit the workspace
  auto pb_fits = [&](int grid, int nchunk) {
    if (!pb) return true;
    const size_t n = (size_t)grid * nchunk * (PW_THR / 64);
    if (n > pb->out->cap) return false;
    *pb->out->nparts = (int)n;
    return true;
  };
  if (narrow) {
    bool ok = false;
    auto go = [&](auto ncb_c, auto nkb_c) {
      constexpr int NC = decltype(ncb_c)::value, NK = decltype(nkb_c)::value;
      constexpr int M = pw_m<NK>() * NC <= 8 ? pw_m<NK>() : (8 / NC > 0 ? 8 / NC : 1);  // <= 128 accumulators
      a.ntiles = ceil_div(a.nvox, 32 * M);
      if (!pb_fits(pw_grid(a.ntiles), 1)) return;
      vsrk_dispatch16(x->dtype, [&](auto tag) {
        ok = launch_fwd_staged<NC, NK, M, decltype(tag)>(a, pw_grid(a.ntiles), 1, pro, s);
        return 0;
      });
    };
    using I1 = std::integral_constant<int, 1>;
    using I2 = std::integral_constant<int, 2>;
    if (narrow == 1 && ncb == 8) go(I1{}, std::integral_constant<int, 8>{});
    else if (narrow == 2 && ncb == 4) go(I2{}, std::integral_constant<int, 4>{});
    else if (narrow == 2 && ncb == 6) go(I2{}, std::integral_constant<int, 6>{});
    else if (narrow == 2 && ncb == 8) go(I2{}, std::integral_constant<int, 8>{});
    else if (narrow == 4 && ncb == 2) go(std::integral_constant<int, 4>{}, I2{});
    else if (narrow == 6 && ncb == 2) go(std::integral_constant<int, 6>{}, I2{});
    else if (narrow == 8 && ncb == 2) go(std::integral_constant<int, 8>{}, I2{});
    else return 0;
    if (!ok) return 0;
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
      vsrk_set_error("conv_fwd_pw: launch failed: %s", hipGetErrorString(e));
      return -(int)VSRK_ERR_LAUNCH;
    }
    return 1;
  }
  if (pb) {  // square forms: the staged kernel, NCB <= 7 (one launch per CIP-channel chunk)
    bool ok = false;
    switch (ncb) {
#define PW_PB_CASE(N)                                                                              \
  case N:                                                                                          \
    a.ntiles = ceil_div(a.nvox, 32 * pw_m<N>());                                                   \
    if (pb_fits(pw_grid(a.ntiles), nchunk))                                                        \
      vsrk_dispatch16(x->dtype, [&](auto tag) {                                                    \
        ok = launch_fwd_staged<N, N, pw_m<N>(), decltype(tag)>(a, pw_grid(a.ntiles), nchunk, pro, s); \
        return 0;                                                                                  \
      });                                                                                          \
    break;
      PW_PB_CASE(2) PW_PB_CASE(3) PW_PB_CASE(4) PW_PB_CASE(5) PW_PB_CASE(6) PW_PB_CASE(7)
#undef PW_PB_CASE
      default:
        break;
    }
    if (!ok) return 0;
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
      vsrk_set_error("conv_fwd_pw: launch failed: %s", hipGetErrorString(e));
      return -(int)VSRK_ERR_LAUNCH;
    }
    return 1;
  }
  switch (ncb) {
#define PW_CASE(N)                                                     \
  case N:                                                              \
    a.ntiles = ceil_div(a.nvox, 32 * pw_m<N>());                       \
    if (!vsrk_dispatch16(x->dtype, [&](auto tag) {                     \
          return (int)launch_fwd<N, pw_m<N>(), decltype(tag)>(a, nchunk, pro, s); \
        }))                                                            \
      return 0;                                                        \
    break;
    PW_CASE(2) PW_CASE(3) PW_CASE(4) PW_CASE(5) PW_CASE(6) PW_CASE(7) PW_CASE(8)
#undef PW_CASE
    default:
      return 0;
  }
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    vsrk_set_error("conv_fwd_pw: launch failed: %s", hipGetErrorString(e));
    return -VSRK_ERR_LAUNCH;
  }
  return 1;
}

extern "C" size_t vsrk_conv_fwd_reduce_workspace(const vsrk_conv_desc* d, const vsrk_tensor5* y) {
  const size_t pw = (size_t)pw_num_cus() * (PW_THR / 64) * 64 * 16 * sizeof(float);
  if (d && y && d->kd == 3) return std::max(pw, vsrk_roll_bnred_ws_floats(y) * sizeof(float));
  return pw;
}

// q (with qx, xo): the BNB input form (vsrk_conv_fwd_reduce_bnb), x = q->dz
static int fwd_reduce_impl(const vsrk_conv_desc* d, const vsrk_tensor5* x, const void* w_packed, const float* bias,
                           const float* pro_scale, const float* pro_shift, const vsrk_tensor5* y, int32_t mode,
                           const vsrk_tensor5* bnx, const float* scale, const float* shift, const float* mean,
                           const float* invstd, float* out_a, float* out_b, void* workspace, size_t workspace_bytes,
                           void* stream, const vsrk_tensor5* qx, const vsrk_bn_contrib* q, const vsrk_tensor5* xo) {
  VSRK_CHECK(d && x && y && w_packed && out_a && out_b, "conv_fwd_reduce: null argument");
  VSRK_CHECK(mode == 1 || mode == 2, "conv_fwd_reduce: mode must be 1 (statistics) or 2 (BN+ReLU backward)");
  hipStream_t s = (hipStream_t)stream;
  if (mode == 2 && d->kd == 3 && !q) {
    // the data gradient of a dense unit's Conv3d 3x3x3 (conv2) feeding bn2's
    // backward: the rolling kernel's epilogue form (conv_roll.hip)
    VSRK_CHECK(bnx && scale && shift && mean && invstd, "conv_fwd_reduce: mode 2 needs bnx and the BN constants");
    VSRK_CHECK(workspace, "conv_fwd_reduce: null workspace");
    vsrk_roll_bnred r{bnx, scale, shift, mean, invstd, (float*)workspace, workspace_bytes / sizeof(float), 0, 0};
    const int rc = vsrk_conv_fwd_roll(d, x, w_packed, bias, nullptr, nullptr, nullptr, nullptr, y, s, nullptr, &r);
    if (rc == 0) return VSRK_ERR_UNSUPPORTED;
    if (rc < 0) return -rc;
    if (r.ntiles == 0) {
      (void)hipMemsetAsync(out_a, 0, sizeof(float) * y->c, s);
      (void)hipMemsetAsync(out_b, 0, sizeof(float) * y->c, s);
      return VSRK_OK;
    }
    return vsrk_roll_bnred_final(r, y->c, out_a, out_b, s);
  }
  // eligible: a square pointwise conv on the staged kernel, no epilogue operands
  if (!pw_enabled() || !vsrk_is16(x->dtype) || y->dtype != x->dtype) return VSRK_ERR_UNSUPPORTED;
  if (d->kd != 1 || d->kh != 1 || d->kw != 1 || d->pd || d->ph || d->pw || d->bias_perm_r > 1) return VSRK_ERR_UNSUPPORTED;
  if (d->act != VSRK_ACT_NONE || d->accumulate || d->out_scale != 1.f) return VSRK_ERR_UNSUPPORTED;
  if ((mode == 1) != (d->prologue != VSRK_PRO_NONE)) return VSRK_ERR_UNSUPPORTED;
  if (x->n != y->n || x->d != y->d || x->h != y->h || x->w != y->w || x->c != y->c) return VSRK_ERR_UNSUPPORTED;
  if (!dhw_dense(x) || !dhw_dense(y) || !chunk_ok(x, 2) || !chunk_ok(y, 2) || x->c % 32) return VSRK_ERR_UNSUPPORTED;
  const int ncb = x->c / 32;
  if (ncb < 2 || ncb > 7) return VSRK_ERR_UNSUPPORTED;
  if (mode == 2) {
    VSRK_CHECK(bnx && scale && shift && mean && invstd, "conv_fwd_reduce: mode 2 needs bnx and the BN constants");
    if (bnx->dtype != x->dtype || bnx->n != y->n || bnx->d != y->d || bnx->h != y->h || bnx->w != y->w ||
        bnx->c != y->c || !dhw_dense(bnx) || !chunk_ok(bnx, 2))
      return VSRK_ERR_UNSUPPORTED;
  }
  auto same_geo = [&](const vsrk_tensor5* t) {
    return t->dtype == x->dtype && t->n == x->n && t->d == x->d && t->h == x->h && t->w == x->w && t->c == x->c &&
           dhw_dense(t) && chunk_ok(t, 2);
  };
  if (q) {
    if (mode != 2 || bias || d->prologue != VSRK_PRO_NONE || !same_geo(qx) || !same_geo(xo)) return VSRK_ERR_UNSUPPORTED;
    VSRK_CHECK(q->shift && q->mean && q->invstd && q->sum_dy && q->sum_dy_xhat && q->count > 0,
               "conv_fwd_reduce_bnb: missing BatchNorm operands");
  }
  PwArgs a;
  if (!pw_fill_args(a, d, x, w_packed, bias, pro_scale, pro_shift, nullptr, y, x->c)) return VSRK_ERR_UNSUPPORTED;
  if (q) {
    const int64_t span_n = 32 * 4 / std::max(a.dhw, 1) + 2;
    for (const vsrk_tensor5* t : {qx, xo})
      if (2 * (span_n * t->sn + (int64_t)a.dhw * t->sw + t->c) >= 0x7FFFFFF0ll) return VSRK_ERR_UNSUPPORTED;
    a.qx = qx->ptr;
    a.qsn = qx->sn;
    a.qsw = qx->sw;
    a.xo = xo->ptr;
    a.osn = xo->sn;
    a.osw = xo->sw;
    a.qsh = q->shift;
    a.qmu = q->mean;
    a.qis = q->invstd;
    a.qgm = q->gamma;
    a.qsdy = q->sum_dy;
    a.qsdyx = q->sum_dy_xhat;
    a.qinv_count = (float)(1.0 / q->count);
  }
  if (mode == 2) {
    const int64_t span_n = 32 * 4 / std::max(a.dhw, 1) + 2;
    if (2 * (span_n * bnx->sn + (int64_t)a.dhw * bnx->sw + bnx->c) >= 0x7FFFFFF0ll) return VSRK_ERR_UNSUPPORTED;
    a.bnx = bnx->ptr;
    a.bsn = bnx->sn;
    a.bsw = bnx->sw;
    a.bsc = scale;
    a.bsh = shift;
    a.bmu = mean;
    a.bis = invstd;
  }
  VSRK_CHECK(workspace && workspace_bytes >= vsrk_conv_fwd_reduce_workspace(d, y),
             "conv_fwd_reduce: workspace %zu < %zu bytes", workspace_bytes, vsrk_conv_fwd_reduce_workspace(d, y));
  a.red_ws = (float*)workspace;
  if (a.nvox == 0) {
    (void)hipMemsetAsync(out_a, 0, sizeof(float) * y->c, s);
    (void)hipMemsetAsync(out_b, 0, sizeof(float) * y->c, s);
    return VSRK_OK;
  }
  int grid = 0;
  vsrk_dispatch16(x->dtype, [&](auto tag) {
    using H = decltype(tag);
    auto go = [&](auto ncb_c) {
      constexpr int NC = decltype(ncb_c)::value;
      a.ntiles = ceil_div(a.nvox, 32 * pw_m<NC>());
      grid = std::min(pw_grid(a.ntiles), pw_num_cus());
      if (mode == 1) launch_fwd_reduce<NC, pw_m<NC>(), 1, H>(a, grid, s);
      else if (q) launch_fwd_reduce<NC, pw_m<NC>(), 2, H, true>(a, grid, s);
      else launch_fwd_reduce<NC, pw_m<NC>(), 2, H>(a, grid, s);
    };
    switch (ncb) {
      case 2: go(std::integral_constant<int, 2>{}); break;
      case 3: go(std::integral_constant<int, 3>{}); break;
      case 4: go(std::integral_constant<int, 4>{}); break;
      case 5: go(std::integral_constant<int, 5>{}); break;
      case 6: go(std::integral_constant<int, 6>{}); break;
      default: go(std::integral_constant<int, 7>{}); break;
    }
    return 0;
  });
  VSRK_LAUNCH_CHECK("conv_fwd_reduce");
  const int ocpr = ncb * 4;
  pw_red_final_kernel<<<y->c, 256, 0, s>>>(a.red_ws, grid, 32 * ncb, ocpr, 64 / ocpr, y->c, out_a, out_b);
  VSRK_LAUNCH_CHECK("conv_fwd_reduce_final");
  return VSRK_OK;
}

extern "C" int vsrk_conv_fwd_reduce(const vsrk_conv_desc* d, const vsrk_tensor5* x, const void* w_packed,
                                    const float* bias, const float* pro_scale, const float* pro_shift,
                                    const vsrk_tensor5* y, int32_t mode, const vsrk_tensor5* bnx, const float* scale,
                                    const float* shift, const float* mean, const float* invstd, float* out_a,
                                    float* out_b, void* workspace, size_t workspace_bytes, void* stream) {
  return fwd_reduce_impl(d, x, w_packed, bias, pro_scale, pro_shift, y, mode, bnx, scale, shift, mean, invstd, out_a,
                         out_b, workspace, workspace_bytes, stream, nullptr, nullptr, nullptr);
}

extern "C" int vsrk_conv_fwd_reduce_bnb(const vsrk_conv_desc* d, const vsrk_tensor5* bn_x, const vsrk_bn_contrib* pre,
                                        const vsrk_tensor5* x_out, const void* w_packed, const vsrk_tensor5* y,
                                        const vsrk_tensor5* bnx, const float* scale, const float* shift,
                                        const float* mean, const float* invstd, float* out_a, float* out_b,
                                        void* workspace, size_t workspace_bytes, void* stream) {
  VSRK_CHECK(bn_x && pre && x_out, "conv_fwd_reduce_bnb: null argument");
  return fwd_reduce_impl(d, &pre->dz, w_packed, nullptr, nullptr, nullptr, y, 2, bnx, scale, shift, mean, invstd,
                         out_a, out_b, workspace, workspace_bytes, stream, bn_x, pre, x_out);
}

namespace {
struct PwWPlan {
  bool ok;
  int nco, ncit, ncoiw, nw, ci_chunks, co_chunks, nchunks, nsplit, slab;
  int64_t vps;
  size_t ws_bytes;
};

PwWPlan pw_wgrad_plan(const vsrk_conv_desc* d, const vsrk_tensor5* x, const vsrk_tensor5* dy) {
  PwWPlan p{};
  p.ok = false;
  if (!pw_enabled()) return p;
  if (!vsrk_is16(x->dtype) || dy->dtype != x->dtype) return p;
  if (d->kd != 1 || d->kh != 1 || d->kw != 1 || d->pd || d->ph || d->pw) return p;
  if (x->n != dy->n || x->d != dy->d || x->h != dy->h || x->w != dy->w) return p;
  if (!dhw_dense(x) || !dhw_dense(dy) || !chunk_ok(x, 2) || !chunk_ok(dy, 2)) return p;
  if (x->c % 8 || dy->c % 8) return p;
  const int cob = ceil_div(dy->c, 32), cib = ceil_div(x->c, 32);
  p.nco = std::min(cob, 8);
  p.co_chunks = ceil_div(cob, p.nco);
  // input chunks of <= 4 blocks, balanced (5 -> 3 + 2): one block per wave
  // and a stage small enough for two workgroups per CU.  Up to 8 blocks per
  // chunk (VSRK_PW_WGRAD_CI8=1: waves own blocks w and w + 4) read dY once
  // but ran 2.3-2.5 TB/s at 160-224 channels (one workgroup per CU, wave 0
  // holding two blocks of five) against 4.4-4.8 TB/s at <= 128.
  // Exception, measured (profiles/r4_pw_wgrad_ci8_ab.txt): where the 4-block
  // split's stage (2 x (nco + 4) x 4 KB) is over 80 KB it keeps one workgroup
  // per CU anyway, and chunks of up to 8 blocks read dY half as often: DUF
  // unit 5 (224 -> 224) 1568 -> 1071 us, the heads 256 -> 512 / 512 -> 400 /
  // 256 -> 256 910 / 1741 / 479 -> 657 / 1169 / 372 us; at 160 and 192
  // channels the split runs two workgroups per CU and stays ahead.
  static int ci8 = -1;
  if (ci8 == -1) {
    const char* e = getenv("VSRK_PW_WGRAD_CI8");
    ci8 = !e ? -2 : (e[0] == '1' ? 1 : 0);  // -2: automatic
  }
  // 8-wave form (VSRK_PW_WGRAD_NW8, default on): chunks of up to 8 X blocks,
  // one per wave, wherever the input has more than 4 blocks
  static int nw8 = -1;
  if (nw8 == -1) {
    const char* e = getenv("VSRK_PW_WGRAD_NW8");
    nw8 = !(e && e[0] == '0');
  }
  p.nw = (nw8 && cib > 4 && ci8 != 0) ? 8 : 4;
  const bool one_chunk = p.nw == 8 || ci8 == 1 || (ci8 == -2 && cib > 4 && std::min(cob, 8) + 4 > 10);
  p.ncit = std::min(cib, one_chunk ? 8 : 4);
  p.ci_chunks = ceil_div(cib, p.ncit);
  if (!one_chunk || p.nw == 8) p.ncit = ceil_div(cib, p.ci_chunks);
  if (p.nco < 2) return p;
  p.ncoiw = ceil_div(p.ncit, p.nw);
  p.nchunks = p.co_chunks * p.ci_chunks;
  const int64_t nvox = (int64_t)x->n * x->d * x->h * x->w;
  if (nvox >= (1ll << 31) - 4096) return p;
  {
    const int dhw = std::max(x->d * x->h * x->w, 1);
    const int64_t span_n = PW_KP / dhw + 2;
    for (const vsrk_tensor5* t : {x, dy})
      if (2 * (span_n * t->sn + (int64_t)dhw * t->sw + t->c) >= 0x7FFFFFF0ll) return p;
  }
  const int64_t steps = std::max<int64_t>(1, ceil_div64(nvox, PW_KP));
  // two workgroups per CU where the double-buffered stage fits LDS twice
  const size_t lds = (size_t)2 * (p.nco + p.nw * p.ncoiw) * PW_KP * 64;
  int want = std::max(1, pw_num_cus() * (lds <= 80 * 1024 ? 2 : 1) / p.nchunks);
  if (vsrk_g_grid_cap > 0) want = std::max(1, vsrk_g_grid_cap / p.nchunks);
  want = (int)std::min<int64_t>(want, steps);
  p.vps = ceil_div64(steps, want) * PW_KP;
  p.nsplit = (int)std::max<int64_t>(1, ceil_div64(nvox, p.vps));
  p.slab = 32 * p.nco * 32 * p.ncit + 32 * p.nco;
  p.ws_bytes = (size_t)p.nsplit * p.nchunks * p.slab * sizeof(float);
  p.ok = true;
  return p;
}

// stages in flight (VSRK_PW_WGRAD_DEPTH=1|2, default 2)
int pw_wgrad_depth() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("VSRK_PW_WGRAD_DEPTH");
    v = (e && e[0] == '1') ? 1 : 2;
  }
  return v;
}

template <int NCO, int NCIW, typename H, int NW = 4>
void launch_wgrad_pw(const PwWArgs& a, int nsplit, hipStream_t s) {
  const size_t lds = (size_t)2 * (NCO + NW * NCIW) * PW_KP * 64;
  auto kern = pw_wgrad_depth() == 2 ? pw_wgrad_kernel<NCO, NCIW, H, 2, NW> : pw_wgrad_kernel<NCO, NCIW, H, 1, NW>;
  (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  kern<<<dim3(nsplit, a.nchunks), NW * 64, lds, s>>>(a);
}
}  // namespace

size_t vsrk_conv_wgrad_pw_workspace(const vsrk_conv_desc* d, const vsrk_tensor5* x, const vsrk_tensor5* dy) {
  const PwWPlan p = pw_wgrad_plan(d, x, dy);
  return p.ok ? p.ws_bytes : 0;
}

// 1 = launched (kernel + reduce), 0 = not eligible, <0 = -status.
int vsrk_conv_wgrad_pw(const vsrk_conv_desc* d, const vsrk_tensor5* x, const vsrk_tensor5* dy,
                       const float* pro_scale, const float* pro_shift, float dy_scale, int32_t perm_r, float* dw,
                       float* dbias, int32_t accumulate, void* workspace, size_t workspace_bytes, hipStream_t s) {
  if (perm_r > 1) return 0;
  const PwWPlan p = pw_wgrad_plan(d, x, dy);
  if (!p.ok) return 0;
  if (!workspace || workspace_bytes < p.ws_bytes) {
    vsrk_set_error("conv_wgrad: workspace %zu < %zu bytes", workspace_bytes, p.ws_bytes);
    return -VSRK_ERR_INVALID;
  }
  PwWArgs a;
  a.x = x->ptr;
  a.dy = dy->ptr;
  a.pro_scale = pro_scale;
  a.pro_shift = pro_shift;
  a.ws = (float*)workspace;
  a.xsn = x->sn; a.xsw = x->sw;
  a.dsn = dy->sn; a.dsw = dy->sw;
  a.nvox = x->n * x->d * x->h * x->w;
  a.vox_per_split = (int)p.vps;
  a.dhw = x->d * x->h * x->w;
  a.fd = make_fastdiv(std::max(a.dhw, 1));
  a.cin = x->c;
  a.cout = dy->c;
  a.prologue = d->prologue;
  a.ncit = p.ncit;
  a.ci_chunks = p.ci_chunks;
  a.nchunks = p.nchunks;
  a.slab = p.slab;
  a.want_bias = dbias != nullptr;
  if (a.nvox > 0) {
    const bool w2 = p.ncoiw == 2, nw8 = p.nw == 8;
    switch (p.nco) {
#define PWW_CASE(N)                                                                   \
  case N:                                                                             \
    vsrk_dispatch16(x->dtype, [&](auto tag) {                                       \
      using H = decltype(tag);                                                      \
      if (nw8) launch_wgrad_pw<N, 1, H, 8>(a, p.nsplit, s);                        \
      else if (w2) launch_wgrad_pw<N, 2, H>(a, p.nsplit, s);                       \
      else launch_wgrad_pw<N, 1, H>(a, p.nsplit, s);                               \
      return 0;                                                                     \
    });                                                                             \
    break;
      PWW_CASE(2) PWW_CASE(3) PWW_CASE(4) PWW_CASE(5) PWW_CASE(6) PWW_CASE(7) PWW_CASE(8)
#undef PWW_CASE
      default:
        return 0;
    }
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
      vsrk_set_error("conv_wgrad_pw: launch failed: %s", hipGetErrorString(e));
      return -VSRK_ERR_LAUNCH;
    }
  } else {
    // no voxels: the gradient is zero (the reduce below sums nothing)
  }
  const int64_t total = (int64_t)dy->c * x->c + (dbias ? dy->c : 0);
  pw_wgrad_reduce<<<(int)ceil_div64(total, 32), 256, 0, s>>>(
      (const float*)workspace, dw, dbias, a.nvox > 0 ? p.nsplit : 0, p.nchunks, p.slab, dy->c, x->c, 32 * p.nco,
      32 * p.ncit, p.ci_chunks, dy_scale, accumulate);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    vsrk_set_error("conv_wgrad_pw_reduce: launch failed: %s", hipGetErrorString(e));
    return -VSRK_ERR_LAUNCH;
  }
  return 1;
}
