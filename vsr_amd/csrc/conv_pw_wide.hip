// Wide pointwise convolution (Conv3d 1x1x1 with more than 256 input channels
// or 256 -> >= 256) as a GEMM on MFMA for 16-bit channels-last views (gfx950):
// DUF's filter head (duf_net.py:40-46: Conv3d(256, 512, 1) + ReLU, Conv3d(512,
// 400, 1) to fp32 logits) and the data gradients of those convs and of the
// residual head's Conv3d(256, 16, 1) (loss.backward(), base_trainer.py:128).
//
// Why not the staged pointwise kernel (conv_pw.hip): it keeps the whole
// weight chunk (<= 256 x 256) in LDS and a whole input row per voxel in
// registers, so it stops at 256 input channels and runs 256 -> 512 as four
// passes over x; round 5 sent the 400 / 512-input convs to the generic tile
// kernel at ~1.5-2 TB/s (5.6 ms of DUF's step).  Here a
// workgroup owns a 256-voxel x 256-channel output tile and walks K in
// 64-channel stages: the stage's x rows and weight rows are register-staged
// from global memory (coalesced 16-byte loads, one stage ahead) into a 2-slot
// LDS ring with 144-byte rows (conflict-free ds_read_b128 fragment reads),
// 8 waves = 4 voxel quarters x 2 channel halves, 64 voxels x 128 channels
// (8 MFMA tiles of 32 x 32, v_mfma_f32_32x32x16) each.  x is read once per
// 256-channel output tile (twice for 512 / 400 outputs, the two tiles of a
// voxel block run back to back on one XCD: the second read is an L2 hit).
//
// Epilogue (in registers, no LDS): v_permlane32_swap + v_permlane16_swap turn
// each 32 x 32 accumulator (lane = voxel, 16 scattered channels) into lanes of
// 8 consecutive channels of two voxels; then bias, out_scale, ReLU, the ReLU
// mask of a data gradient (y = mask > 0 ? y : 0), the accumulate (y += old y)
// and a 16-byte (bf16 / fp16) or 2 x 16-byte (fp32) store per lane and voxel.
#include "conv_common.h"

namespace {
using namespace vsrk_conv;

constexpr int WT = 512;          // 8 waves
constexpr int WBM = 256;         // voxels per tile
constexpr int WBN = 256;         // output channels per tile
constexpr int WBK = 64;          // input channels per stage
constexpr int WRS = 2 * WBK + 16;  // LDS row stride (bytes): 144 = 36 dwords (see the layout note below)
constexpr int WSLOT = (WBM + WBN) * WRS;  // x rows then weight rows
constexpr int WLDS = 2 * WSLOT;            // 147456 bytes

typedef int wv4i __attribute__((ext_vector_type(4)));
typedef __amdgpu_buffer_rsrc_t WRsrc;
constexpr uint32_t W_OOB = 0x80000000u;
__device__ __forceinline__ WRsrc w_rsrc(const void* base) {
  const uint64_t b = (uint64_t)base;
  const uint64_t u = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(b >> 32)) << 32) |
                     (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)b);
  return __builtin_amdgcn_make_buffer_rsrc((void*)u, 0, 0x7FFFFFF0, 0x00020000);
}
__device__ __forceinline__ uint4 w_bload16(WRsrc r, uint32_t off) {
  return __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 0));
}
__device__ __forceinline__ void w_bstore16(WRsrc r, uint32_t off, uint4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(wv4i, v), r, (int)off, 0, 0);
}

struct WideArgs {
  const char* x;   // voxel v at x + v * xsv (elements), channels contiguous
  char* y;
  const char* msk;
  const void* w;   // packed [cout_rows][cin_pad]
  const float* bias;
  int64_t nvox;
  int xsv, ysv, msv;  // voxel strides (elements)
  int cin, cout, cin_pad, cout_rows;
  int ntn;            // output-channel tiles
  int nstage;         // K stages
  float out_scale;
  int relu_in, relu_out;
};

// LDS layout of a slot: row i (x: voxel i of the tile; weights: output channel
// i of the tile) at i * 144 bytes, its 64 channels as 8 16-byte pieces.  A
// fragment read (ds_read_b128, lane (r, hf) reads piece 2 ks + hf of row
// r0 + r) touches rows r0 .. r0 + 31 at 36-dword strides: 36 r mod 64 over 16
// consecutive rows = 16 distinct multiples of 4, so every 16-lane group of the
// instruction covers all 64 banks once (conflict-free).
template <typename H, bool YF32, bool MASK, bool ACC>
__global__ __launch_bounds__(WT, 1) void pw_wide_kernel(WideArgs a) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int tid = threadIdx.x, lane = tid & 63, r = lane & 31, hf = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;  // voxel quarter (64), channel half (128)
  // tile order: the channel tiles of a voxel block back to back (x re-read from L2)
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int mt = bid / a.ntn, nt = bid - mt * a.ntn;
  const int64_t v0 = (int64_t)mt * WBM;
  const int n0 = nt * WBN;

  // staging roles: 512 threads x 4 pieces of 16 bytes = 256 x rows + 256 weight rows of 64 channels
  // piece p of thread t: row (t + 512 p) >> 3 ... (8 pieces per row): rows 0..255 x, 256..511 weights
  const WRsrc rx = w_rsrc(reinterpret_cast<const H*>(a.x) + v0 * a.xsv);
  const WRsrc rw = w_rsrc(reinterpret_cast<const H*>(a.w) + (int64_t)n0 * a.cin_pad);
  uint4 st[8];  // this thread's 8 pieces of the next stage (4 x, 4 weights)
  auto load_stage = [&](int s) __attribute__((always_inline)) {
    const int k0 = s * WBK;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int i = tid + WT * p, row = i >> 3, pc = i & 7;
      const int c = k0 + 8 * pc;
      const bool ok = v0 + row < a.nvox && c < a.cin;
      st[p] = w_bload16(rx, ok ? 2u * (uint32_t)(row * a.xsv + c) : W_OOB);
    }
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int i = tid + WT * p, row = i >> 3, pc = i & 7;
      const int c = k0 + 8 * pc;
      const bool ok = n0 + row < a.cout_rows && c < a.cin_pad;
      st[4 + p] = w_bload16(rw, ok ? 2u * (uint32_t)(row * a.cin_pad + c) : W_OOB);
    }
  };
  auto put_stage = [&](int slot) __attribute__((always_inline)) {
    char* sl = lds + slot * WSLOT;
#pragma unroll
    for (int p = 0; p < 8; ++p) {
      const int i = tid + WT * (p & 3), row = (i >> 3) + (p >= 4 ? WBM : 0), pc = i & 7;
      uint4 v = st[p];
      if (p < 4 && a.relu_in) {
        float f[8];
        Chunk<H>::unpack(v, f);
#pragma unroll
        for (int e = 0; e < 8; ++e) f[e] = fmaxf(f[e], 0.f);
        v = Chunk<H>::pack(f);
      }
      *reinterpret_cast<uint4*>(sl + row * WRS + pc * 16) = v;
    }
  };

  f32x16 acc[2][4];  // [voxel block][channel block]
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

  // fragment bases (bytes within a slot)
  const uint32_t xb = (uint32_t)((wm * 64 + r) * WRS + hf * 16);
  const uint32_t wb = (uint32_t)((WBM + wn * 128 + r) * WRS + hf * 16);
  load_stage(0);
  put_stage(0);
  if (a.nstage > 1) load_stage(1);
  __syncthreads();
  for (int s = 0; s < a.nstage; ++s) {
    const char* sl = lds + (s & 1) * WSLOT;
    // compute stage s: 4 k-steps of 16 channels
#pragma unroll
    for (int ks = 0; ks < WBK / 16; ++ks) {
      uint4 bx[2], aw[4];
#pragma unroll
      for (int i = 0; i < 2; ++i) bx[i] = *reinterpret_cast<const uint4*>(sl + xb + i * 32 * WRS + ks * 32);
#pragma unroll
      for (int j = 0; j < 4; ++j) aw[j] = *reinterpret_cast<const uint4*>(sl + wb + j * 32 * WRS + ks * 32);
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int i = 0; i < 2; ++i) mma<H>(acc[i][j], aw[j], bx[i]);
    }
    if (s + 1 < a.nstage) {
      // the next stage's registers (loaded one stage ago) into the other slot:
      // every wave finished stage s - 1, which read it (the barrier below)
      put_stage((s + 1) & 1);
      if (s + 2 < a.nstage) load_stage(s + 2);
    }
    __syncthreads();
  }

  // ---- epilogue ----
  const int ecc = 2 * (r >> 4) + hf;  // the lane's 8-channel chunk of a 32-channel block
  const float osc = a.out_scale;
  const WRsrc ry = w_rsrc(reinterpret_cast<const char*>(a.y) +
                          v0 * a.ysv * (int64_t)(YF32 ? 4 : 2));
  const WRsrc rm = w_rsrc(reinterpret_cast<const H*>(MASK ? a.msk : a.y) + v0 * a.msv);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int co = n0 + wn * 128 + j * 32 + 8 * ecc;
    const bool cok = co < a.cout;  // (cout % 8 == 0: whole chunks)
    float bs[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) bs[e] = (a.bias && cok) ? a.bias[co + e] : 0.f;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      float v[16];
#pragma unroll
      for (int e = 0; e < 16; ++e) v[e] = acc[i][j][e];
#pragma unroll
      for (int g = 0; g < 4; g += 2) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const auto sw = __builtin_amdgcn_permlane32_swap(__builtin_bit_cast(uint32_t, v[4 * g + q]),
                                                           __builtin_bit_cast(uint32_t, v[4 * g + 4 + q]), false, false);
          v[4 * g + q] = __builtin_bit_cast(float, (uint32_t)sw[0]);
          v[4 * g + 4 + q] = __builtin_bit_cast(float, (uint32_t)sw[1]);
        }
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const auto sw = __builtin_amdgcn_permlane16_swap(__builtin_bit_cast(uint32_t, v[e]),
                                                         __builtin_bit_cast(uint32_t, v[8 + e]), false, false);
        v[e] = __builtin_bit_cast(float, (uint32_t)sw[0]);
        v[8 + e] = __builtin_bit_cast(float, (uint32_t)sw[1]);
      }
#pragma unroll
      for (int q = 0; q < 2; ++q) {  // voxel wm * 64 + 32 i + (r & 15) + 16 q of the tile
        const int vt = wm * 64 + 32 * i + (r & 15) + 16 * q;
        const bool ok = cok && v0 + vt < a.nvox;
        float t[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          t[e] = (v[8 * q + e] + bs[e]) * osc;
          if (a.relu_out) t[e] = fmaxf(t[e], 0.f);
        }
        if constexpr (MASK) {
          float m[8];
          Chunk<H>::unpack(w_bload16(rm, ok ? 2u * (uint32_t)(vt * a.msv + co) : W_OOB), m);
#pragma unroll
          for (int e = 0; e < 8; ++e) t[e] = m[e] > 0.f ? t[e] : 0.f;
        }
        if constexpr (YF32) {
          const uint32_t off = ok ? 4u * (uint32_t)(vt * a.ysv + co) : W_OOB;
          if constexpr (ACC) {
            const uint4 o0 = w_bload16(ry, off), o1 = w_bload16(ry, ok ? off + 16u : W_OOB);
            t[0] += __builtin_bit_cast(float, o0.x); t[1] += __builtin_bit_cast(float, o0.y);
            t[2] += __builtin_bit_cast(float, o0.z); t[3] += __builtin_bit_cast(float, o0.w);
            t[4] += __builtin_bit_cast(float, o1.x); t[5] += __builtin_bit_cast(float, o1.y);
            t[6] += __builtin_bit_cast(float, o1.z); t[7] += __builtin_bit_cast(float, o1.w);
          }
          w_bstore16(ry, off, make_uint4(__builtin_bit_cast(uint32_t, t[0]), __builtin_bit_cast(uint32_t, t[1]),
                                          __builtin_bit_cast(uint32_t, t[2]), __builtin_bit_cast(uint32_t, t[3])));
          w_bstore16(ry, ok ? off + 16u : W_OOB,
                     make_uint4(__builtin_bit_cast(uint32_t, t[4]), __builtin_bit_cast(uint32_t, t[5]),
                                __builtin_bit_cast(uint32_t, t[6]), __builtin_bit_cast(uint32_t, t[7])));
        } else {
          const uint32_t off = ok ? 2u * (uint32_t)(vt * a.ysv + co) : W_OOB;
          if constexpr (ACC) {
            float o[8];
            Chunk<H>::unpack(w_bload16(ry, off), o);
#pragma unroll
            for (int e = 0; e < 8; ++e) t[e] += o[e];
          }
          w_bstore16(ry, off, Chunk<H>::pack(t));
        }
      }
    }
  }
}

template <typename H, bool YF32, bool MASK, bool ACC>
int launch_wide(const WideArgs& a, int grid, hipStream_t s) {
  auto k = pw_wide_kernel<H, YF32, MASK, ACC>;
  (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, WLDS);
  k<<<grid, WT, WLDS, s>>>(a);
  return VSRK_OK;
}

// voxel-dense view: voxels of (n, d, h, w) at one stride (returned), or 0
int64_t voxel_stride(const vsrk_tensor5* t) {
  if (t->shuffle > 1) return 0;
  const int64_t sw = t->sw;
  if (t->sh != sw * t->w || t->sd != t->sh * t->h || t->sn != t->sd * t->d) {
    // a singleton dimension's stride does not matter
    if (!((t->h == 1 || t->sh == sw * t->w) && (t->d == 1 || t->sd == (int64_t)t->h * t->w * sw) &&
          (t->n == 1 || t->sn == (int64_t)t->d * t->h * t->w * sw)))
      return 0;
  }
  return sw;
}

}  // namespace

int g_pw_wide_mode = -1;  // -1: from VSRK_PW_WIDE (default on), 0 off

// 1 = launched, 0 = not eligible (the caller goes on to the other kernels),
// < 0 = -(error status)
int vsrk_conv_fwd_pw_wide(const vsrk_conv_desc* d, const vsrk_tensor5* x, const void* w_packed, const float* bias,
                          const vsrk_tensor5* residual, const vsrk_tensor5* mask, const vsrk_tensor5* y,
                          hipStream_t s) {
  if (g_pw_wide_mode < 0) {
    const char* e = getenv("VSRK_PW_WIDE");
    g_pw_wide_mode = (e && e[0] == '0') ? 0 : 1;
  }
  if (!g_pw_wide_mode) return 0;
  if (d->kd != 1 || d->kh != 1 || d->kw != 1 || d->pd || d->ph || d->pw) return 0;
  if (!vsrk_is16(x->dtype) || !(y->dtype == x->dtype || y->dtype == VSRK_F32)) return 0;
  // the wide shapes only: more than 256 input channels, or 256 -> >= 256
  if (!(x->c > 256 || (x->c >= 256 && y->c >= 256))) return 0;
  if (residual || d->bias_perm_r > 1 || d->mask_slope) return 0;
  if (d->act != VSRK_ACT_NONE && d->act != VSRK_ACT_RELU) return 0;
  if (d->prologue != VSRK_PRO_NONE && d->prologue != VSRK_PRO_RELU) return 0;
  if (x->c % 8 || y->c % 8) return 0;
  if (x->n != y->n || x->d != y->d || x->h != y->h || x->w != y->w) return 0;
  const int64_t xsv = voxel_stride(x), ysv = voxel_stride(y);
  const int64_t msv = mask ? voxel_stride(mask) : 0;
  if (!xsv || !ysv || (mask && (!msv || mask->dtype != x->dtype || mask->c != y->c || mask->n != y->n ||
                                mask->d != y->d || mask->h != y->h || mask->w != y->w)))
    return 0;
  const int es = vsrk_esize(x->dtype), ys = vsrk_esize(y->dtype);
  if (((uintptr_t)x->ptr) % 16 || ((uintptr_t)y->ptr) % 16 || (mask && ((uintptr_t)mask->ptr) % 16) ||
      (xsv * es) % 16 || (ysv * ys) % 16 || (msv * es) % 16)
    return 0;
  const int64_t nvox = (int64_t)x->n * x->d * x->h * x->w;
  if (nvox == 0) return 1;
  // 32-bit byte offsets inside a tile's buffer window
  if ((int64_t)WBM * std::max(xsv * es, std::max(ysv * ys, msv * es)) >= (1ll << 30)) return 0;
  WideArgs a;
  a.x = (const char*)x->ptr;
  a.y = (char*)y->ptr;
  a.msk = mask ? (const char*)mask->ptr : nullptr;
  a.w = w_packed;
  a.bias = bias;
  a.nvox = nvox;
  a.xsv = (int)xsv;
  a.ysv = (int)ysv;
  a.msv = (int)msv;
  a.cin = x->c;
  a.cout = y->c;
  a.cin_pad = round_up(x->c, 32);
  a.cout_rows = round_up(y->c, 128);
  a.ntn = ceil_div(y->c, WBN);
  a.nstage = ceil_div(a.cin_pad, WBK);
  a.out_scale = d->out_scale;
  a.relu_in = d->prologue == VSRK_PRO_RELU;
  a.relu_out = d->act == VSRK_ACT_RELU;
  const int64_t nblk = ceil_div64(nvox, WBM) * a.ntn;
  if (nblk >= (1ll << 31)) return 0;
  const int grid = (int)nblk;
  const bool yf = y->dtype == VSRK_F32, m = mask != nullptr, acc = d->accumulate != 0;
  const int rc = vsrk_dispatch16(x->dtype, [&](auto tag) {
    using H = decltype(tag);
    if (yf) {
      if (m) return acc ? launch_wide<H, true, true, true>(a, grid, s) : launch_wide<H, true, true, false>(a, grid, s);
      return acc ? launch_wide<H, true, false, true>(a, grid, s) : launch_wide<H, true, false, false>(a, grid, s);
    }
    if (m) return acc ? launch_wide<H, false, true, true>(a, grid, s) : launch_wide<H, false, true, false>(a, grid, s);
    return acc ? launch_wide<H, false, false, true>(a, grid, s) : launch_wide<H, false, false, false>(a, grid, s);
  });
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    vsrk_set_error("conv_fwd(pw_wide): launch failed: %s", hipGetErrorString(e));
    return -(int)VSRK_ERR_LAUNCH;
  }
  return rc == VSRK_OK ? 1 : -rc;
}
