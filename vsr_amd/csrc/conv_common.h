// Shared pieces of the implicit-GEMM convolution kernels (conv_fwd.hip,
// conv_wgrad.hip).  See conv_fwd.hip for the design notes.
#pragma once
#include "vsrk_common.h"
#include "vsrk_internal.h"
#include <type_traits>

namespace vsrk_conv {


constexpr int NTHR = 512;  // 8 waves per workgroup
constexpr int TW = 32;     // tile columns = one MFMA column block
constexpr int GTH = 8;     // weight-gradient tile rows: 8 x 32 = 256 voxels
constexpr int ROWB = 80;   // forward LDS bytes per staged input row (64 data + 16 pad)
constexpr int GTHR = 256;  // weight-gradient workgroup: 4 waves, one per SIMD (512 VGPRs each)
constexpr int MAXK = 3;    // kh, kw <= 3

// XCD-aware block order: under round-robin dispatch blocks b and b+8 share an
// XCD; give each XCD a contiguous range of logical tiles so neighbouring
// tiles' halo rows and the shared weight slices are re-read from one L2.
// Bijective for any grid size (speed only, never correctness).
__device__ __forceinline__ int xcd_remap(int bid, int nblk) {
  const int xcd = bid & 7, q = nblk >> 3, rr = nblk & 7;
  const int base = xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q;
  return base + (bid >> 3);
}

struct ConvArgs {
  View x, y, res, msk;
  const char* w;
  const float* bias;
  const float* pro_scale;
  const float* pro_shift;
  int cin, cout, cin_pad, cout_pad;
  int kd, kh, kw, pd, ph, pw;
  int prologue, act, accumulate, has_res, has_mask, xvec, bias_r;
  float out_scale;
  const float* act_param;   // PReLU slope (device scalar)
  const float* mask_slope;  // masked-off scale (device scalar) or null (0)
  int tiles_h, tiles_w, ntn, nblk;
  int ntiles;  // output tiles (incl. N tiles) walked by the persistent grid
};

// Zero the channels of a chunk at or beyond `nvalid` (the partial last chunk
// of a view whose storage is padded: padding may hold anything).
template <typename T>
__device__ __forceinline__ uint4 mask_tail(uint4 v, int nvalid) {
  constexpr int E = Chunk<T>::E;
  if (nvalid >= E) return v;
  float f[E];
  Chunk<T>::unpack(v, f);
#pragma unroll
  for (int e = 0; e < E; ++e) f[e] = e < nvalid ? f[e] : 0.f;
  return Chunk<T>::pack(f);
}

// Raw 16-byte chunk of channels [c, c+E) at logical voxel (n,d,h,w): one vector
// load when the view allows it, else element loads (zero past cin).
template <typename T>
__device__ __forceinline__ uint4 load_raw(const View& v, int n, int d, int h, int w, int c, int cin, bool vec) {
  constexpr int E = Chunk<T>::E;
  const T* p = reinterpret_cast<const T*>(v.ptr) + view_off(v, n, d, h, w, c);
  if (vec && c + E <= cin) return *reinterpret_cast<const uint4*>(p);
  float f[E];
#pragma unroll
  for (int e = 0; e < E; ++e) f[e] = (c + e < cin) ? to_f32<T>(p[e]) : 0.f;
  return Chunk<T>::pack(f);
}

// Per-channel affine + optional ReLU (a fused BatchNorm+ReLU) with scale/shift
// staged in LDS: real channels carry (scale, shift) — (1, 0) for a ReLU-only
// prologue — padding channels carry (0, 0), so the transform is branchless and
// padding stays zero.
template <typename T>
__device__ __forceinline__ uint4 prologue_lds(uint4 v, int c, bool relu, const float* lsc, const float* lsh) {
  constexpr int E = Chunk<T>::E;
  float f[E];
  Chunk<T>::unpack(v, f);
#pragma unroll
  for (int e = 0; e < E; ++e) {
    float t = fmaf(f[e], lsc[c + e], lsh[c + e]);
    f[e] = relu ? fmaxf(t, 0.f) : t;
  }
  return Chunk<T>::pack(f);
}

// Stage the prologue's per-channel (scale, shift) into LDS, zero-padded to cpad.
__device__ __forceinline__ void stage_prologue(float* lsc, float* lsh, int mode, const float* sc, const float* sh,
                                               int cin, int cpad, int tid, int nthr) {
  for (int i = tid; i < cpad; i += nthr) {
    const bool ok = i < cin;
    const bool aff = (mode & VSRK_PRO_AFFINE) != 0;
    lsc[i] = ok ? (aff ? sc[i] : 1.f) : 0.f;
    lsh[i] = ok ? (aff ? sh[i] : 0.f) : 0.f;
  }
}

// One 16-byte-per-lane LDS-DMA (global_load_lds_dwordx4): lane l's 16 bytes
// from `gsrc` land at LDS byte address lds_base + 16*l.  Written as inline asm
// so hipcc does not track it: with the builtin, hipcc cannot tell the DMA's
// target buffer from the one being read and drains it (s_waitcnt vmcnt(0))
// before the first ds_read of the stage, serialising every load with the
// MFMAs it should overlap.  The caller retires it with its own
// `s_waitcnt vmcnt` + barrier before reading the buffer.  M0 is set and
// restored inside the statement (hipcc reserves it).
__device__ __forceinline__ void glds16(const void* gsrc, uint32_t lds_base) {
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %2\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %1, off\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(gsrc), "s"(lds_base)
      : "memory");
}
// glds16 without saving / restoring M0: for kernels in which nothing else
// uses M0 (checked in their ISA: conv_roll.hip, conv_wgrad_roll.hip) -- two
// scalar instructions less per 1 KB piece
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
__device__ __forceinline__ void glds16_m0(const void* gsrc, uint32_t lds_base) {
  asm volatile(
      "s_mov_b32 m0, %1\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %0, off"
      :
      : "v"(gsrc), "s"(lds_base)
      : "memory", "m0");
}
#pragma clang diagnostic pop
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)(p);
}

// Epilogue activation / mask helpers shared by the conv kernels.
__device__ __forceinline__ float act_apply(int act, float t, float slope) {
  if (act == VSRK_ACT_RELU) return fmaxf(t, 0.f);
  if (act == VSRK_ACT_PRELU) return t > 0.f ? t : slope * t;
  return t;
}
__device__ __forceinline__ float mask_apply(float m, float t, float mslope) {
  return m > 0.f ? t : (mslope != 0.f ? mslope * t : 0.f);
}

// acc += W(32 rows of co, 16-byte k slice) x X(16-byte k slice, 32 voxels)
template <typename T>
__device__ __forceinline__ void mma(f32x16& acc, uint4 a, uint4 b);
template <>
__device__ __forceinline__ void mma<bf16>(f32x16& acc, uint4 a, uint4 b) {
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a),
                                                __builtin_bit_cast(bf16x8, b), acc, 0, 0, 0);
}
template <>
__device__ __forceinline__ void mma<f16>(f32x16& acc, uint4 a, uint4 b) {
  acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), acc, 0,
                                               0, 0);
}
template <>
__device__ __forceinline__ void mma<float>(f32x16& acc, uint4 a, uint4 b) {
  // lane half hf supplies k = 4*hf + j for MFMA j on both operands, so the
  // four k=2 products cover the 8 channels of the slice exactly once.
  acc = __builtin_amdgcn_mfma_f32_32x32x2f32(__builtin_bit_cast(float, a.x), __builtin_bit_cast(float, b.x), acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x2f32(__builtin_bit_cast(float, a.y), __builtin_bit_cast(float, b.y), acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x2f32(__builtin_bit_cast(float, a.z), __builtin_bit_cast(float, b.z), acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x2f32(__builtin_bit_cast(float, a.w), __builtin_bit_cast(float, b.w), acc, 0, 0, 0);
}

// 8-element 16-bit MFMA operand vectors per element type, and the matching
// v_mfma_f32_32x32x16_{bf16,f16}
template <typename H> struct V8;
template <> struct V8<bf16> { typedef bf16x8 type; };
template <> struct V8<f16> { typedef f16x8 type; };
__device__ __forceinline__ f32x16 mfma32x16(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x16 mfma32x16(f16x8 a, f16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}

// 4 consecutive channels of an epilogue tensor, kept packed (uint2 for bf16,
// uint4 for fp32) between the batched loads and the stores.
template <typename YT, typename Pk>
__device__ __forceinline__ Pk load_pk(const char* base, int64_t off, bool vec, int valid) {
  const YT* p = reinterpret_cast<const YT*>(base) + off;
  if (vec) return *reinterpret_cast<const Pk*>(p);
  Pk v;
  YT* q = reinterpret_cast<YT*>(&v);
  for (int e = 0; e < 4; ++e) q[e] = e < valid ? p[e] : from_f32<YT>(0.f);
  return v;
}
template <typename YT, typename Pk>
__device__ __forceinline__ void unpack_pk(Pk v, float* f) {
  const YT* q = reinterpret_cast<const YT*>(&v);
#pragma unroll
  for (int e = 0; e < 4; ++e) f[e] = to_f32<YT>(q[e]);
}
template <typename YT>
__device__ __forceinline__ void unpack_pk(uint2 v, float* f) { unpack_pk<YT, uint2>(v, f); }
template <typename YT>
__device__ __forceinline__ void unpack_pk(uint4 v, float* f) { unpack_pk<YT, uint4>(v, f); }
template <typename YT, typename Pk>
__device__ __forceinline__ Pk pack_pk(const float* f) {
  Pk v;
  YT* q = reinterpret_cast<YT*>(&v);
#pragma unroll
  for (int e = 0; e < 4; ++e) q[e] = from_f32<YT>(f[e]);
  return v;
}

template <typename YT>
__device__ __forceinline__ void load4(const char* base, int64_t off, bool vec, int valid, float* v) {
  const YT* p = reinterpret_cast<const YT*>(base) + off;
  if (vec) {
    if constexpr (sizeof(YT) == 4) {
      float4 t = *reinterpret_cast<const float4*>(p);
      v[0] = t.x; v[1] = t.y; v[2] = t.z; v[3] = t.w;
    } else {
      uint2 t = *reinterpret_cast<const uint2*>(p);
      const YT* b = reinterpret_cast<const YT*>(&t);
      for (int e = 0; e < 4; ++e) v[e] = to_f32<YT>(b[e]);
    }
  } else {
    for (int e = 0; e < 4; ++e) v[e] = e < valid ? to_f32<YT>(p[e]) : 0.f;
  }
}

struct WgradArgs {
  View x, dy;
  const float* pro_scale;
  const float* pro_shift;
  float* ws;
  int cin, cout;
  int kd, kh, kw, pd, ph, pw;
  int prologue, xvec, dyvec;
  int tiles_h, tiles_w, ntiles, tiles_per_split, nsplit, ncombos, nblk;
  int n_ci_chunks, n_co_tiles, kd_bias, slab, want_bias, cin_pad;
  // sub-pixel weight (desc->subpixel): taps with a nonzero weight per
  // 32-channel block of the shuffled operand (dy: sp_by 1, x: sp_by 2);
  // the others' gradients are structurally discarded (vsrk_subpixel_wgrad_fold)
  int sp_by;
  uint16_t sptap[64];
};

typedef short v4i16 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4i16 lds_v4i16;

__device__ __forceinline__ v4i16 ds_read_tr(const char* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)(p));
}

}  // namespace vsrk_conv



// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
// Can the kernels read this view in 16-byte chunks?  (aligned base, strides
// and channel count multiples of one chunk; sub-pixel blocks chunk-aligned)
static inline bool chunk_ok(const vsrk_tensor5* t, int esize) {
  // Whole 16-byte chunks may be read at every chunk-aligned channel: aligned
  // base and strides.  c need not be a multiple of a chunk (channels past c
  // are masked), but a sub-pixel block must be.
  const int epc = 16 / esize;
  const int r = t->shuffle > 1 ? t->shuffle : 1;
  const bool block_ok = r == 1 || (t->c / (r * r)) % epc == 0;
  const bool stride_ok = t->sw >= epc || (t->w == 1);
  return ((uintptr_t)t->ptr) % 16 == 0 && t->sn % epc == 0 && t->sd % epc == 0 && t->sh % epc == 0 &&
         t->sw % epc == 0 && block_ok && stride_ok;
}

// Tap mask (bit kh*3 + kw of the PACKED weight) of sub-pixel phase `sub` for
// a VSRK_SUBPIXEL(k, s, p, transposed, flipped) weight: the kernel row of tap
// kh at phase row si is s*(kh - 1) + si + p (strided conv) or s*(1 - kh) + si
// + p (transposed), as vsrk_subpixel_conv_weight builds it (drf.hip); a mode-1
// packing flips the taps.  All taps when the descriptor carries no structure.
static inline uint16_t subpixel_tapmask(int32_t code, int r, int sub) {
  if (code == 0) return 0x1ff;
  const int k = code & 0xff, sp = (code >> 8) & 0xff, p = (code >> 16) & 0xff;
  const bool tr = (code >> 24) & 1, flip = (code >> 25) & 1;
  if (sp != r) return 0x1ff;
  const int si = sub / r, sj = sub % r;
  auto row = [&](int tap, int ph) { return tr ? sp * (1 - tap) + ph + p : sp * (tap - 1) + ph + p; };
  uint16_t m = 0;
  for (int kh = 0; kh < 3; ++kh)
    for (int kw = 0; kw < 3; ++kw) {
      const int th = flip ? 2 - kh : kh, tw = flip ? 2 - kw : kw;
      const int ky = row(th, si), kx = row(tw, sj);
      if (ky >= 0 && ky < k && kx >= 0 && kx < k) m |= (uint16_t)(1u << (kh * 3 + kw));
    }
  return m;
}

// pipelined 16-bit 3x3(x3) weight gradient (conv_wgrad_pipe.hip): 1 = launched the slab kernel, 0 = not eligible.
int vsrk_conv_wgrad_pipe(const vsrk_conv::WgradArgs& a, int nco, int nci, int dtype, hipStream_t s);
// rolling-depth 16-bit Conv3d 3x3x3 weight gradient (conv_wgrad_roll.hip):
// plan (false = not eligible) and launch (1 = launched the slab kernel, whose
// slabs wgrad_reduce_kernel sums over 2 * nsplit splits and 3 * nci * nco
// combos; 0 = not eligible)
bool vsrk_wgrad_roll_plan(const vsrk_conv_desc* d, const vsrk_tensor5* x, const vsrk_tensor5* dy, int* nsplit,
                          int* tps, int* ntiles, int* dzc, size_t* ws_bytes);
int vsrk_conv_wgrad_roll(const vsrk_conv_desc* d, const vsrk_tensor5* x, const vsrk_tensor5* dy,
                         const float* pro_scale, const float* pro_shift, int want_bias, float* ws, size_t ws_bytes,
                         int* nsplit_out, hipStream_t s);
void vsrk_conv_set_wgrad_roll_mode(int mode);
extern int vsrk_g_roll_dz;  // vsrk_conv_set_roll_depth (conv_roll.hip)
// rolling-row 16-bit Conv2d 3x3 weight gradient (conv_wgrad_row.hip): plan
// (false = not eligible) and launch (1 = launched the slab kernel, whose slabs
// wgrad_reduce_kernel sums over nsplit splits and ncot * ncic combos of
// cot_w x 64 channels; 0 = not eligible)
struct VsrkRowPlan {
  int bands, band_h, nseg, ncot, ncic, nsplit;
  int cot_w, slab;  // output channels per combo, floats per slab
  size_t ws_bytes;
};
bool vsrk_wgrad_row_plan(const vsrk_conv_desc* d, const vsrk_tensor5* x, const vsrk_tensor5* dy, VsrkRowPlan* p);
int vsrk_conv_wgrad_row(const vsrk_conv_desc* d, const vsrk_tensor5* x, const vsrk_tensor5* dy, int want_bias,
                        float* ws, size_t ws_bytes, VsrkRowPlan* plan, hipStream_t s);
void vsrk_conv_set_wgrad_row_mode(int mode);
// thin-channel weight gradient (conv_thin.hip): 1 = launched the slab kernel, 0 = not eligible.
int vsrk_conv_wgrad_thin(const vsrk_conv::WgradArgs& a, int nco, int nci, int perm_r, int dtype, hipStream_t s);

static inline bool view_ok(const vsrk_tensor5* t, const char* what) {
  if (!t || !t->ptr) {
    vsrk_set_error("%s: null view", what);
    return false;
  }
  const int r = t->shuffle > 1 ? t->shuffle : 1;
  if (t->c % (r * r) != 0 || (r > 1 && (t->c / (r * r)) % 8 != 0)) {
    vsrk_set_error("%s: sub-pixel view needs channels divisible by 8*shuffle^2 (c=%d, r=%d)", what, t->c, r);
    return false;
  }
  return true;
}

