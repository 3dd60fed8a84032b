// Shared device/host helpers for the vsrk HIP kernels (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stddef.h>
#include "../../include/vsrk.h"

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16;
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

// ---- error reporting (thread-local last error string, see vsrk_last_error) ----
void vsrk_set_error(const char* fmt, ...);
#define VSRK_CHECK(cond, ...)                                   \
  do {                                                          \
    if (!(cond)) {                                              \
      vsrk_set_error(__VA_ARGS__);                              \
      return VSRK_ERR_INVALID;                                  \
    }                                                           \
  } while (0)
#define VSRK_LAUNCH_CHECK(name)                                                 \
  do {                                                                          \
    hipError_t _e = hipGetLastError();                                          \
    if (_e != hipSuccess) {                                                     \
      vsrk_set_error("%s: launch failed: %s", name, hipGetErrorString(_e));     \
      return VSRK_ERR_LAUNCH;                                                   \
    }                                                                           \
  } while (0)

// ---- element conversions ----
template <typename T> __device__ __forceinline__ float to_f32(T v);
template <> __device__ __forceinline__ float to_f32<float>(float v) { return v; }
template <> __device__ __forceinline__ float to_f32<bf16>(bf16 v) { return (float)v; }
template <> __device__ __forceinline__ float to_f32<f16>(f16 v) { return (float)v; }
template <typename T> __device__ __forceinline__ T from_f32(float v);
template <> __device__ __forceinline__ float from_f32<float>(float v) { return v; }
template <> __device__ __forceinline__ bf16 from_f32<bf16>(float v) { return (bf16)v; }
template <> __device__ __forceinline__ f16 from_f32<f16>(float v) { return (f16)v; }

// 16-byte chunk <-> float lanes.  A chunk holds 8 bf16 or 4 f32 channels.
template <typename T> struct Chunk;
template <> struct Chunk<bf16> {
  static constexpr int E = 8;
  __device__ static inline void unpack(uint4 v, float* f) {
    const bf16* p = reinterpret_cast<const bf16*>(&v);
#pragma unroll
    for (int i = 0; i < 8; ++i) f[i] = (float)p[i];
  }
  __device__ static inline uint4 pack(const float* f) {
    uint4 v;
    bf16* p = reinterpret_cast<bf16*>(&v);
#pragma unroll
    for (int i = 0; i < 8; ++i) p[i] = (bf16)f[i];
    return v;
  }
};
template <> struct Chunk<f16> {
  static constexpr int E = 8;
  __device__ static inline void unpack(uint4 v, float* f) {
    const f16* p = reinterpret_cast<const f16*>(&v);
#pragma unroll
    for (int i = 0; i < 8; ++i) f[i] = (float)p[i];
  }
  __device__ static inline uint4 pack(const float* f) {
    uint4 v;
    f16* p = reinterpret_cast<f16*>(&v);
#pragma unroll
    for (int i = 0; i < 8; ++i) p[i] = (f16)f[i];
    return v;
  }
};
template <> struct Chunk<float> {
  static constexpr int E = 4;
  __device__ static inline void unpack(uint4 v, float* f) {
    const float* p = reinterpret_cast<const float*>(&v);
#pragma unroll
    for (int i = 0; i < 4; ++i) f[i] = p[i];
  }
  __device__ static inline uint4 pack(const float* f) {
    uint4 v;
    float* p = reinterpret_cast<float*>(&v);
#pragma unroll
    for (int i = 0; i < 4; ++i) p[i] = f[i];
    return v;
  }
};

__host__ __device__ inline int64_t ceil_div64(int64_t a, int64_t b) { return (a + b - 1) / b; }
__host__ __device__ inline int ceil_div(int a, int b) { return (a + b - 1) / b; }
__host__ __device__ inline int round_up(int a, int b) { return ceil_div(a, b) * b; }

// Channels-last element offset of logical (n,d,h,w,c) in a view; honours the
// sub-pixel ("shuffle") addressing mode of vsrk_tensor5 (see include/vsrk.h).
struct View {
  char* ptr;
  int n, d, h, w, c;
  int64_t sn, sd, sh, sw;
  int r;       // sub-pixel factor (1 = plain)
  int cphys;   // physical channels per sub-pixel = c / (r*r)
};
inline View make_view(const vsrk_tensor5* t) {
  View v;
  v.ptr = (char*)t->ptr;
  v.n = t->n; v.d = t->d; v.h = t->h; v.w = t->w; v.c = t->c;
  v.sn = t->sn; v.sd = t->sd; v.sh = t->sh; v.sw = t->sw;
  v.r = t->shuffle > 1 ? t->shuffle : 1;
  v.cphys = v.c / (v.r * v.r);
  return v;
}
// element offset (not bytes) of (n,d,h,w,c)
__device__ __forceinline__ int64_t view_off(const View& v, int n, int d, int h, int w, int c) {
  if (v.r == 1) return n * v.sn + d * v.sd + h * v.sh + w * v.sw + c;
  int sub = c / v.cphys;
  int cc = c - sub * v.cphys;
  int i = sub / v.r, j = sub - (sub / v.r) * v.r;
  return n * v.sn + d * v.sd + (int64_t)(h * v.r + i) * v.sh + (int64_t)(w * v.r + j) * v.sw + cc;
}

// ---- PReLU slope gradient partials ----
// The fused and separate PReLU backward kernels (drf.hip, conv_roll.hip,
// conv_pw.hip) reduce sum_{x<0} g x to one double per wave (or workgroup)
// in a fixed order; vsrk_slope_final (drf.hip) sums those in a fixed order
// into *da.  (A last-workgroup finish inside the producing kernel needs an
// agent-scope release per workgroup -- an L2 writeback on gfx950 -- and made
// the DRF step 20 % slower; the per-lane float partials of round 4 made the
// final launch read 64 K floats, 19 us each.)
__device__ __forceinline__ double vsrk_wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// ---- host-side dtype helpers ----
// 16-bit storage types (bf16, fp16) share every kernel family; the MFMA
// flavour follows the type (v_mfma_f32_32x32x16_bf16 / _f16).
static inline bool vsrk_is16(int dt) { return dt == VSRK_BF16 || dt == VSRK_F16; }
static inline int vsrk_esize(int dt) { return dt == VSRK_F32 ? 4 : 2; }
// Call f(tag) with a value of the 16-bit element type of dtype dt.
template <typename Fn>
static inline auto vsrk_dispatch16(int dt, Fn&& f) {
  if (dt == VSRK_F16) return f(f16{});
  return f(bf16{});
}
