// Measured peaks of this device for the roofline fractions bench.py reports
// ("re-measure with a GEMM microbench on the box"): the dense
// bf16 MFMA rate (v_mfma_f32_32x32x16_bf16 back to back on register
// operands, four independent accumulators per wave, two waves per SIMD on
// every CU) and the HBM copy rate (16-byte loads, four in flight per thread,
// grid-stride, read + write counted).  Not on the product path.
#include "vsrk_common.h"

namespace {

__global__ __launch_bounds__(256) void peak_mfma_kernel(int iters, float* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  bf16x8 a, b;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    // random-looking finite operands (the clock under load depends on the data)
    a[e] = (__bf16)(0.01f * (float)((lane * 37 + e * 11) % 29) - 0.14f);
    b[e] = (__bf16)(0.01f * (float)((lane * 13 + e * 7) % 31) - 0.15f);
  }
  f32x16 c0 = {}, c1 = {}, c2 = {}, c3 = {};
  for (int i = 0; i < iters; ++i) {
    c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b, a, c1, 0, 0, 0);
    c2 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, a, c2, 0, 0, 0);
    c3 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b, b, c3, 0, 0, 0);
  }
  float s = 0.f;
#pragma unroll
  for (int e = 0; e < 16; ++e) s += c0[e] + c1[e] + c2[e] + c3[e];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void peak_copy_kernel(const uint4* __restrict__ src, uint4* __restrict__ dst,
                                                        int64_t n) {
  constexpr int U = 4;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += U * stride) {
    uint4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (i + u * stride < n) v[u] = src[i + u * stride];
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (i + u * stride < n) dst[i + u * stride] = v[u];
  }
}

// Block-contiguous form: each workgroup copies one contiguous chunk of
// 256 x U x 16 bytes, U loads in flight per lane before the stores; non-
// temporal loads and stores (each byte is touched once).  The grid covers the
// whole buffer (no grid-stride loop).  Round 5, 2 GiB copy, best of 10, read
// + write bytes: U = 4 6.22-6.30 TB/s (MI355X_MICROARCH.md: 6.29 measured),
// U = 8 4.2-4.3, the grid-stride peak_copy_kernel (PEAK_COPY 0) 4.7.
typedef uint32_t pk_u32x4 __attribute__((ext_vector_type(4)));
template <int U>
__global__ __launch_bounds__(256) void peak_copy_chunk_kernel(const pk_u32x4* __restrict__ src,
                                                              pk_u32x4* __restrict__ dst, int64_t n) {
  const int64_t base = (int64_t)blockIdx.x * 256 * U + threadIdx.x;
  pk_u32x4 v[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t i = base + u * 256;
    if (i < n) v[u] = __builtin_nontemporal_load(src + i);
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t i = base + u * 256;
    if (i < n) __builtin_nontemporal_store(v[u], dst + i);
  }
}

int num_cus() {
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) !=
                                              hipSuccess)
    return 0;
  return cus;
}

}  // namespace

extern "C" int32_t vsrk_peak_mfma_blocks(void) { return 2 * num_cus(); }

extern "C" int vsrk_peak_mfma(int32_t iters, float* out, void* stream) {
  VSRK_CHECK(out && iters > 0, "peak_mfma: bad argument");
  const int blocks = 2 * num_cus();
  VSRK_CHECK(blocks > 0, "peak_mfma: no device");
  peak_mfma_kernel<<<blocks, 256, 0, (hipStream_t)stream>>>(iters, out);
  VSRK_LAUNCH_CHECK("peak_mfma");
  return VSRK_OK;
}

extern "C" int vsrk_peak_copy(const void* src, void* dst, int64_t bytes, void* stream) {
  VSRK_CHECK(src && dst && bytes > 0 && bytes % 16 == 0, "peak_copy: bad argument");
  const int64_t n = bytes / 16;
#ifndef PEAK_COPY
#define PEAK_COPY 1
#endif
  if (PEAK_COPY == 0) {
    const int blocks = 8 * num_cus();
    VSRK_CHECK(blocks > 0, "peak_copy: no device");
    peak_copy_kernel<<<blocks, 256, 0, (hipStream_t)stream>>>(reinterpret_cast<const uint4*>(src),
                                                             reinterpret_cast<uint4*>(dst), n);
  } else {
    constexpr int U = PEAK_COPY == 1 ? 4 : 8;
    const int64_t blocks = (n + 256 * U - 1) / (256 * U);
    VSRK_CHECK(blocks < (1ll << 31), "peak_copy: buffer too large");
    peak_copy_chunk_kernel<U><<<(unsigned)blocks, 256, 0, (hipStream_t)stream>>>(
        reinterpret_cast<const pk_u32x4*>(src), reinterpret_cast<pk_u32x4*>(dst), n);
  }
  VSRK_LAUNCH_CHECK("peak_copy");
  return VSRK_OK;
}
