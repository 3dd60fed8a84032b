// Probe of two CDNA4 primitives the k3 conv kernel relies on:
//  (1) __builtin_amdgcn_permlane32_swap(vdst, src) lane semantics;
//  (2) buffer_load_dwordx4 ... lds with an out-of-range voffset (+ soffset):
//      zeros land in LDS, in-range lanes land at M0 + 16 * lane.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
typedef int32_t i32x4 __attribute__((ext_vector_type(4)));

__global__ void swap_probe(int* out) {
  const int l = threadIdx.x;
  int a = 1000 + l, b = 2000 + l;
  auto r = __builtin_amdgcn_permlane32_swap(a, b, false, false);
  out[l] = r[0];
  out[64 + l] = r[1];
}

__global__ void dma_probe(const int* src, int* out, uint32_t soff) {
  __shared__ __attribute__((aligned(16))) int lds[64 * 4 * 2];
  for (int i = threadIdx.x; i < 512; i += 64) lds[i] = -7;
  __syncthreads();
  const uint64_t b = (uint64_t)src;
  i32x4 r;
  r[0] = (int)(uint32_t)b;
  r[1] = (int)(uint32_t)(b >> 32) & 0xffff;
  r[2] = 0x7FFFFFF0;
  r[3] = 0x00020000;
  const int l = threadIdx.x;
  uint32_t voff = (l % 3 == 2) ? 0x80000000u : (uint32_t)(l * 16);
  uint32_t base = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) int*)lds + 1024;
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %4\n\ts_nop 0\n\t"
      "buffer_load_dwordx4 %1, %2, %3 offen lds\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(r), "s"(__builtin_amdgcn_readfirstlane(soff)), "s"(__builtin_amdgcn_readfirstlane(base)));
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int i = threadIdx.x; i < 512; i += 64) out[i] = lds[i];
}

int main() {
  int *d, *dsrc;
  hipMalloc(&d, 4096);
  hipMalloc(&dsrc, 8192);
  std::vector<int> h(2048);
  for (int i = 0; i < 2048; ++i) h[i] = i;
  hipMemcpy(dsrc, h.data(), 8192, hipMemcpyHostToDevice);
  swap_probe<<<1, 64>>>(d);
  hipMemcpy(h.data(), d, 512, hipMemcpyDeviceToHost);
  printf("swap r0: lane0=%d lane31=%d lane32=%d lane63=%d\n", h[0], h[31], h[32], h[63]);
  printf("swap r1: lane0=%d lane31=%d lane32=%d lane63=%d\n", h[64], h[95], h[96], h[127]);
  dma_probe<<<1, 64>>>(dsrc, d, 64);  // soffset 64 bytes = 16 ints
  hipMemcpy(h.data(), d, 2048, hipMemcpyDeviceToHost);
  printf("dma lds[0..3]=%d %d %d %d (expect -7: below M0 base)\n", h[0], h[1], h[2], h[3]);
  for (int l = 0; l < 6; ++l)
    printf("dma lane %d -> lds[%d..]: %d %d %d %d (expect %s)\n", l, 256 + 4 * l, h[256 + 4 * l], h[257 + 4 * l],
           h[258 + 4 * l], h[259 + 4 * l], l % 3 == 2 ? "zeros" : "src[16 + 4l ...]");
  hipError_t e = hipDeviceSynchronize();
  printf("status %s\n", hipGetErrorString(e));
  return 0;
}
