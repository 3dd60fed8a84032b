// Batched window / crop / flip gather of training samples from HBM-resident
// cine volumes (include/vsrk_data.h).  One thread per output voxel, the
// sample's index map read once per thread from a 24-byte record (L1/L2
// broadcast); consecutive threads walk x, so loads and stores are coalesced
// (reversed for a horizontal flip, still one cache line per 16 lanes).
#include "vsrk_common.h"
#include "../../include/vsrk_data.h"

namespace {

__global__ __launch_bounds__(256) void gather_windows_kernel(const float* __restrict__ src, int T, int h, int w,
                                                             const int* __restrict__ map, int frames, int oh, int ow,
                                                             int64_t total, float* __restrict__ dst) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int x = (int)(i % ow);
  int64_t r = i / ow;
  const int y = (int)(r % oh);
  r /= oh;
  const int t = (int)(r % frames);
  const int b = (int)(r / frames);
  const int* m = map + 6 * b;
  const int vol = m[0], t0 = m[1], y0 = m[2], dy = m[3], x0 = m[4], dx = m[5];
  int ts = (t0 + t) % T;
  if (ts < 0) ts += T;
  const int ys = y0 + dy * y, xs = x0 + dx * x;
  dst[i] = src[(((int64_t)vol * T + ts) * h + ys) * w + xs];
}

}  // namespace

extern "C" int vsrk_gather_windows(const float* src, int32_t nvol, int32_t T, int32_t h, int32_t w,
                                   const int32_t* map, int32_t nb, int32_t frames, int32_t oh, int32_t ow, float* dst,
                                   void* stream) {
  VSRK_CHECK(src && map && dst, "gather_windows: null argument");
  VSRK_CHECK(nvol > 0 && T > 0 && h > 0 && w > 0 && nb >= 0 && frames > 0 && oh > 0 && ow > 0 && oh <= h && ow <= w,
             "gather_windows: bad shape");
  const int64_t total = (int64_t)nb * frames * oh * ow;
  if (total == 0) return VSRK_OK;
  const int64_t blocks = (total + 255) / 256;
  VSRK_CHECK(blocks < (1ll << 31), "gather_windows: too large");
  gather_windows_kernel<<<(unsigned)blocks, 256, 0, (hipStream_t)stream>>>(src, T, h, w, map, frames, oh, ow, total,
                                                                           dst);
  VSRK_LAUNCH_CHECK("gather_windows");
  return VSRK_OK;
}
