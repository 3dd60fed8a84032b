// SSIM (src/model/metrics.py:39-113), fused: [denormalize (utils.py:1-20),]
// the five depthwise 11x11 Gaussian filters (mu1, mu2, E[x^2], E[y^2], E[xy];
// valid convolution, no padding), the SSIM map and its mean, in one pass over
// the images plus a fixed-order final reduction.
//
// The reference builds its window as exp(-((x - 5) / (2 * 1.5))^2) per axis
// (metrics.py:74 -- note 2*sigma inside the square), takes the outer product
// and normalises it to sum 1; that product of two normalised 1-D windows is
// applied here separably (rows, then columns) from an LDS tile:
//   tile = 16 x 32 output pixels of one (n, c) image, input tile 26 x 42,
//   horizontal pass -> 26 x 32 x 5 partial moments in LDS, vertical pass ->
//   per-pixel SSIM -> block sum -> partial[n][tile] (double).
#include "vsrk_common.h"
#include "vsrk_internal.h"

namespace {

constexpr int SW = 11;  // window size (metrics.py:68)
constexpr int TX = 32, TY = 16;
constexpr int IX = TX + SW - 1, IY = TY + SW - 1;

struct SsimArgs {
  const float* out;
  const float* tgt;
  int h, w, ho, wo, channels;
  int denorm;
  float mean, std, c1, c2;
  float g[SW];
  int tiles_x, tiles_y;
};

__global__ __launch_bounds__(256) void ssim_partial_kernel(SsimArgs a, double* __restrict__ part) {
  __shared__ float sx[IY][IX], sy[IY][IX];
  __shared__ float hm[5][IY][TX];
  const int img = blockIdx.z;  // n * channels + c
  const int x0 = blockIdx.x * TX, y0 = blockIdx.y * TY;
  const float* po = a.out + (int64_t)img * a.h * a.w;
  const float* pt = a.tgt + (int64_t)img * a.h * a.w;
  for (int i = threadIdx.x; i < IY * IX; i += blockDim.x) {
    const int yy = i / IX, xx = i - yy * IX;
    const int gy = y0 + yy, gx = x0 + xx;
    float u = 0.f, v = 0.f;
    if (gy < a.h && gx < a.w) {
      u = po[(int64_t)gy * a.w + gx];
      v = pt[(int64_t)gy * a.w + gx];
      if (a.denorm) {
        u = fminf(fmaxf(rintf(u * a.std + a.mean), 0.f), 255.f);
        v = fminf(fmaxf(rintf(v * a.std + a.mean), 0.f), 255.f);
      }
    }
    sx[yy][xx] = u;
    sy[yy][xx] = v;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < IY * TX; i += blockDim.x) {
    const int yy = i / TX, xx = i - yy * TX;
    float m1 = 0.f, m2 = 0.f, s11 = 0.f, s22 = 0.f, s12 = 0.f;
#pragma unroll
    for (int k = 0; k < SW; ++k) {
      const float gk = a.g[k], u = sx[yy][xx + k], v = sy[yy][xx + k];
      m1 = fmaf(gk, u, m1);
      m2 = fmaf(gk, v, m2);
      s11 = fmaf(gk, u * u, s11);
      s22 = fmaf(gk, v * v, s22);
      s12 = fmaf(gk, u * v, s12);
    }
    hm[0][yy][xx] = m1;
    hm[1][yy][xx] = m2;
    hm[2][yy][xx] = s11;
    hm[3][yy][xx] = s22;
    hm[4][yy][xx] = s12;
  }
  __syncthreads();
  double acc = 0.0;
  for (int i = threadIdx.x; i < TY * TX; i += blockDim.x) {
    const int yy = i / TX, xx = i - yy * TX;
    if (y0 + yy >= a.ho || x0 + xx >= a.wo) continue;
    float q[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < SW; ++k) {
      const float gk = a.g[k];
#pragma unroll
      for (int m = 0; m < 5; ++m) q[m] = fmaf(gk, hm[m][yy + k][xx], q[m]);
    }
    const float mu1 = q[0], mu2 = q[1];
    const float s1 = q[2] - mu1 * mu1, s2 = q[3] - mu2 * mu2, s12 = q[4] - mu1 * mu2;
    const float num = (2.f * mu1 * mu2 + a.c1) * (2.f * s12 + a.c2);
    const float den = (mu1 * mu1 + mu2 * mu2 + a.c1) * (s1 + s2 + a.c2);
    acc += (double)(num / den);
  }
  __shared__ double red[256];
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int k = 128; k > 0; k >>= 1) {
    if (threadIdx.x < k) red[threadIdx.x] += red[threadIdx.x + k];
    __syncthreads();
  }
  if (threadIdx.x == 0) part[((int64_t)img * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x] = red[0];
}

// per sample n: sum over its channels' tiles (fixed order) / (C * ho * wo)
__global__ void ssim_final_kernel(const double* __restrict__ part, int batch, int per_sample_tiles, double count,
                                  float* __restrict__ per, float* __restrict__ mean_out) {
  if (threadIdx.x != 0) return;
  double all = 0.0;
  for (int b = 0; b < batch; ++b) {
    double s = 0.0;
    for (int k = 0; k < per_sample_tiles; ++k) s += part[(int64_t)b * per_sample_tiles + k];
    per[b] = (float)(s / count);
    all += s;
  }
  *mean_out = (float)(all / (count * batch));
}

}  // namespace

extern "C" size_t vsrk_ssim_workspace_size(int32_t batch, int32_t channels, int32_t h, int32_t w) {
  const int tx = ceil_div(std::max(w - SW + 1, 1), TX), ty = ceil_div(std::max(h - SW + 1, 1), TY);
  return (size_t)batch * channels * tx * ty * sizeof(double);
}

extern "C" int vsrk_ssim(const float* out, const float* target, int32_t batch, int32_t channels, int32_t h, int32_t w,
                         int32_t denormalize, float mean, float std, float value_range, float* ssim_per_sample,
                         float* ssim_mean, void* workspace, size_t workspace_bytes, void* stream) {
  VSRK_CHECK(out && target && ssim_per_sample && ssim_mean, "ssim: null argument");
  VSRK_CHECK(batch > 0 && channels > 0, "ssim: empty batch");
  VSRK_CHECK(h >= SW && w >= SW, "ssim: images must be at least %dx%d (valid 11x11 window), got %dx%d", SW, SW, h, w);
  const size_t need = vsrk_ssim_workspace_size(batch, channels, h, w);
  VSRK_CHECK(workspace && workspace_bytes >= need, "ssim: workspace %zu < %zu bytes", workspace_bytes, need);
  SsimArgs a;
  a.out = out;
  a.tgt = target;
  a.h = h;
  a.w = w;
  a.ho = h - SW + 1;
  a.wo = w - SW + 1;
  a.channels = channels;
  a.denorm = denormalize;
  a.mean = mean;
  a.std = std;
  a.c1 = (0.01f * value_range) * (0.01f * value_range);  // metrics.py:57-58
  a.c2 = (0.03f * value_range) * (0.03f * value_range);
  // 1-D factor of the reference window (fp32, as torch builds it), normalised
  float g[SW], sum = 0.f;
  for (int i = 0; i < SW; ++i) {
    const float z = ((float)i - (float)(SW / 2)) / (2.f * 1.5f);
    g[i] = 1.f / (1.5f * sqrtf(2.f * 3.14159265358979f)) * expf(-z * z);
    sum += g[i];
  }
  for (int i = 0; i < SW; ++i) a.g[i] = g[i] / sum;
  a.tiles_x = ceil_div(a.wo, TX);
  a.tiles_y = ceil_div(a.ho, TY);
  hipStream_t s = (hipStream_t)stream;
  dim3 grid(a.tiles_x, a.tiles_y, batch * channels);
  ssim_partial_kernel<<<grid, 256, 0, s>>>(a, (double*)workspace);
  VSRK_LAUNCH_CHECK("ssim_partial");
  ssim_final_kernel<<<1, 64, 0, s>>>((const double*)workspace, batch, channels * a.tiles_x * a.tiles_y,
                                     (double)channels * a.ho * a.wo, ssim_per_sample, ssim_mean);
  VSRK_LAUNCH_CHECK("ssim_final");
  return VSRK_OK;
}
