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
  const float* mom;  // 3-D: depth-filtered moments [plane][5][h][w] (ssim3d_depth_kernel)
  int h, w, ho, wo, channels;
  int denorm;
  float mean, std, c1, c2;
  float g[SW];
  int tiles_x, tiles_y;
};

__device__ __forceinline__ float denorm_px(float u, const SsimArgs& a) {
  return a.denorm ? fminf(fmaxf(rintf(u * a.std + a.mean), 0.f), 255.f) : u;
}

// SSIM(dim=3): the window is the outer product of three normalised 1-D
// windows, so the depth axis is filtered first -- one thread per (volume,
// output depth, y, x) sums the 11 depth taps of the five moments (u, v, u^2,
// v^2, uv) into mom[(vol * dout + dz)][m][y][x] -- and each output depth's 5
// moment planes then go through the 2-D kernel's separable (x, y) filter.
__global__ __launch_bounds__(256) void ssim3d_depth_kernel(SsimArgs a, int d, int dout, int64_t total,
                                                          float* __restrict__ mom) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int64_t hw = (int64_t)a.h * a.w;
  const int64_t p = i % hw;
  const int64_t t = i / hw;  // vol * dout + dz
  const int dz = (int)(t % dout);
  const int64_t vol = t / dout;
  const float* po = a.out + (vol * d + dz) * hw + p;
  const float* pt = a.tgt + (vol * d + dz) * hw + p;
  float m[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int k = 0; k < SW; ++k) {
    const float u = denorm_px(po[k * hw], a), v = denorm_px(pt[k * hw], a), gk = a.g[k];
    m[0] = fmaf(gk, u, m[0]);
    m[1] = fmaf(gk, v, m[1]);
    m[2] = fmaf(gk, u * u, m[2]);
    m[3] = fmaf(gk, v * v, m[3]);
    m[4] = fmaf(gk, u * v, m[4]);
  }
  float* o = mom + t * 5 * hw + p;
#pragma unroll
  for (int c = 0; c < 5; ++c) o[c * hw] = m[c];
}

// MOM = false: 2-D images, moments from the (denormalized) pixels.  MOM =
// true: plane img of the 3-D path, the five depth-filtered moment planes.
template <bool MOM>
__global__ __launch_bounds__(256) void ssim_partial_kernel(SsimArgs a, double* __restrict__ part) {
  __shared__ float sx[MOM ? 5 : 2][IY][IX];
  __shared__ float hm[5][IY][TX];
  const int img = blockIdx.z;  // n * channels + c (2-D); (n * channels + c) * dout + dz (3-D)
  const int x0 = blockIdx.x * TX, y0 = blockIdx.y * TY;
  const int64_t hw = (int64_t)a.h * a.w;
  const float* po = MOM ? a.mom + (int64_t)img * 5 * hw : a.out + (int64_t)img * hw;
  const float* pt = a.tgt + (int64_t)img * hw;
  for (int i = threadIdx.x; i < IY * IX; i += blockDim.x) {
    const int yy = i / IX, xx = i - yy * IX;
    const int gy = y0 + yy, gx = x0 + xx;
    const bool in = gy < a.h && gx < a.w;
    if constexpr (MOM) {
#pragma unroll
      for (int c = 0; c < 5; ++c) sx[c][yy][xx] = in ? po[c * hw + (int64_t)gy * a.w + gx] : 0.f;
    } else {
      float u = 0.f, v = 0.f;
      if (in) {
        u = denorm_px(po[(int64_t)gy * a.w + gx], a);
        v = denorm_px(pt[(int64_t)gy * a.w + gx], a);
      }
      sx[0][yy][xx] = u;
      sx[1][yy][xx] = v;
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < IY * TX; i += blockDim.x) {
    const int yy = i / TX, xx = i - yy * TX;
    float m[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < SW; ++k) {
      const float gk = a.g[k];
      if constexpr (MOM) {
#pragma unroll
        for (int c = 0; c < 5; ++c) m[c] = fmaf(gk, sx[c][yy][xx + k], m[c]);
      } else {
        const float u = sx[0][yy][xx + k], v = sx[1][yy][xx + k];
        m[0] = fmaf(gk, u, m[0]);
        m[1] = fmaf(gk, v, m[1]);
        m[2] = fmaf(gk, u * u, m[2]);
        m[3] = fmaf(gk, v * v, m[3]);
        m[4] = fmaf(gk, u * v, m[4]);
      }
    }
#pragma unroll
    for (int c = 0; c < 5; ++c) hm[c][yy][xx] = m[c];
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

// per sample n: sum over its channels' tiles (fixed order: lane-strided
// partials, then a fixed LDS tree) / (C * ho * wo).  One workgroup of 1024
// lanes walks the samples; a single lane summing every tile serially took
// 1.7 ms at cfg 2 (64 samples x ~1 K tiles), 18x the partial kernel.
__global__ __launch_bounds__(1024) void ssim_final_kernel(const double* __restrict__ part, int batch,
                                                          int per_sample_tiles, double count,
                                                          float* __restrict__ per, float* __restrict__ mean_out) {
  __shared__ double red[1024];
  double all = 0.0;
  for (int b = 0; b < batch; ++b) {
    const double* p = part + (int64_t)b * per_sample_tiles;
    double s = 0.0;
    for (int k = threadIdx.x; k < per_sample_tiles; k += 1024) s += p[k];
    red[threadIdx.x] = s;
    __syncthreads();
    for (int k = 512; k > 0; k >>= 1) {
      if (threadIdx.x < k) red[threadIdx.x] += red[threadIdx.x + k];
      __syncthreads();
    }
    if (threadIdx.x == 0) {
      per[b] = (float)(red[0] / count);
      all += red[0];
    }
    __syncthreads();  // red is rewritten by the next sample
  }
  if (threadIdx.x == 0) *mean_out = (float)(all / (count * batch));
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
  ssim_partial_kernel<false><<<grid, 256, 0, s>>>(a, (double*)workspace);
  VSRK_LAUNCH_CHECK("ssim_partial");
  ssim_final_kernel<<<1, 1024, 0, s>>>((const double*)workspace, batch, channels * a.tiles_x * a.tiles_y,
                                     (double)channels * a.ho * a.wo, ssim_per_sample, ssim_mean);
  VSRK_LAUNCH_CHECK("ssim_final");
  return VSRK_OK;
}

// SSIM(dim=3) of (N, C, D, H, W) volumes (metrics.py:39-113 with dim=3): a
// valid 11x11x11 window.  Workspace: the depth-filtered moments plus the
// per-tile partials.
extern "C" size_t vsrk_ssim3d_workspace_size(int32_t batch, int32_t channels, int32_t d, int32_t h, int32_t w) {
  const int dout = std::max(d - SW + 1, 1);
  const int tx = ceil_div(std::max(w - SW + 1, 1), TX), ty = ceil_div(std::max(h - SW + 1, 1), TY);
  const size_t mom = ((size_t)batch * channels * dout * 5 * h * w * sizeof(float) + 255) / 256 * 256;
  return mom + (size_t)batch * channels * dout * tx * ty * sizeof(double);
}

extern "C" int vsrk_ssim3d(const float* out, const float* target, int32_t batch, int32_t channels, int32_t d,
                           int32_t h, int32_t w, int32_t denormalize, float mean, float std, float value_range,
                           float* ssim_per_sample, float* ssim_mean, void* workspace, size_t workspace_bytes,
                           void* stream) {
  VSRK_CHECK(out && target && ssim_per_sample && ssim_mean, "ssim3d: null argument");
  VSRK_CHECK(batch > 0 && channels > 0, "ssim3d: empty batch");
  VSRK_CHECK(d >= SW && h >= SW && w >= SW, "ssim3d: volumes must be at least %d^3 (valid window), got %dx%dx%d", SW,
             d, h, w);
  const size_t need = vsrk_ssim3d_workspace_size(batch, channels, d, h, w);
  VSRK_CHECK(workspace && workspace_bytes >= need, "ssim3d: workspace %zu < %zu bytes", workspace_bytes, need);
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
  a.c1 = (0.01f * value_range) * (0.01f * value_range);
  a.c2 = (0.03f * value_range) * (0.03f * value_range);
  float g[SW], sum = 0.f;
  for (int i = 0; i < SW; ++i) {
    const float z = ((float)i - (float)(SW / 2)) / (2.f * 1.5f);
    g[i] = 1.f / (1.5f * sqrtf(2.f * 3.14159265358979f)) * expf(-z * z);
    sum += g[i];
  }
  for (int i = 0; i < SW; ++i) a.g[i] = g[i] / sum;
  a.tiles_x = ceil_div(a.wo, TX);
  a.tiles_y = ceil_div(a.ho, TY);
  const int dout = d - SW + 1;
  const size_t mom_bytes = ((size_t)batch * channels * dout * 5 * h * w * sizeof(float) + 255) / 256 * 256;
  float* mom = (float*)workspace;
  double* part = (double*)((char*)workspace + mom_bytes);
  a.mom = mom;
  hipStream_t s = (hipStream_t)stream;
  const int64_t total = (int64_t)batch * channels * dout * h * w;
  ssim3d_depth_kernel<<<(int)ceil_div64(total, 256), 256, 0, s>>>(a, d, dout, total, mom);
  VSRK_LAUNCH_CHECK("ssim3d_depth");
  dim3 grid(a.tiles_x, a.tiles_y, batch * channels * dout);
  ssim_partial_kernel<true><<<grid, 256, 0, s>>>(a, part);
  VSRK_LAUNCH_CHECK("ssim3d_partial");
  ssim_final_kernel<<<1, 1024, 0, s>>>(part, batch, channels * dout * a.tiles_x * a.tiles_y,
                                     (double)channels * dout * a.ho * a.wo, ssim_per_sample, ssim_mean);
  VSRK_LAUNCH_CHECK("ssim3d_final");
  return VSRK_OK;
}
