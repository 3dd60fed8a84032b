// Memory-bound kernels around the convs: layout moves, per-channel reductions,
// ReLU backward, skip-connection adds, losses and the denormalize+PSNR metric.
// All reductions are two-pass (per-block partials, then a fixed-order final
// sum) so results are bitwise reproducible run to run.
#include <stdarg.h>
#include <stdio.h>
#include "vsrk_common.h"
#include "vsrk_internal.h"

static thread_local char g_err[512];

void vsrk_set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

extern "C" const char* vsrk_last_error(void) { return g_err; }
extern "C" const char* vsrk_version(void) { return "vsrk 0.1 gfx950"; }

namespace {

constexpr int RED_BLOCKS = 1024;

__device__ __forceinline__ void decode_voxel(int64_t v, const View& t, int& n, int& d, int& h, int& w) {
  w = v % t.w;
  v /= t.w;
  h = v % t.h;
  v /= t.h;
  d = v % t.d;
  n = v / t.d;
}

template <typename T>
__global__ void ncdhw_to_view_kernel(const float* __restrict__ src, int n, int c, int d, int h, int w, View dst,
                                     int64_t total) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= total) return;  // total = voxels * dst.c
  const int ch = idx % dst.c;
  const int64_t vox = idx / dst.c;
  int nn, dd, hh, ww;
  decode_voxel(vox, dst, nn, dd, hh, ww);
  float v = 0.f;
  if (ch < c) v = src[((((int64_t)nn * c + ch) * d + dd) * h + hh) * w + ww];
  reinterpret_cast<T*>(dst.ptr)[view_off(dst, nn, dd, hh, ww, ch)] = from_f32<T>(v);
}

// Dense channels-last destination (the network edges: the LR input and the HR
// output gradient in their zero-padded 8-channel storage).  One thread per
// voxel writes whole 16-byte chunks (padding channels as zeros); the only
// division is voxel -> (sample, spatial offset).  The generic kernel above
// spends its time in the 64-bit div/mod chain of decode_voxel per element.
template <typename T>
__global__ void ncdhw_to_dense_kernel(const float* __restrict__ src, int c, int dhw, int cp, int nvox,
                                      T* __restrict__ dst) {
  constexpr int E = Chunk<T>::E;
  const int v = blockIdx.x * blockDim.x + threadIdx.x;
  if (v >= nvox) return;
  const int nn = v / dhw, rem = v - nn * dhw;
  const float* s = src + (int64_t)nn * c * dhw + rem;
  uint4* o = reinterpret_cast<uint4*>(dst + (int64_t)v * cp);
  for (int c0 = 0; c0 < cp; c0 += E) {
    float f[E];
#pragma unroll
    for (int e = 0; e < E; ++e) f[e] = (c0 + e < c) ? __builtin_nontemporal_load(s + (int64_t)(c0 + e) * dhw) : 0.f;
    o[c0 / E] = Chunk<T>::pack(f);
  }
}

template <typename T>
__global__ void view_to_ncdhw_kernel(View src, float* __restrict__ dst, int c, int64_t total) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= total) return;  // total = n*c*d*h*w, NCDHW order
  int64_t v = idx;
  const int ww = v % src.w; v /= src.w;
  const int hh = v % src.h; v /= src.h;
  const int dd = v % src.d; v /= src.d;
  const int ch = v % c;
  const int nn = v / c;
  dst[idx] = to_f32<T>(reinterpret_cast<const T*>(src.ptr)[view_off(src, nn, dd, hh, ww, ch)]);
}

// per-channel sum (mode 0) or sum + sum of squares (mode 1) over every voxel
template <typename T>
__global__ void channel_partial_kernel(View x, int64_t nvox, int mode, float* __restrict__ part) {
  // part layout: [blocks][2][C]
  const int C = x.c;
  const int64_t per = (nvox + gridDim.x - 1) / gridDim.x;
  const int64_t v0 = blockIdx.x * per, v1 = min(nvox, v0 + per);
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    double s = 0.0, q = 0.0;
    for (int64_t v = v0; v < v1; ++v) {
      int n, d, h, w;
      decode_voxel(v, x, n, d, h, w);
      const float f = to_f32<T>(reinterpret_cast<const T*>(x.ptr)[view_off(x, n, d, h, w, c)]);
      s += f;
      if (mode) q += (double)f * f;
    }
    part[((int64_t)blockIdx.x * 2) * C + c] = (float)s;
    if (mode) part[((int64_t)blockIdx.x * 2 + 1) * C + c] = (float)q;
  }
}

__global__ void channel_final_kernel(const float* __restrict__ part, int nblk, int C, int mode, int perm_r,
                                     float scale, float* __restrict__ sum, float* __restrict__ sumsq,
                                     int accumulate) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  double s = 0.0, q = 0.0;
  for (int b = 0; b < nblk; ++b) {
    s += part[((int64_t)b * 2) * C + c];
    if (mode) q += part[((int64_t)b * 2 + 1) * C + c];
  }
  int ct = c;
  if (perm_r > 1) {
    const int rr = perm_r * perm_r, cp = C / rr;
    const int sub = c / cp, cc = c - sub * cp;
    ct = cc * rr + sub;
  }
  const float fs = (float)(s * scale);
  sum[ct] = accumulate ? sum[ct] + fs : fs;
  if (mode) sumsq[ct] = (float)(q * scale);
}

template <typename T>
__global__ void relu_bwd_kernel(View y, View dy, View dx, int64_t total) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= total) return;
  const int c = idx % y.c;
  int n, d, h, w;
  decode_voxel(idx / y.c, y, n, d, h, w);
  const float yv = to_f32<T>(reinterpret_cast<const T*>(y.ptr)[view_off(y, n, d, h, w, c)]);
  const float g = to_f32<T>(reinterpret_cast<const T*>(dy.ptr)[view_off(dy, n, d, h, w, c)]);
  reinterpret_cast<T*>(dx.ptr)[view_off(dx, n, d, h, w, c)] = from_f32<T>(yv > 0.f ? g : 0.f);
}

template <typename T>
__global__ void add_kernel(View a, View b, View o, int64_t total) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= total) return;
  const int c = idx % a.c;
  int n, d, h, w;
  decode_voxel(idx / a.c, a, n, d, h, w);
  const float av = to_f32<T>(reinterpret_cast<const T*>(a.ptr)[view_off(a, n, d, h, w, c)]);
  const float bv = to_f32<T>(reinterpret_cast<const T*>(b.ptr)[view_off(b, n, d, h, w, c)]);
  reinterpret_cast<T*>(o.ptr)[view_off(o, n, d, h, w, c)] = from_f32<T>(av + bv);
}

// ---- losses ----
__device__ __forceinline__ float loss_val(int kind, float p, float d) {
  const float a = fabsf(d);
  switch (kind) {
    case 0: return a;
    case 1: return d * d;
    case 2: {
      const float q = fminf(a, p);
      return 0.5f * q * q + p * (a - q);
    }
    default: return sqrtf(d * d + p);
  }
}
__device__ __forceinline__ float loss_grad(int kind, float p, float d) {
  switch (kind) {
    case 0: return d > 0.f ? 1.f : (d < 0.f ? -1.f : 0.f);
    case 1: return 2.f * d;
    case 2: return fabsf(d) < p ? d : (d > 0.f ? p : (d < 0.f ? -p : 0.f));
    default: return d / sqrtf(d * d + p);
  }
}

__global__ void loss_partial_kernel(int kind, float p, const float* __restrict__ o, const float* __restrict__ t,
                                    int64_t count, double* __restrict__ part) {
  __shared__ double sh[256];
  double s = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < count; i += (int64_t)gridDim.x * blockDim.x)
    s += loss_val(kind, p, o[i] - t[i]);
  sh[threadIdx.x] = s;
  __syncthreads();
  for (int k = 128; k > 0; k >>= 1) {
    if (threadIdx.x < k) sh[threadIdx.x] += sh[threadIdx.x + k];
    __syncthreads();
  }
  if (threadIdx.x == 0) part[blockIdx.x] = sh[0];
}

__global__ void loss_final_kernel(const double* __restrict__ part, int nblk, int64_t count, float* __restrict__ loss) {
  __shared__ double sh[256];
  double s = 0.0;
  for (int b = threadIdx.x; b < nblk; b += blockDim.x) s += part[b];
  sh[threadIdx.x] = s;
  __syncthreads();
  for (int k = 128; k > 0; k >>= 1) {
    if (threadIdx.x < k) sh[threadIdx.x] += sh[threadIdx.x + k];
    __syncthreads();
  }
  if (threadIdx.x == 0) *loss = (float)(sh[0] / (double)count);
}

template <typename T>
__global__ void loss_bwd_kernel(int kind, float p, const float* __restrict__ o, const float* __restrict__ t,
                                int64_t count, const float* __restrict__ gscale, T* __restrict__ g) {
  const float sc = (gscale ? *gscale : 1.f) / (float)count;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < count; i += (int64_t)gridDim.x * blockDim.x)
    g[i] = from_f32<T>(loss_grad(kind, p, o[i] - t[i]) * sc);
}

// ---- denormalize + PSNR ----
__global__ void psnr_partial_kernel(const float* __restrict__ o, const float* __restrict__ t, int64_t per,
                                    int denorm, float mean, float std, int chunks, double* __restrict__ part) {
  // grid: (chunks, batch)
  __shared__ double sh[256];
  const int b = blockIdx.y;
  const int64_t per_chunk = (per + chunks - 1) / chunks;
  const int64_t i0 = blockIdx.x * per_chunk, i1 = min(per, i0 + per_chunk);
  const float* ob = o + (int64_t)b * per;
  const float* tb = t + (int64_t)b * per;
  double s = 0.0;
  for (int64_t i = i0 + threadIdx.x; i < i1; i += blockDim.x) {
    float a = ob[i], c = tb[i];
    if (denorm) {
      a = fminf(fmaxf(rintf(a * std + mean), 0.f), 255.f);
      c = fminf(fmaxf(rintf(c * std + mean), 0.f), 255.f);
    }
    const float d = a - c;
    s += (double)(d * d);
  }
  sh[threadIdx.x] = s;
  __syncthreads();
  for (int k = 128; k > 0; k >>= 1) {
    if (threadIdx.x < k) sh[threadIdx.x] += sh[threadIdx.x + k];
    __syncthreads();
  }
  if (threadIdx.x == 0) part[(int64_t)b * chunks + blockIdx.x] = sh[0];
}

// per sample: the chunk partials in a fixed order (lane-strided, then a
// fixed LDS tree); one lane walking every chunk took ~220 us at cfg 2
__global__ __launch_bounds__(1024) void psnr_final_kernel(const double* __restrict__ part, int batch, int chunks,
                                                          int64_t per, float maxv, float* __restrict__ psnr,
                                                          float* __restrict__ mean_out) {
  __shared__ double red[1024];
  float acc = 0.f;
  for (int b = 0; b < batch; ++b) {
    double s = 0.0;
    for (int k = threadIdx.x; k < chunks; k += 1024) s += part[(int64_t)b * chunks + k];
    red[threadIdx.x] = s;
    __syncthreads();
    for (int k = 512; k > 0; k >>= 1) {
      if (threadIdx.x < k) red[threadIdx.x] += red[threadIdx.x + k];
      __syncthreads();
    }
    if (threadIdx.x == 0) {
      const float mse = (float)(red[0] / (double)per);
      const float p = 10.f * log10f(maxv * maxv / (mse + 1e-10f));
      psnr[b] = p;
      acc += p;
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) *mean_out = acc / (float)batch;
}

}  // namespace

// ---------------------------------------------------------------------------
static inline int esize(int dt) { return vsrk_esize(dt); }
static inline int64_t nvox(const vsrk_tensor5* t) { return (int64_t)t->n * t->d * t->h * t->w; }

size_t vsrk_channel_reduce_ws_bytes(int c) { return (size_t)RED_BLOCKS * 2 * c * sizeof(float); }

int vsrk_channel_reduce_internal(const vsrk_tensor5* x, int mode, int perm_r, float scale, float* sum,
                                 float* sumsq, int accumulate, void* ws, size_t ws_bytes, hipStream_t s) {
  View v = make_view(x);
  const int64_t nv = nvox(x);
  const int nblk = (int)std::min<int64_t>(RED_BLOCKS, std::max<int64_t>(1, nv / 64));
  const size_t need = (size_t)nblk * 2 * x->c * sizeof(float);
  VSRK_CHECK(ws && ws_bytes >= need, "channel_reduce: workspace %zu < %zu bytes", ws_bytes, need);
  float* part = (float*)ws;
  if (x->dtype == VSRK_BF16)
    channel_partial_kernel<bf16><<<nblk, 256, 0, s>>>(v, nv, mode, part);
  else if (x->dtype == VSRK_F16)
    channel_partial_kernel<f16><<<nblk, 256, 0, s>>>(v, nv, mode, part);
  else
    channel_partial_kernel<float><<<nblk, 256, 0, s>>>(v, nv, mode, part);
  VSRK_LAUNCH_CHECK("channel_partial");
  channel_final_kernel<<<ceil_div(x->c, 256), 256, 0, s>>>(part, nblk, x->c, mode, perm_r, scale, sum, sumsq,
                                                           accumulate);
  VSRK_LAUNCH_CHECK("channel_final");
  return VSRK_OK;
}

extern "C" int vsrk_ncdhw_to_view(const float* src, int32_t n, int32_t c, int32_t d, int32_t h, int32_t w,
                                  const vsrk_tensor5* dst, void* stream) {
  VSRK_CHECK(src && dst && dst->ptr, "ncdhw_to_view: null argument");
  VSRK_CHECK(dst->n == n && dst->d == d && dst->h == h && dst->w == w && dst->c >= c,
             "ncdhw_to_view: shape mismatch");
  View v = make_view(dst);
  const int64_t total = nvox(dst) * dst->c;
  hipStream_t s = (hipStream_t)stream;
  const int64_t cp = dst->c, dhw = (int64_t)d * h * w;
  const int esz = vsrk_esize(dst->dtype);
  const bool dense = dst->shuffle <= 1 && dst->sw == cp && dst->sh == w * cp && dst->sd == h * dst->sh &&
                     dst->sn == d * dst->sd && (cp * esz) % 16 == 0 && ((uintptr_t)dst->ptr) % 16 == 0 &&
                     nvox(dst) < (1ll << 31) && dhw * c < (1ll << 31);
  if (dense) {
    const int nv = (int)nvox(dst);
    if (dst->dtype == VSRK_BF16)
      ncdhw_to_dense_kernel<bf16><<<ceil_div(nv, 256), 256, 0, s>>>(src, c, (int)dhw, (int)cp, nv, (bf16*)dst->ptr);
    else if (dst->dtype == VSRK_F16)
      ncdhw_to_dense_kernel<f16><<<ceil_div(nv, 256), 256, 0, s>>>(src, c, (int)dhw, (int)cp, nv, (f16*)dst->ptr);
    else
      ncdhw_to_dense_kernel<float><<<ceil_div(nv, 256), 256, 0, s>>>(src, c, (int)dhw, (int)cp, nv, (float*)dst->ptr);
    VSRK_LAUNCH_CHECK("ncdhw_to_view(dense)");
    return VSRK_OK;
  }
  if (dst->dtype == VSRK_BF16)
    ncdhw_to_view_kernel<bf16><<<(int)ceil_div64(total, 256), 256, 0, s>>>(src, n, c, d, h, w, v, total);
  else if (dst->dtype == VSRK_F16)
    ncdhw_to_view_kernel<f16><<<(int)ceil_div64(total, 256), 256, 0, s>>>(src, n, c, d, h, w, v, total);
  else
    ncdhw_to_view_kernel<float><<<(int)ceil_div64(total, 256), 256, 0, s>>>(src, n, c, d, h, w, v, total);
  VSRK_LAUNCH_CHECK("ncdhw_to_view");
  return VSRK_OK;
}

extern "C" int vsrk_view_to_ncdhw(const vsrk_tensor5* src, float* dst, int32_t c, void* stream) {
  VSRK_CHECK(src && dst && src->ptr, "view_to_ncdhw: null argument");
  VSRK_CHECK(c <= src->c, "view_to_ncdhw: c > view channels");
  View v = make_view(src);
  const int64_t total = nvox(src) * c;
  hipStream_t s = (hipStream_t)stream;
  if (src->dtype == VSRK_BF16)
    view_to_ncdhw_kernel<bf16><<<(int)ceil_div64(total, 256), 256, 0, s>>>(v, dst, c, total);
  else if (src->dtype == VSRK_F16)
    view_to_ncdhw_kernel<f16><<<(int)ceil_div64(total, 256), 256, 0, s>>>(v, dst, c, total);
  else
    view_to_ncdhw_kernel<float><<<(int)ceil_div64(total, 256), 256, 0, s>>>(v, dst, c, total);
  VSRK_LAUNCH_CHECK("view_to_ncdhw");
  return VSRK_OK;
}

extern "C" int vsrk_relu_bwd(const vsrk_tensor5* y, const vsrk_tensor5* dy, const vsrk_tensor5* dx, void* stream) {
  VSRK_CHECK(y && dy && dx, "relu_bwd: null argument");
  VSRK_CHECK(y->dtype == dy->dtype && y->dtype == dx->dtype, "relu_bwd: dtype mismatch");
  const int64_t total = nvox(y) * y->c;
  hipStream_t s = (hipStream_t)stream;
  if (y->dtype == VSRK_BF16)
    relu_bwd_kernel<bf16><<<(int)ceil_div64(total, 256), 256, 0, s>>>(make_view(y), make_view(dy), make_view(dx), total);
  else if (y->dtype == VSRK_F16)
    relu_bwd_kernel<f16><<<(int)ceil_div64(total, 256), 256, 0, s>>>(make_view(y), make_view(dy), make_view(dx), total);
  else
    relu_bwd_kernel<float><<<(int)ceil_div64(total, 256), 256, 0, s>>>(make_view(y), make_view(dy), make_view(dx), total);
  VSRK_LAUNCH_CHECK("relu_bwd");
  return VSRK_OK;
}

extern "C" int vsrk_add(const vsrk_tensor5* a, const vsrk_tensor5* b, const vsrk_tensor5* out, void* stream) {
  VSRK_CHECK(a && b && out, "add: null argument");
  VSRK_CHECK(a->dtype == b->dtype && a->dtype == out->dtype, "add: dtype mismatch");
  const int64_t total = nvox(a) * a->c;
  hipStream_t s = (hipStream_t)stream;
  if (a->dtype == VSRK_BF16)
    add_kernel<bf16><<<(int)ceil_div64(total, 256), 256, 0, s>>>(make_view(a), make_view(b), make_view(out), total);
  else if (a->dtype == VSRK_F16)
    add_kernel<f16><<<(int)ceil_div64(total, 256), 256, 0, s>>>(make_view(a), make_view(b), make_view(out), total);
  else
    add_kernel<float><<<(int)ceil_div64(total, 256), 256, 0, s>>>(make_view(a), make_view(b), make_view(out), total);
  VSRK_LAUNCH_CHECK("add");
  return VSRK_OK;
}

extern "C" size_t vsrk_loss_workspace_size(int64_t count) { return 1024 * sizeof(double); }

extern "C" int vsrk_loss_fwd(int32_t kind, float param, const float* out, const float* target, int64_t count,
                             float* loss, void* workspace, size_t workspace_bytes, void* stream) {
  VSRK_CHECK(out && target && loss && workspace, "loss_fwd: null argument");
  VSRK_CHECK(kind >= 0 && kind <= 3, "loss_fwd: unknown kind %d", kind);
  VSRK_CHECK(workspace_bytes >= 1024 * sizeof(double), "loss_fwd: workspace too small");
  const int nblk = (int)std::min<int64_t>(1024, std::max<int64_t>(1, ceil_div64(count, 256 * 8)));
  hipStream_t s = (hipStream_t)stream;
  loss_partial_kernel<<<nblk, 256, 0, s>>>(kind, param, out, target, count, (double*)workspace);
  VSRK_LAUNCH_CHECK("loss_partial");
  loss_final_kernel<<<1, 256, 0, s>>>((const double*)workspace, nblk, count, loss);
  VSRK_LAUNCH_CHECK("loss_final");
  return VSRK_OK;
}

extern "C" int vsrk_loss_bwd(int32_t kind, float param, const float* out, const float* target, int64_t count,
                             const float* gscale, void* grad, int32_t grad_dtype, void* stream) {
  VSRK_CHECK(out && target && grad, "loss_bwd: null argument");
  const int nblk = (int)std::min<int64_t>(4096, std::max<int64_t>(1, ceil_div64(count, 256)));
  hipStream_t s = (hipStream_t)stream;
  if (grad_dtype == VSRK_BF16)
    loss_bwd_kernel<bf16><<<nblk, 256, 0, s>>>(kind, param, out, target, count, gscale, (bf16*)grad);
  else if (grad_dtype == VSRK_F16)
    loss_bwd_kernel<f16><<<nblk, 256, 0, s>>>(kind, param, out, target, count, gscale, (f16*)grad);
  else
    loss_bwd_kernel<float><<<nblk, 256, 0, s>>>(kind, param, out, target, count, gscale, (float*)grad);
  VSRK_LAUNCH_CHECK("loss_bwd");
  return VSRK_OK;
}

extern "C" size_t vsrk_psnr_workspace_size(int32_t batch, int64_t per_sample) {
  return (size_t)batch * 64 * sizeof(double);
}

extern "C" int vsrk_psnr(const float* out, const float* target, int32_t batch, int64_t per_sample,
                         int32_t denormalize, float mean, float std, float max_value, float* psnr_per_sample, float* psnr_mean, void* workspace,
                         size_t workspace_bytes, void* stream) {
  VSRK_CHECK(out && target && psnr_per_sample && psnr_mean && workspace, "psnr: null argument");
  VSRK_CHECK(workspace_bytes >= vsrk_psnr_workspace_size(batch, per_sample), "psnr: workspace too small");
  VSRK_CHECK(batch >= 1 && per_sample >= 1, "psnr: empty input");
  const int chunks = 64;
  hipStream_t s = (hipStream_t)stream;
  psnr_partial_kernel<<<dim3(chunks, batch), 256, 0, s>>>(out, target, per_sample, denormalize, mean, std, chunks,
                                                         (double*)workspace);
  VSRK_LAUNCH_CHECK("psnr_partial");
  psnr_final_kernel<<<1, 1024, 0, s>>>((const double*)workspace, batch, chunks, per_sample, max_value,
                                     psnr_per_sample, psnr_mean);
  VSRK_LAUNCH_CHECK("psnr_final");
  return VSRK_OK;
}

// ---------------------------------------------------------------------------
// LR synthesis (acdc_preprocess.py:102-180, Downscale): the bicubic resize of
// the k-space-truncated image, cv2.resize(INTER_CUBIC) on float64 input as
// OpenCV computes it: the source coordinate fx = float((d + 0.5) * s - 0.5),
// the Keys cubic (A = -0.75) weights of its fraction in float, indices clamped
// at the borders, a horizontal pass per source row then the vertical pass,
// each as a left-to-right sum of double products (no contraction) -- then
// np.clip(img.round(), 0, 255).  One thread per output pixel (offline data
// preparation, tiny next to the step).
namespace {
__device__ __forceinline__ void cubic_w(float x, float* w) {
#pragma clang fp contract(off)
  const float A = -0.75f;
  w[0] = ((A * (x + 1) - 5 * A) * (x + 1) + 8 * A) * (x + 1) - 4 * A;
  w[1] = ((A + 2) * x - (A + 3)) * x * x + 1;
  w[2] = ((A + 2) * (1 - x) - (A + 3)) * (1 - x) * (1 - x) + 1;
  w[3] = 1.f - w[0] - w[1] - w[2];
}
__global__ void resize_bicubic_kernel(const double* __restrict__ src, int n, int ih, int iw, int oh, int ow,
                                      double* __restrict__ dst, int round_clip) {
#pragma clang fp contract(off)
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)n * oh * ow) return;
  const int x = (int)(i % ow);
  const int64_t t = i / ow;
  const int y = (int)(t % oh);
  const int b = (int)(t / oh);
  const double scy = 1.0 / ((double)oh / ih), scx = 1.0 / ((double)ow / iw);
  float fy = (float)((y + 0.5) * scy - 0.5), fx = (float)((x + 0.5) * scx - 0.5);
  const int y0 = (int)floorf(fy), x0 = (int)floorf(fx);
  fy -= y0;
  fx -= x0;
  float wy[4], wx[4];
  cubic_w(fy, wy);
  cubic_w(fx, wx);
  const double* im = src + (int64_t)b * ih * iw;
  double rows[4];
#pragma unroll
  for (int a = 0; a < 4; ++a) {
    const double* r = im + (int64_t)min(max(y0 - 1 + a, 0), ih - 1) * iw;
    const double s0 = r[min(max(x0 - 1, 0), iw - 1)], s1 = r[min(max(x0, 0), iw - 1)];
    const double s2 = r[min(max(x0 + 1, 0), iw - 1)], s3 = r[min(max(x0 + 2, 0), iw - 1)];
    rows[a] = s0 * (double)wx[0] + s1 * (double)wx[1] + s2 * (double)wx[2] + s3 * (double)wx[3];
  }
  double acc = rows[0] * (double)wy[0] + rows[1] * (double)wy[1] + rows[2] * (double)wy[2] + rows[3] * (double)wy[3];
  if (round_clip) acc = fmin(fmax(rint(acc), 0.0), 255.0);
  dst[i] = acc;
}
}  // namespace

extern "C" int vsrk_resize_bicubic(const double* src, int32_t n, int32_t ih, int32_t iw, int32_t oh, int32_t ow,
                                   double* dst, int32_t round_clip, void* stream) {
  VSRK_CHECK(src && dst && n > 0 && ih > 0 && iw > 0 && oh > 0 && ow > 0, "resize_bicubic: bad argument");
  const int64_t total = (int64_t)n * oh * ow;
  resize_bicubic_kernel<<<(int)ceil_div64(total, 256), 256, 0, (hipStream_t)stream>>>(src, n, ih, iw, oh, ow, dst,
                                                                                      round_clip);
  VSRK_LAUNCH_CHECK("resize_bicubic");
  return VSRK_OK;
}
