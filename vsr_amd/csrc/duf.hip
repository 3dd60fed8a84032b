// DUF dynamic upsampling filter, fused (duf_net.py:67-97).
//
// Reference sequence per channel: reshape the filter logits to (N, k*k, r*r,
// ...), softmax over the k*k taps (duf_net.py:69-70), unfold the centre frame
// with an identity k x k conv2d (pad k/2, :79-82), (1 x k*k) @ (k*k x r*r)
// matmul per LR pixel (:84-88), pixel_shuffle(r) (:89), plus the residual
// branch's pixel_shuffle(r) (:95-97).  Here one thread owns one (LR pixel,
// sub-pixel s): it reads the k*k logits of s (contiguous across the 16 threads
// of the pixel: coalesced), the k*k neighbourhood of the centre frame, and
// writes HR pixel (r*h + s/r, r*w + s%r).  Nothing is materialised.
//
// Backward (x is data: no gradient): with P = softmax, o = sum_t P_t x_t,
//   d residual_s = g_s,  d logit_{t,s} = P_t * g_s * (x_t - o).
#include "vsrk_common.h"

namespace {

constexpr int MAXKK = 49;  // k <= 7

// The filter size K is a template parameter so the per-tap arrays below are
// fully unrolled into registers; with a runtime k they were dynamically
// indexed and lived in scratch memory (2.97 ms forward at DUF cfg 2, about
// 0.6 TB/s on the 1.68 GB of fp32 logits).
template <bool BWD, typename GT, int K>
__global__ __launch_bounds__(256) void duf_kernel(const float* __restrict__ x, const float* __restrict__ logits,
                                                  const float* __restrict__ res, float* __restrict__ out,
                                                  const float* __restrict__ gout, GT* __restrict__ dlogits,
                                                  GT* __restrict__ dres, int n, int h, int w, int r) {
  constexpr int k = K, kk = K * K;
  const int rr = r * r;
  const int total = n * h * w * rr;  // < 2^31 (checked on the host): 32-bit decode
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= total) return;
  const int pixi = idx / rr;
  const int s = idx - pixi * rr;
  const int64_t pix = pixi;
  const int t1 = pixi / w;
  const int ww = pixi - t1 * w;
  const int nb = t1 / h;
  const int hh = t1 - nb * h;
  const float* lg = logits + pix * kk * rr + s;
  float l[kk], xv[kk];
  float mx = -INFINITY;
#pragma unroll
  for (int t = 0; t < kk; ++t) {
    l[t] = lg[(int64_t)t * rr];
    mx = fmaxf(mx, l[t]);
    const int dy = t / k - k / 2, dx = t % k - k / 2;
    const int y = hh + dy, xx = ww + dx;
    xv[t] = (y >= 0 && y < h && xx >= 0 && xx < w) ? x[((int64_t)nb * h + y) * w + xx] : 0.f;
  }
  float den = 0.f;
#pragma unroll
  for (int t = 0; t < kk; ++t) {
    l[t] = __expf(l[t] - mx);
    den += l[t];
  }
  const float inv = 1.f / den;
  float o = 0.f;
#pragma unroll
  for (int t = 0; t < kk; ++t) o = fmaf(l[t] * inv, xv[t], o);
  const int64_t hr = ((int64_t)nb * h * r + (hh * r + s / r)) * (w * r) + (ww * r + s % r);
  if (!BWD) {
    out[hr] = o + res[pix * rr + s];
  } else {
    const float g = gout[hr];
    dres[pix * rr + s] = from_f32<GT>(g);
    GT* dl = dlogits + pix * kk * rr + s;
#pragma unroll
    for (int t = 0; t < kk; ++t) dl[(int64_t)t * rr] = from_f32<GT>(l[t] * inv * g * (xv[t] - o));
  }
}

template <bool BWD, typename GT>
void launch_duf(int k, int64_t total, hipStream_t s, const float* x, const float* logits, const float* res,
                float* out, const float* gout, GT* dl, GT* dr, int n, int h, int w, int r) {
  const int grid = (int)ceil_div64(total, 256);
#define VSRK_DUF_K(KV) \
  case KV: duf_kernel<BWD, GT, KV><<<grid, 256, 0, s>>>(x, logits, res, out, gout, dl, dr, n, h, w, r); break
  switch (k) {
    VSRK_DUF_K(1); VSRK_DUF_K(2); VSRK_DUF_K(3); VSRK_DUF_K(4); VSRK_DUF_K(5); VSRK_DUF_K(6); VSRK_DUF_K(7);
    default: break;
  }
#undef VSRK_DUF_K
}

}  // namespace

extern "C" int vsrk_duf_dynfilter_fwd(const float* x, const float* logits, const float* residual, int32_t n,
                                      int32_t h, int32_t w, int32_t size_filter, int32_t upscale, float* out,
                                      void* stream) {
  VSRK_CHECK(x && logits && residual && out, "duf_dynfilter_fwd: null argument");
  VSRK_CHECK(size_filter >= 1 && size_filter * size_filter <= MAXKK && upscale >= 1, "duf_dynfilter_fwd: k/r");
  const int64_t total = (int64_t)n * h * w * upscale * upscale;
  VSRK_CHECK(total < (1ll << 31), "duf_dynfilter: too many output pixels");
  launch_duf<false, float>(size_filter, total, (hipStream_t)stream, x, logits, residual, out, nullptr, nullptr,
                           nullptr, n, h, w, upscale);
  VSRK_LAUNCH_CHECK("duf_dynfilter_fwd");
  return VSRK_OK;
}

extern "C" int vsrk_duf_dynfilter_bwd(const float* x, const float* logits, const float* grad_out, int32_t n,
                                      int32_t h, int32_t w, int32_t size_filter, int32_t upscale,
                                      void* grad_logits, void* grad_residual, int32_t grad_dtype, void* stream) {
  VSRK_CHECK(x && logits && grad_out && grad_logits && grad_residual, "duf_dynfilter_bwd: null argument");
  VSRK_CHECK(size_filter >= 1 && size_filter * size_filter <= MAXKK && upscale >= 1, "duf_dynfilter_bwd: k/r");
  const int64_t total = (int64_t)n * h * w * upscale * upscale;
  VSRK_CHECK(total < (1ll << 31), "duf_dynfilter: too many output pixels");
  hipStream_t s = (hipStream_t)stream;
  if (grad_dtype == VSRK_BF16)
    launch_duf<true, bf16>(size_filter, total, s, x, logits, nullptr, nullptr, grad_out, (bf16*)grad_logits,
                           (bf16*)grad_residual, n, h, w, upscale);
  else if (grad_dtype == VSRK_F16)
    launch_duf<true, f16>(size_filter, total, s, x, logits, nullptr, nullptr, grad_out, (f16*)grad_logits,
                           (f16*)grad_residual, n, h, w, upscale);
  else
    launch_duf<true, float>(size_filter, total, s, x, logits, nullptr, nullptr, grad_out, (float*)grad_logits,
                            (float*)grad_residual, n, h, w, upscale);
  VSRK_LAUNCH_CHECK("duf_dynfilter_bwd");
  return VSRK_OK;
}
