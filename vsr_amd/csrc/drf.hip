// Kernels specific to the DRF feedback generator (drf_net.py:8-147).
//
//  * Sub-pixel weight transforms: the feedback block's strided projections
//    nn.Conv2d(k, stride s, pad p) / nn.ConvTranspose2d(k, s, p)
//    (drf_net.py:70-102) become 3x3 pad-1 convolutions on the low-res grid
//    (see include/vsrk.h), so they run on the implicit-GEMM MFMA kernels with
//    a shuffle-s input view (strided conv) or output view (transposed conv).
//    For an output sub-pixel offset i in [0, s) and conv tap kh in {0,1,2}
//    (input row offset kh - 1):
//        strided conv:    kernel row s*(kh - 1) + i + p
//        transposed conv: kernel row s*(1 - kh) + i + p
//    (zero when outside [0, k)); every kernel entry has exactly one image.
//  * PReLU slope gradient: da = sum_{y<0} dx * y / a^2 over a channels-last
//    view, two-pass fixed-order reduction (deterministic).
#include <algorithm>
#include "vsrk_common.h"
#include "vsrk_internal.h"

namespace {

__device__ __forceinline__ int sp_row(int transposed, int s, int p, int tap, int sub) {
  return transposed ? s * (1 - tap) + sub + p : s * (tap - 1) + sub + p;
}

// one thread per equivalent-weight element (torch layout (co', ci', 3, 3))
__global__ void subpixel_weight_kernel(const float* __restrict__ w, const float* __restrict__ bias, int cin,
                                       int cout, int k, int s, int p, int transposed, float* __restrict__ weq,
                                       float* __restrict__ beq, int64_t total) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= total) return;
  const int kw = idx % 3, kh = (idx / 3) % 3;
  const int64_t t = idx / 9;
  const int cip = transposed ? cin : s * s * cin;  // equivalent input channels
  const int ci_e = t % cip, co_e = t / cip;
  int co, ci, sub;
  if (transposed) {
    sub = co_e / cout;
    co = co_e - sub * cout;
    ci = ci_e;
  } else {
    sub = ci_e / cin;
    ci = ci_e - sub * cin;
    co = co_e;
  }
  const int si = sub / s, sj = sub - si * s;
  const int ky = sp_row(transposed, s, p, kh, si), kx = sp_row(transposed, s, p, kw, sj);
  float v = 0.f;
  if (ky >= 0 && ky < k && kx >= 0 && kx < k) {
    const int64_t widx = transposed ? (((int64_t)ci * cout + co) * k + ky) * k + kx
                                    : (((int64_t)co * cin + ci) * k + ky) * k + kx;
    v = w[widx];
  }
  weq[idx] = v;
  if (beq && kh == 0 && kw == 0 && ci_e == 0) beq[co_e] = bias ? bias[co] : 0.f;
}

// one thread per k x k weight element: gather its single equivalent entry
__global__ void subpixel_fold_kernel(const float* __restrict__ dweq, const float* __restrict__ dbeq, int cin,
                                     int cout, int k, int s, int p, int transposed, float* __restrict__ dw,
                                     float* __restrict__ db, int accumulate, int64_t total) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx < total) {
    const int kx = idx % k, ky = (idx / k) % k;
    const int64_t t = idx / (k * k);
    // transposed: idx over (cin, cout, k, k); else (cout, cin, k, k)
    const int b = t % (transposed ? cout : cin), a = t / (transposed ? cout : cin);
    const int ci = transposed ? a : b, co = transposed ? b : a;
    // solve ky = s*(+-(kh-1)) + si + p for (kh, si) with kh in {0,1,2}, si in [0, s)
    int kh = -1, si = 0, kw = -1, sj = 0;
    for (int q = 0; q < 3; ++q) {
      const int ry = ky - sp_row(transposed, s, p, q, 0);
      if (ry >= 0 && ry < s) { kh = q; si = ry; }
      const int rx = kx - sp_row(transposed, s, p, q, 0);
      if (rx >= 0 && rx < s) { kw = q; sj = rx; }
    }
    float v = 0.f;
    if (kh >= 0 && kw >= 0) {
      const int sub = si * s + sj;
      const int co_e = transposed ? sub * cout + co : co;
      const int ci_e = transposed ? ci : sub * cin + ci;
      const int cip = transposed ? cin : s * s * cin;
      v = dweq[(((int64_t)co_e * cip + ci_e) * 3 + kh) * 3 + kw];
    }
    dw[idx] = accumulate ? dw[idx] + v : v;
  }
  if (db && idx < cout) {
    float v = 0.f;
    if (transposed) {
      for (int sub = 0; sub < s * s; ++sub) v += dbeq[sub * cout + idx];  // fixed order
    } else {
      v = dbeq[idx];
    }
    db[idx] = accumulate ? db[idx] + v : v;
  }
}

constexpr int PRELU_BLOCKS = 2048;  // 8 per CU: enough loads in flight for the high-res rows

template <typename T>
__global__ __launch_bounds__(256) void prelu_partial_kernel(View y, View dx, int64_t nvox, double* __restrict__ part) {
  // each thread walks 8-channel chunks of voxels: (voxel, chunk) flattened
  constexpr int E = 16 / sizeof(T);
  const int cpv = (y.c + E - 1) / E;
  const int64_t total = nvox * cpv;
  double s = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int ch = (int)(i % cpv) * E;
    int64_t v = i / cpv;
    const int w = v % y.w; v /= y.w;
    const int h = v % y.h; v /= y.h;
    const int d = v % y.d;
    const int n = v / y.d;
    const T* py = reinterpret_cast<const T*>(y.ptr) + view_off(y, n, d, h, w, ch);
    const T* pd = reinterpret_cast<const T*>(dx.ptr) + view_off(dx, n, d, h, w, ch);
    float acc = 0.f;
#pragma unroll
    for (int e = 0; e < E; ++e) {
      if (ch + e < y.c) {
        const float yv = to_f32<T>(py[e]);
        if (yv < 0.f) acc = fmaf(to_f32<T>(pd[e]), yv, acc);
      }
    }
    s += acc;
  }
  __shared__ double sh[256];
  sh[threadIdx.x] = s;
  __syncthreads();
  for (int k = 128; k > 0; k >>= 1) {
    if (threadIdx.x < k) sh[threadIdx.x] += sh[threadIdx.x + k];
    __syncthreads();
  }
  if (threadIdx.x == 0) part[blockIdx.x] = sh[0];
}

// Fixed-order sum of <= a few thousand double partials (one per wave or
// workgroup): 256 lanes, U independent loads in flight per lane, then a
// fixed LDS tree.  pre = 0: output-based partials (sum dx y), divided by a^2
// -- the tape holds PReLU outputs, y < 0 marks x < 0 only while a > 0, so a
// slope <= 0 poisons da with NaN (the nets route such slopes through pre = 1,
// the pre-activation form: partials are already sum_{x<0} g x).
__global__ __launch_bounds__(256) void slope_final_kernel(const double* __restrict__ part, int n,
                                                          const float* __restrict__ a, float* __restrict__ da,
                                                          int accumulate, int pre) {
  // U loads in flight per lane: a deferred DRF region is T x 4096 doubles
  // (~1 MB at cfg 3), read by this one workgroup -- latency-bound (U = 4:
  // 64 us per PReLU, 18 finals on the step's critical path)
  constexpr int U = 16;
  __shared__ double sh[256];
  double s = 0.0;
  for (int base = threadIdx.x; base < n; base += 256 * U) {
    double v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = base + 256 * u < n ? part[base + 256 * u] : 0.0;
#pragma unroll
    for (int u = 0; u < U; ++u) s += v[u];
  }
  sh[threadIdx.x] = s;
  __syncthreads();
  for (int k = 128; k > 0; k >>= 1) {
    if (threadIdx.x < k) sh[threadIdx.x] += sh[threadIdx.x + k];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const double av = (double)*a;
    const float v = pre ? (float)sh[0] : av > 0.0 ? (float)(sh[0] / (av * av)) : __builtin_nanf("");
    *da = accumulate ? *da + v : v;
  }
}

}  // namespace

extern "C" int vsrk_subpixel_conv_weight(const float* w, const float* bias, int32_t cin, int32_t cout, int32_t k,
                                         int32_t s, int32_t p, int32_t transposed, float* weq, float* beq,
                                         void* stream) {
  VSRK_CHECK(w && weq, "subpixel_conv_weight: null pointer");
  VSRK_CHECK(s >= 1 && p >= 0 && p <= s && k <= p + 2 * s && k >= 1,
             "subpixel_conv_weight: (k=%d, s=%d, p=%d) is not a 3x3 sub-pixel conv (needs p <= s, k <= p + 2s)", k, s,
             p);
  const int cop = transposed ? s * s * cout : cout, cip = transposed ? cin : s * s * cin;
  const int64_t total = (int64_t)cop * cip * 9;
  subpixel_weight_kernel<<<(int)ceil_div64(total, 256), 256, 0, (hipStream_t)stream>>>(w, bias, cin, cout, k, s, p,
                                                                                       transposed, weq, beq, total);
  VSRK_LAUNCH_CHECK("subpixel_conv_weight");
  return VSRK_OK;
}

extern "C" int vsrk_subpixel_wgrad_fold(const float* dweq, const float* dbeq, int32_t cin, int32_t cout, int32_t k,
                                        int32_t s, int32_t p, int32_t transposed, float* dw, float* db,
                                        int32_t accumulate, void* stream) {
  VSRK_CHECK(dweq && dw, "subpixel_wgrad_fold: null pointer");
  VSRK_CHECK(!db || dbeq, "subpixel_wgrad_fold: dbias needs the equivalent dbias");
  VSRK_CHECK(s >= 1 && p >= 0 && p <= s && k <= p + 2 * s && k >= 1, "subpixel_wgrad_fold: bad (k, s, p)");
  const int64_t total = (int64_t)cin * cout * k * k;
  const int64_t n = std::max<int64_t>(total, db ? cout : 0);
  subpixel_fold_kernel<<<(int)ceil_div64(n, 256), 256, 0, (hipStream_t)stream>>>(dweq, dbeq, cin, cout, k, s, p,
                                                                                transposed, dw, db, accumulate, total);
  VSRK_LAUNCH_CHECK("subpixel_wgrad_fold");
  return VSRK_OK;
}

void vsrk_slope_final(const double* part, int nparts, const float* a, float* da, int accumulate, int pre,
                      hipStream_t s) {
  slope_final_kernel<<<1, 256, 0, s>>>(part, nparts, a, da, accumulate, pre);
}

extern "C" size_t vsrk_slope_slot_doubles(void) {  // the most partials any PReLU backward entry point writes
  return std::max<size_t>(PRELU_BLOCKS, std::max(vsrk_roll_slope_ws_bytes(), vsrk_pw_pbwd_ws_bytes()) / sizeof(double));
}

extern "C" int vsrk_slope_final_sum(const double* part, int64_t nparts, const float* a, float* da,
                                    int32_t accumulate, int32_t pre, void* stream) {
  VSRK_CHECK(part && a && da && nparts >= 0 && nparts < (1ll << 31), "slope_final_sum: bad argument");
  vsrk_slope_final(part, (int)nparts, a, da, accumulate, pre, (hipStream_t)stream);
  VSRK_LAUNCH_CHECK("slope_final_sum");
  return VSRK_OK;
}

extern "C" size_t vsrk_prelu_workspace_size(void) { return PRELU_BLOCKS * sizeof(double); }

extern "C" int vsrk_prelu_wgrad(const vsrk_tensor5* y, const vsrk_tensor5* dx, const float* a, float* da,
                                int32_t accumulate, void* workspace, size_t workspace_bytes, void* stream) {
  VSRK_CHECK(y && dx && y->ptr && dx->ptr && a && da, "prelu_wgrad: null argument");
  VSRK_CHECK(y->dtype == dx->dtype, "prelu_wgrad: dtype mismatch");
  VSRK_CHECK(y->n == dx->n && y->d == dx->d && y->h == dx->h && y->w == dx->w && y->c == dx->c,
             "prelu_wgrad: shape mismatch");
  VSRK_CHECK(y->shuffle <= 1 && dx->shuffle <= 1, "prelu_wgrad: plain views only");
  VSRK_CHECK(workspace && workspace_bytes >= vsrk_prelu_workspace_size(), "prelu_wgrad: workspace too small");
  const View vy = make_view(y), vd = make_view(dx);
  const int64_t nvox = (int64_t)y->n * y->d * y->h * y->w;
  hipStream_t s = (hipStream_t)stream;
  double* part = (double*)workspace;
  if (y->dtype == VSRK_BF16)
    prelu_partial_kernel<bf16><<<PRELU_BLOCKS, 256, 0, s>>>(vy, vd, nvox, part);
  else if (y->dtype == VSRK_F16)
    prelu_partial_kernel<f16><<<PRELU_BLOCKS, 256, 0, s>>>(vy, vd, nvox, part);
  else
    prelu_partial_kernel<float><<<PRELU_BLOCKS, 256, 0, s>>>(vy, vd, nvox, part);
  VSRK_LAUNCH_CHECK("prelu_partial");
  vsrk_slope_final(part, PRELU_BLOCKS, a, da, accumulate, 0, s);
  VSRK_LAUNCH_CHECK("prelu_final");
  return VSRK_OK;
}

// ---------------------------------------------------------------------------
// PReLU backward (drf_net.py:56-106): dx = (dy [+ dy2]) * (y > 0 ? 1 : a) and,
// in the same pass, da = sum_{y<0} dx * y / a^2, as per-block partials
// reduced in a fixed order.
namespace {
// Threads are (voxel lane vl, chunk position ch) with ch fixed; block b walks
// the (n, d, h) rows b, b + grid, ... (fixed assignment: deterministic
// partials), one 32-bit decode per row, 16-byte vector accesses when every
// view is chunk-aligned.  The first version decoded each chunk with a 64-bit
// div/mod chain and moved single bf16 elements: 99 us per call, 21 % of the
// DRF step.
template <typename T>
// pre = 0: y is the PReLU OUTPUT (x < 0 read as y < 0, exact while a > 0):
// slope partials sum dx * y, divided by a^2 in vsrk_slope_final.
// pre = 1: y is the PRE-ACTIVATION x (nn.PReLU's own saved input, any a):
// dx = x > 0 ? g : a g, slope partials sum_{x<0} g x (g = dy [+ dy2] in fp32)
__global__ __launch_bounds__(256) void prelu_bwd_kernel(View y, View dy, View dy2, int has2, const float* __restrict__ a,
                                                        View dx, int nrows, int vec, double* __restrict__ part,
                                                        int pre) {
  constexpr int E = 16 / sizeof(T);
  const int C = y.c;
  const int cpv = (C + E - 1) / E;
  const int vpb = blockDim.x / cpv;
  const int ch = threadIdx.x % cpv, vl = threadIdx.x / cpv;
  const int c0 = ch * E;
  const bool vfull = vec && c0 + E <= C;
  const float av = *a;
  double s = 0.0;
  auto roff = [](const View& v, int r) __attribute__((always_inline)) {
    const int h = r % v.h, t = r / v.h;
    return v.sn * (t / v.d) + (int64_t)(t % v.d) * v.sd + (int64_t)h * v.sh;
  };
  if (vl < vpb) {
    for (int r = blockIdx.x; r < nrows; r += gridDim.x) {
      const T* yr = reinterpret_cast<const T*>(y.ptr) + roff(y, r) + c0;
      const T* gr = reinterpret_cast<const T*>(dy.ptr) + roff(dy, r) + c0;
      const T* g2r = has2 ? reinterpret_cast<const T*>(dy2.ptr) + roff(dy2, r) + c0 : gr;
      T* orow = reinterpret_cast<T*>(dx.ptr) + roff(dx, r) + c0;
      if (vfull) {
        // U voxels per pass with every load issued first (up to 3U 16-byte
        // loads in flight per thread; one at a time streamed the high-res
        // gradients at ~2.5 TB/s); same voxel order for the slope partial
        constexpr int U = 4;
        for (int wb = vl; wb < y.w; wb += U * vpb) {
          uint4 ry[U], rg[U], rg2[U];
#pragma unroll
          for (int u = 0; u < U; ++u) {
            const int w = wb + u * vpb;
            ry[u] = rg[u] = rg2[u] = make_uint4(0, 0, 0, 0);
            if (w < y.w) {
              ry[u] = *reinterpret_cast<const uint4*>(yr + (int64_t)w * y.sw);
              rg[u] = *reinterpret_cast<const uint4*>(gr + (int64_t)w * dy.sw);
              if (has2) rg2[u] = *reinterpret_cast<const uint4*>(g2r + (int64_t)w * dy2.sw);
            }
          }
#pragma unroll
          for (int u = 0; u < U; ++u) {
            const int w = wb + u * vpb;
            if (w >= y.w) break;
            float yv[E], g[E], o[E];
            Chunk<T>::unpack(ry[u], yv);
            Chunk<T>::unpack(rg[u], g);
            if (has2) {
              float g2[E];
              Chunk<T>::unpack(rg2[u], g2);
#pragma unroll
              for (int e = 0; e < E; ++e) g[e] += g2[e];
            }
#pragma unroll
            for (int e = 0; e < E; ++e) o[e] = yv[e] > 0.f ? g[e] : av * g[e];
            const uint4 ov = Chunk<T>::pack(o);
            *reinterpret_cast<uint4*>(orow + (int64_t)w * dx.sw) = ov;
            float orr[E];
            Chunk<T>::unpack(ov, orr);  // the rounded stored value, as in the reference's dtype
            float acc = 0.f;
#pragma unroll
            for (int e = 0; e < E; ++e)
              if (yv[e] < 0.f) acc = fmaf(pre ? g[e] : orr[e], yv[e], acc);
            s += acc;
          }
        }
        continue;
      }
      for (int w = vl; w < y.w; w += vpb) {
        const T* py = yr + (int64_t)w * y.sw;
        const T* pg = gr + (int64_t)w * dy.sw;
        const T* pg2 = g2r + (int64_t)w * dy2.sw;
        T* po = orow + (int64_t)w * dx.sw;
        float acc = 0.f;
        if (vfull) {
          float yv[E], g[E], o[E];
          Chunk<T>::unpack(*reinterpret_cast<const uint4*>(py), yv);
          Chunk<T>::unpack(*reinterpret_cast<const uint4*>(pg), g);
          if (has2) {
            float g2[E];
            Chunk<T>::unpack(*reinterpret_cast<const uint4*>(pg2), g2);
#pragma unroll
            for (int e = 0; e < E; ++e) g[e] += g2[e];
          }
#pragma unroll
          for (int e = 0; e < E; ++e) o[e] = yv[e] > 0.f ? g[e] : av * g[e];
          const uint4 ov = Chunk<T>::pack(o);
          *reinterpret_cast<uint4*>(po) = ov;
          float orr[E];
          Chunk<T>::unpack(ov, orr);  // the rounded stored value, as in the reference's dtype
#pragma unroll
          for (int e = 0; e < E; ++e)
            if (yv[e] < 0.f) acc = fmaf(pre ? g[e] : orr[e], yv[e], acc);
        } else {
#pragma unroll
          for (int e = 0; e < E; ++e) {
            if (c0 + e < C) {
              const float yv = to_f32<T>(py[e]);
              float g = to_f32<T>(pg[e]);
              if (has2) g += to_f32<T>(pg2[e]);
              const T o = from_f32<T>(yv > 0.f ? g : av * g);
              po[e] = o;
              if (yv < 0.f) acc = fmaf(pre ? g : to_f32<T>(o), yv, acc);
            }
          }
        }
        s += acc;
      }
    }
  }
  __shared__ double sh[256];
  sh[threadIdx.x] = s;
  __syncthreads();
  for (int k = 128; k > 0; k >>= 1) {
    if (threadIdx.x < k) sh[threadIdx.x] += sh[threadIdx.x + k];
    __syncthreads();
  }
  if (threadIdx.x == 0) part[blockIdx.x] = sh[0];
}
}  // namespace

static int prelu_bwd_impl(const vsrk_tensor5* y, const vsrk_tensor5* dy, const vsrk_tensor5* dy2, const float* a,
                          const vsrk_tensor5* dx, float* da, int32_t accumulate_da, void* workspace,
                          size_t workspace_bytes, void* stream, int pre) {
  VSRK_CHECK(y && dy && dx && a && y->ptr && dy->ptr && dx->ptr, "prelu_bwd: null argument");
  for (const vsrk_tensor5* t : {dy, dy2, dx}) {
    if (!t) continue;
    VSRK_CHECK(t->dtype == y->dtype && t->n == y->n && t->d == y->d && t->h == y->h && t->w == y->w &&
                   t->c == y->c && t->shuffle <= 1,
               "prelu_bwd: view mismatch");
  }
  VSRK_CHECK(y->shuffle <= 1, "prelu_bwd: plain views only");
  VSRK_CHECK(workspace && workspace_bytes >= vsrk_prelu_workspace_size(), "prelu_bwd: workspace too small");
  const View vy = make_view(y), vg = make_view(dy), vo = make_view(dx);
  const View vg2 = dy2 ? make_view(dy2) : vg;
  const int64_t nr64 = (int64_t)y->n * y->d * y->h;
  VSRK_CHECK(nr64 < (1ll << 31), "prelu_bwd: too many rows");
  VSRK_CHECK(ceil_div(y->c, vsrk_is16(y->dtype) ? 8 : 4) <= 256, "prelu_bwd: too many channels (%d)", y->c);
  const int esz = vsrk_esize(y->dtype), E = 16 / esz;
  int vec = 1;
  for (const vsrk_tensor5* t : {y, dy, dy2, dx}) {
    if (!t) continue;
    if (((uintptr_t)t->ptr) % 16 || t->sn % E || t->sd % E || t->sh % E || t->sw % E) vec = 0;
  }
  VSRK_CHECK(((uintptr_t)workspace & 15) == 0, "prelu_bwd: workspace must be 16-byte aligned");
  hipStream_t s = (hipStream_t)stream;
  double* part = (double*)workspace;
  if (y->dtype == VSRK_BF16)
    prelu_bwd_kernel<bf16><<<PRELU_BLOCKS, 256, 0, s>>>(vy, vg, vg2, dy2 != nullptr, a, vo, (int)nr64, vec, part, pre);
  else if (y->dtype == VSRK_F16)
    prelu_bwd_kernel<f16><<<PRELU_BLOCKS, 256, 0, s>>>(vy, vg, vg2, dy2 != nullptr, a, vo, (int)nr64, vec, part, pre);
  else
    prelu_bwd_kernel<float><<<PRELU_BLOCKS, 256, 0, s>>>(vy, vg, vg2, dy2 != nullptr, a, vo, (int)nr64, vec, part, pre);
  VSRK_LAUNCH_CHECK("prelu_bwd");
  if (da) {  // (da == NULL: the partials stay in the workspace slot, vsrk_slope_final_sum later)
    vsrk_slope_final(part, PRELU_BLOCKS, a, da, accumulate_da, pre, s);
    VSRK_LAUNCH_CHECK("prelu_final");
  }
  return VSRK_OK;
}

extern "C" int vsrk_prelu_bwd(const vsrk_tensor5* y, const vsrk_tensor5* dy, const vsrk_tensor5* dy2, const float* a,
                              const vsrk_tensor5* dx, float* da, int32_t accumulate_da, void* workspace,
                              size_t workspace_bytes, void* stream) {
  return prelu_bwd_impl(y, dy, dy2, a, dx, da, accumulate_da, workspace, workspace_bytes, stream, 0);
}

extern "C" int vsrk_prelu_bwd_pre(const vsrk_tensor5* x, const vsrk_tensor5* dy, const vsrk_tensor5* dy2,
                                  const float* a, const vsrk_tensor5* dx, float* da, int32_t accumulate_da,
                                  void* workspace, size_t workspace_bytes, void* stream) {
  return prelu_bwd_impl(x, dy, dy2, a, dx, da, accumulate_da, workspace, workspace_bytes, stream, 1);
}
