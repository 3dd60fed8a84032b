// BatchNorm3d (training statistics) around the fused BN+ReLU conv prologue.
//
// Replaces nn.BatchNorm3d + nn.ReLU of the DUF dense blocks and tail
// (duf_net.py:116-118,195-214).  The normalisation itself is never
// materialised: the forward folds (gamma, beta, batch mean, batch var) into a
// per-channel (scale, shift) that the consuming conv applies while staging its
// input (VSRK_PRO_AFFINE_RELU).  Backward recomputes the pre-ReLU value from x.
//
// Reductions are channels-last: each thread owns one 16-byte chunk position
// (8 bf16 / 4 fp32 channels) of a run of voxels and accumulates in registers;
// the per-block partials are reduced in a fixed order in double precision
// (deterministic, and robust for sum-of-squares variance).
#include "vsrk_common.h"
#include "vsrk_internal.h"

namespace {

constexpr int RB = 2048;  // reduction blocks (partials): 8 per CU

// Row decomposition: a "row" is one (n, d, h) line of W voxels.  Threads are
// (voxel lane vl, chunk position ch) with ch fixed for the launch, so a
// thread's per-channel constants live in registers; the (n, d, h) decode is
// 32-bit and once per row, and consecutive lanes read consecutive 16-byte
// chunks of a voxel row (coalesced for dense tensors and channel slices of
// the DUF concat buffer alike).  The first version decoded every voxel with a
// 64-bit div/mod chain and re-read the per-channel tables per element: the
// BN+ReLU backward apply took 8.5 ms per launch at the DUF cfg-2 shapes.
__device__ __forceinline__ int64_t row_off(const View& v, int r) {
  const int h = r % v.h, t = r / v.h;
  const int d = t % v.d, n = t / v.d;
  return n * v.sn + (int64_t)d * v.sd + (int64_t)h * v.sh;
}

// modes: 0 = sum x, sum x^2 (stats); 1 = sum dy, sum dy*xhat with
// dy = dz * (x*scale + shift > 0) (BN+ReLU backward).  Block b reduces rows
// [b*rpb, (b+1)*rpb) into partial b (fixed order: deterministic).
template <typename T, int MODE>
__global__ __launch_bounds__(256) void chan_reduce_kernel(View x, View dz, const float* __restrict__ scale,
                                                          const float* __restrict__ shift,
                                                          const float* __restrict__ mean,
                                                          const float* __restrict__ invstd, int rpg, int bpg,
                                                          int rpb, float* __restrict__ part) {
  constexpr int E = Chunk<T>::E;
  const int C = x.c;
  const int cpv = (C + E - 1) / E;  // chunks per voxel
  const int vpb = blockDim.x / cpv; // voxel lanes (blockDim is a multiple of cpv)
  const int ch = threadIdx.x % cpv, vl = threadIdx.x / cpv;
  const int c0 = ch * E;
  const bool full = c0 + E <= C;
  float s1[E], s2[E], sc[E], sh[E], mu[E], is[E];
#pragma unroll
  for (int e = 0; e < E; ++e) {
    s1[e] = 0.f;
    s2[e] = 0.f;
    const int c = min(c0 + e, C - 1);
    if (MODE == 1) {
      sc[e] = scale[c];
      sh[e] = shift[c];
      mu[e] = mean[c];
      is[e] = invstd[c];
    }
  }
  if (vl < vpb) {
    // rows of group g = blockIdx / bpg are [g*rpg, (g+1)*rpg); this block
    // takes its rpb-row share of them
    const int g = blockIdx.x / bpg, bi = blockIdx.x - g * bpg;
    const int r0 = g * rpg + min(rpg, bi * rpb), r1 = g * rpg + min(rpg, (bi + 1) * rpb);
    // U voxels per thread per pass, all loads issued before any is used:
    // U (stats) or 2U (backward) 16-byte loads in flight per thread.  One
    // load at a time (the first version) streamed at ~3.1 TB/s.
    constexpr int U = 4;
    for (int r = r0; r < r1; ++r) {
      const T* xr = reinterpret_cast<const T*>(x.ptr) + row_off(x, r) + c0;
      const T* gr = MODE == 1 ? reinterpret_cast<const T*>(dz.ptr) + row_off(dz, r) + c0 : nullptr;
      for (int wb = vl; wb < x.w; wb += U * vpb) {
        uint4 rx[U], rg[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int w = wb + u * vpb;
          rx[u] = make_uint4(0, 0, 0, 0);
          rg[u] = make_uint4(0, 0, 0, 0);
          if (full && w < x.w) {
            rx[u] = *reinterpret_cast<const uint4*>(xr + (int64_t)w * x.sw);
            if (MODE == 1) rg[u] = *reinterpret_cast<const uint4*>(gr + (int64_t)w * dz.sw);
          }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int w = wb + u * vpb;
          if (w >= x.w) break;
          float f[E], g[E];
          if (full) {
            Chunk<T>::unpack(rx[u], f);
            if (MODE == 1) Chunk<T>::unpack(rg[u], g);
          } else {
            const T* px = xr + (int64_t)w * x.sw;
#pragma unroll
            for (int e = 0; e < E; ++e) f[e] = c0 + e < C ? to_f32<T>(px[e]) : 0.f;
            if (MODE == 1) {
              const T* pg = gr + (int64_t)w * dz.sw;
#pragma unroll
              for (int e = 0; e < E; ++e) g[e] = c0 + e < C ? to_f32<T>(pg[e]) : 0.f;
            }
          }
          if (MODE == 0) {
#pragma unroll
            for (int e = 0; e < E; ++e) {
              s1[e] += f[e];
              s2[e] = fmaf(f[e], f[e], s2[e]);
            }
          } else {
#pragma unroll
            for (int e = 0; e < E; ++e) {
              const float dy = fmaf(f[e], sc[e], sh[e]) > 0.f ? g[e] : 0.f;
              s1[e] += dy;
              s2[e] = fmaf(dy, (f[e] - mu[e]) * is[e], s2[e]);
            }
          }
        }
      }
    }
  }
  // block reduce over the vpb voxel lanes of each chunk position (fixed order)
  __shared__ float red[2][256 * 8];
#pragma unroll
  for (int e = 0; e < E; ++e) {
    red[0][threadIdx.x * E + e] = s1[e];
    red[1][threadIdx.x * E + e] = s2[e];
  }
  __syncthreads();
  for (int i = threadIdx.x; i < cpv * E; i += blockDim.x) {
    const int chk = i / E, e = i % E;
    float a = 0.f, b = 0.f;
    for (int k = 0; k < vpb; ++k) {
      a += red[0][(k * cpv + chk) * E + e];
      b += red[1][(k * cpv + chk) * E + e];
    }
    const int c = chk * E + e;
    if (c < C) {
      part[((int64_t)blockIdx.x * 2) * C + c] = a;
      part[((int64_t)blockIdx.x * 2 + 1) * C + c] = b;
    }
  }
}

// One block per channel: each thread sums a strided subset of the partials in
// double, then a fixed-shape tree (deterministic).  The first version ran one
// thread per channel over all partials serially (133 us per call, 26 calls
// per DUF step).
__global__ __launch_bounds__(256) void chan_final_kernel(const float* __restrict__ part, int bpg, int C,
                                                         float* __restrict__ o1, float* __restrict__ o2) {
  // block (c, g): channel c of row group g, whose partials are blocks
  // [g*bpg, (g+1)*bpg)
  const int c = blockIdx.x, g = blockIdx.y, t = threadIdx.x;
  double a = 0.0, b = 0.0;
  for (int k = g * bpg + t; k < (g + 1) * bpg; k += 256) {
    a += part[((int64_t)k * 2) * C + c];
    b += part[((int64_t)k * 2 + 1) * C + c];
  }
  __shared__ double ra[256], rb[256];
  ra[t] = a;
  rb[t] = b;
  __syncthreads();
  for (int off = 128; off > 0; off >>= 1) {
    if (t < off) {
      ra[t] += ra[t + off];
      rb[t] += rb[t + off];
    }
    __syncthreads();
  }
  if (t == 0) {
    o1[(int64_t)g * C + c] = (float)ra[0];
    o2[(int64_t)g * C + c] = (float)rb[0];
  }
}

// count_dev (may be null): the voxel count is count * *count_dev, read on the
// device (SyncBN: the global batch's N*H*W, all-reduced without a host read)
__global__ void bn_finalize_kernel(const float* __restrict__ sum, const float* __restrict__ sumsq, double count,
                                   const double* __restrict__ count_dev, const float* __restrict__ gamma,
                                   const float* __restrict__ beta, float eps, float momentum,
                                   float* __restrict__ rmean, float* __restrict__ rvar, float* __restrict__ scale,
                                   float* __restrict__ shift, float* __restrict__ mean, float* __restrict__ invstd,
                                   int C) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  if (count_dev) count *= *count_dev;
  const double m = (double)sum[c] / count;
  double var = (double)sumsq[c] / count - m * m;
  if (var < 0) var = 0;
  const float is = (float)(1.0 / sqrt(var + (double)eps));
  const float g = gamma ? gamma[c] : 1.f, b = beta ? beta[c] : 0.f;
  scale[c] = g * is;
  shift[c] = b - (float)m * g * is;
  mean[c] = (float)m;
  invstd[c] = is;
  if (rmean && rvar) {  // running stats: momentum update, unbiased variance (torch semantics)
    const double uvar = count > 1 ? var * count / (count - 1) : var;
    rmean[c] = (1.f - momentum) * rmean[c] + momentum * (float)m;
    rvar[c] = (1.f - momentum) * rvar[c] + momentum * (float)uvar;
  }
}

// eval mode: fold running statistics
__global__ void bn_fold_running_kernel(const float* __restrict__ gamma, const float* __restrict__ beta,
                                       const float* __restrict__ rmean, const float* __restrict__ rvar, float eps,
                                       float* __restrict__ scale, float* __restrict__ shift,
                                       float* __restrict__ mean, float* __restrict__ invstd, int C) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const float is = 1.f / sqrtf(rvar[c] + eps);
  const float g = gamma ? gamma[c] : 1.f, b = beta ? beta[c] : 0.f;
  scale[c] = g * is;
  shift[c] = b - rmean[c] * g * is;
  if (mean) mean[c] = rmean[c];
  if (invstd) invstd[c] = is;
}

// dx [+]= gamma*invstd*(dy - sum_dy/M - xhat*sum_dy_xhat/M), dy = dz*(x*scale+shift > 0),
// folded per channel into dx = k1*dy + k2*x + k3 (constants in registers).
template <typename T>
__global__ __launch_bounds__(256) void bn_relu_bwd_apply_kernel(View x, View dz, View dx,
                                                                const float* __restrict__ scale,
                                                                const float* __restrict__ shift,
                                                                const float* __restrict__ mean,
                                                                const float* __restrict__ invstd,
                                                                const float* __restrict__ gamma,
                                                                const float* __restrict__ sdy,
                                                                const float* __restrict__ sdyx, float inv_count,
                                                                int nrows, int accumulate) {
  constexpr int E = Chunk<T>::E;
  const int C = x.c;
  const int cpv = (C + E - 1) / E;
  const int vpb = blockDim.x / cpv;
  const int ch = threadIdx.x % cpv, vl = threadIdx.x / cpv;
  if (vl >= vpb) return;
  const int c0 = ch * E;
  const bool full = c0 + E <= C;
  float sc[E], sh[E], k1[E], k2[E], k3[E];
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const int c = min(c0 + e, C - 1);
    const float is = invstd[c], gm = gamma ? gamma[c] : 1.f;
    const float a = gm * is, b = is * sdyx[c] * inv_count;
    sc[e] = scale[c];
    sh[e] = shift[c];
    k1[e] = a;
    k2[e] = -a * b;
    k3[e] = a * (mean[c] * b - sdy[c] * inv_count);
  }
  for (int r = blockIdx.x; r < nrows; r += gridDim.x) {
    const T* xr = reinterpret_cast<const T*>(x.ptr) + row_off(x, r) + c0;
    const T* gr = reinterpret_cast<const T*>(dz.ptr) + row_off(dz, r) + c0;
    T* orow = reinterpret_cast<T*>(dx.ptr) + row_off(dx, r) + c0;
    // U voxels per pass, every load issued before any is used (up to 3U
    // 16-byte loads in flight per thread)
    constexpr int U = 2;
    for (int wb = vl; wb < x.w; wb += U * vpb) {
      uint4 rx[U], rg[U], ro[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int w = wb + u * vpb;
        rx[u] = rg[u] = ro[u] = make_uint4(0, 0, 0, 0);
        if (full && w < x.w) {
          rx[u] = *reinterpret_cast<const uint4*>(xr + (int64_t)w * x.sw);
          rg[u] = *reinterpret_cast<const uint4*>(gr + (int64_t)w * dz.sw);
          if (accumulate) ro[u] = *reinterpret_cast<const uint4*>(orow + (int64_t)w * dx.sw);
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int w = wb + u * vpb;
        if (w >= x.w) break;
        const T* px = xr + (int64_t)w * x.sw;
        const T* pg = gr + (int64_t)w * dz.sw;
        T* po = orow + (int64_t)w * dx.sw;
        float f[E], g[E], o[E];
        if (full) {
          Chunk<T>::unpack(rx[u], f);
          Chunk<T>::unpack(rg[u], g);
          Chunk<T>::unpack(ro[u], o);
        } else {
#pragma unroll
          for (int e = 0; e < E; ++e) {
            const bool ok = c0 + e < C;
            f[e] = ok ? to_f32<T>(px[e]) : 0.f;
            g[e] = ok ? to_f32<T>(pg[e]) : 0.f;
            o[e] = (ok && accumulate) ? to_f32<T>(po[e]) : 0.f;
          }
        }
#pragma unroll
        for (int e = 0; e < E; ++e) {
          const float dy = fmaf(f[e], sc[e], sh[e]) > 0.f ? g[e] : 0.f;
          float rr = fmaf(k1[e], dy, fmaf(k2[e], f[e], k3[e]));
          if (accumulate) rr += o[e];
          o[e] = rr;
        }
        if (full) {
          *reinterpret_cast<uint4*>(po) = Chunk<T>::pack(o);
        } else {
#pragma unroll
          for (int e = 0; e < E; ++e)
            if (c0 + e < C) po[e] = from_f32<T>(o[e]);
        }
      }
    }
  }
}

#ifndef BN_MULTI_U  // voxels per pass (A/B knob; r5 same-box DUF step: U = 4 +0.6 ms, U = 1 flat)
#define BN_MULTI_U 2
#endif
// NC contributors' BN+ReLU backward applies into one output block (see
// vsrk_bn_relu_bwd_apply_multi): the same row walk and per-thread constants
// as bn_relu_bwd_apply_kernel, x and dx moved once, each contributor's dz
// read on the rows (depths) it covers.
struct ContribDev {
  View dz;
  int d0, d1;
  const float *scale, *shift, *mean, *invstd, *gamma, *sdy, *sdyx;
  float inv_count;
};
template <int NC>
struct ContribPack {
  ContribDev c[NC];
};

template <typename T, int NC>
__global__ __launch_bounds__(256) void bn_relu_bwd_apply_multi_kernel(View x, View dx, ContribPack<NC> cp, int nrows,
                                                                      int accumulate) {
  constexpr int E = Chunk<T>::E;
  const int C = x.c;
  const int cpv = (C + E - 1) / E;
  const int vpb = blockDim.x / cpv;
  const int ch = threadIdx.x % cpv, vl = threadIdx.x / cpv;
  if (vl >= vpb) return;
  const int c0 = ch * E;
  const bool full = c0 + E <= C;
  float sc[NC][E], sh[NC][E], k1[NC][E], k2[NC][E], k3[NC][E];
#pragma unroll
  for (int i = 0; i < NC; ++i)
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const ContribDev& q = cp.c[i];
      const int c = min(c0 + e, C - 1);
      const float is = q.invstd[c], gm = q.gamma ? q.gamma[c] : 1.f;
      const float a = gm * is, b = is * q.sdyx[c] * q.inv_count;
      sc[i][e] = q.scale[c];
      sh[i][e] = q.shift[c];
      k1[i][e] = a;
      k2[i][e] = -a * b;
      k3[i][e] = a * (q.mean[c] * b - q.sdy[c] * q.inv_count);
    }
  for (int r = blockIdx.x; r < nrows; r += gridDim.x) {
    const int h = r % x.h, t = r / x.h, d = t % x.d, n = t / x.d;
    const T* xr = reinterpret_cast<const T*>(x.ptr) + row_off(x, r) + c0;
    T* orow = reinterpret_cast<T*>(dx.ptr) + row_off(dx, r) + c0;
    const T* gr[NC];
    bool on[NC];
#pragma unroll
    for (int i = 0; i < NC; ++i) {
      const ContribDev& q = cp.c[i];
      on[i] = d >= q.d0 && d < q.d1;
      gr[i] = reinterpret_cast<const T*>(q.dz.ptr) +
              (n * q.dz.sn + (int64_t)(on[i] ? d - q.d0 : 0) * q.dz.sd + (int64_t)h * q.dz.sh) + c0;
    }
    // U voxels per pass with every load (x, dx, each active dz) issued before
    // any is used; a scalar path for a partial last chunk
    constexpr int U = BN_MULTI_U;
    for (int wb = vl; wb < x.w; wb += U * vpb) {
      uint4 rx[U], ro[U], rg[NC][U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int w = wb + u * vpb;
        const bool ok = full && w < x.w;
        rx[u] = ok ? *reinterpret_cast<const uint4*>(xr + (int64_t)w * x.sw) : make_uint4(0, 0, 0, 0);
        ro[u] = (ok && accumulate) ? *reinterpret_cast<const uint4*>(orow + (int64_t)w * dx.sw)
                                   : make_uint4(0, 0, 0, 0);
#pragma unroll
        for (int i = 0; i < NC; ++i)
          rg[i][u] = (ok && on[i]) ? *reinterpret_cast<const uint4*>(gr[i] + (int64_t)w * cp.c[i].dz.sw)
                                   : make_uint4(0, 0, 0, 0);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int w = wb + u * vpb;
        if (w >= x.w) break;
        float f[E], o[E], g[NC][E];
        if (full) {
          Chunk<T>::unpack(rx[u], f);
          Chunk<T>::unpack(ro[u], o);
#pragma unroll
          for (int i = 0; i < NC; ++i) Chunk<T>::unpack(rg[i][u], g[i]);
        } else {
#pragma unroll
          for (int e = 0; e < E; ++e) {
            const bool ok = c0 + e < C;
            f[e] = ok ? to_f32<T>(xr[(int64_t)w * x.sw + e]) : 0.f;
            o[e] = (ok && accumulate) ? to_f32<T>(orow[(int64_t)w * dx.sw + e]) : 0.f;
#pragma unroll
            for (int i = 0; i < NC; ++i)
              g[i][e] = (ok && on[i]) ? to_f32<T>(gr[i][(int64_t)w * cp.c[i].dz.sw + e]) : 0.f;
          }
        }
#pragma unroll
        for (int i = 0; i < NC; ++i) {
          if (!on[i]) continue;  // uniform per row
#pragma unroll
          for (int e = 0; e < E; ++e) {
            const float dy = fmaf(f[e], sc[i][e], sh[i][e]) > 0.f ? g[i][e] : 0.f;
            o[e] += fmaf(k1[i][e], dy, fmaf(k2[i][e], f[e], k3[i][e]));
          }
        }
        T* po = orow + (int64_t)w * dx.sw;
        if (full) {
          *reinterpret_cast<uint4*>(po) = Chunk<T>::pack(o);
        } else {
#pragma unroll
          for (int e = 0; e < E; ++e)
            if (c0 + e < C) po[e] = from_f32<T>(o[e]);
        }
      }
    }
  }
}

// The same for 4..8 contributors in ONE pass (round 5 split them into passes
// of three, each re-reading the block's x and dx: DUF's head block took three
// passes, its first three unit blocks two).  The per-channel constants of
// every contributor (scale, shift, k1, k2, k3) live in LDS instead of
// registers (40 floats per contributor and thread would not fit); a row reads
// each active contributor's five 8-channel groups once for its U voxels.
// Same fp32 operations in the same contributor order as the register form.
constexpr int BN_MULTI_LDS_C = 256;  // channels per block the LDS form takes
template <typename T, int NC>
__global__ __launch_bounds__(256) void bn_relu_bwd_apply_multi_lds_kernel(View x, View dx, ContribPack<NC> cp,
                                                                          int nrows, int accumulate) {
  constexpr int E = Chunk<T>::E;
  const int C = x.c;
  const int cpv = (C + E - 1) / E;
  const int vpb = blockDim.x / cpv;
  const int ch = threadIdx.x % cpv, vl = threadIdx.x / cpv;
  const int c0 = ch * E;
  const bool full = c0 + E <= C;
  const int CP = cpv * E;  // padded channel count of the tables
  __shared__ __attribute__((aligned(16))) float cst[NC * 5 * BN_MULTI_LDS_C];  // [i][sc, sh, k1, k2, k3][CP]
  for (int j = threadIdx.x; j < NC * CP; j += blockDim.x) {
    const int i = j / CP, cc = j - i * CP;
    const ContribDev& q = cp.c[i];
    const int c = min(cc, C - 1);
    const float is = q.invstd[c], gm = q.gamma ? q.gamma[c] : 1.f;
    const float a = gm * is, b = is * q.sdyx[c] * q.inv_count;
    float* t = cst + i * 5 * CP + cc;
    t[0] = q.scale[c];
    t[CP] = q.shift[c];
    t[2 * CP] = a;
    t[3 * CP] = -a * b;
    t[4 * CP] = a * (q.mean[c] * b - q.sdy[c] * q.inv_count);
  }
  __syncthreads();
  if (vl >= vpb) return;
  for (int r = blockIdx.x; r < nrows; r += gridDim.x) {
    const int h = r % x.h, t = r / x.h, d = t % x.d, n = t / x.d;
    const T* xr = reinterpret_cast<const T*>(x.ptr) + row_off(x, r) + c0;
    T* orow = reinterpret_cast<T*>(dx.ptr) + row_off(dx, r) + c0;
    const T* gr[NC];
    bool on[NC];
#pragma unroll
    for (int i = 0; i < NC; ++i) {
      const ContribDev& q = cp.c[i];
      on[i] = d >= q.d0 && d < q.d1;
      gr[i] = reinterpret_cast<const T*>(q.dz.ptr) +
              (n * q.dz.sn + (int64_t)(on[i] ? d - q.d0 : 0) * q.dz.sd + (int64_t)h * q.dz.sh) + c0;
    }
    constexpr int U = BN_MULTI_U;
    for (int wb = vl; wb < x.w; wb += U * vpb) {
      uint4 rx[U], ro[U], rg[NC][U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int w = wb + u * vpb;
        const bool ok = full && w < x.w;
        rx[u] = ok ? *reinterpret_cast<const uint4*>(xr + (int64_t)w * x.sw) : make_uint4(0, 0, 0, 0);
        ro[u] = (ok && accumulate) ? *reinterpret_cast<const uint4*>(orow + (int64_t)w * dx.sw)
                                   : make_uint4(0, 0, 0, 0);
#pragma unroll
        for (int i = 0; i < NC; ++i)
          rg[i][u] = (ok && on[i]) ? *reinterpret_cast<const uint4*>(gr[i] + (int64_t)w * cp.c[i].dz.sw)
                                   : make_uint4(0, 0, 0, 0);
      }
      float f[U][E], o[U][E];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int w = wb + u * vpb;
        if (full) {
          Chunk<T>::unpack(rx[u], f[u]);
          Chunk<T>::unpack(ro[u], o[u]);
        } else {
#pragma unroll
          for (int e = 0; e < E; ++e) {
            const bool ok = c0 + e < C && w < x.w;
            f[u][e] = ok ? to_f32<T>(xr[(int64_t)w * x.sw + e]) : 0.f;
            o[u][e] = (ok && accumulate) ? to_f32<T>(orow[(int64_t)w * dx.sw + e]) : 0.f;
          }
        }
      }
#pragma unroll
      for (int i = 0; i < NC; ++i) {
        if (!on[i]) continue;  // uniform per row
        float k[5][E];
#pragma unroll
        for (int j = 0; j < 5; ++j)
#pragma unroll
          for (int e = 0; e < E; e += 4)
            *reinterpret_cast<float4*>(&k[j][e]) = *reinterpret_cast<const float4*>(cst + (i * 5 + j) * CP + c0 + e);
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int w = wb + u * vpb;
          float g[E];
          if (full) {
            Chunk<T>::unpack(rg[i][u], g);
          } else {
#pragma unroll
            for (int e = 0; e < E; ++e)
              g[e] = (c0 + e < C && w < x.w) ? to_f32<T>(gr[i][(int64_t)w * cp.c[i].dz.sw + e]) : 0.f;
          }
#pragma unroll
          for (int e = 0; e < E; ++e) {
            const float dy = fmaf(f[u][e], k[0][e], k[1][e]) > 0.f ? g[e] : 0.f;
            o[u][e] += fmaf(k[2][e], dy, fmaf(k[3][e], f[u][e], k[4][e]));
          }
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int w = wb + u * vpb;
        if (w >= x.w) break;
        T* po = orow + (int64_t)w * dx.sw;
        if (full) {
          *reinterpret_cast<uint4*>(po) = Chunk<T>::pack(o[u]);
        } else {
#pragma unroll
          for (int e = 0; e < E; ++e)
            if (c0 + e < C) po[e] = from_f32<T>(o[u][e]);
        }
      }
    }
  }
}

template <typename T, int NC>
void launch_apply_multi(const vsrk_tensor5* x, const vsrk_tensor5* dx, int accumulate, const vsrk_bn_contrib* cs,
                        int grid, int thr, int nrows, hipStream_t s) {
  ContribPack<NC> cp;
  for (int i = 0; i < NC; ++i) {
    const vsrk_bn_contrib& q = cs[i];
    cp.c[i] = ContribDev{make_view(&q.dz), q.d0, q.d0 + q.dz.d, q.scale, q.shift, q.mean, q.invstd, q.gamma,
                         q.sum_dy, q.sum_dy_xhat, (float)(1.0 / q.count)};
  }
  if constexpr (NC <= 3)
    bn_relu_bwd_apply_multi_kernel<T, NC><<<grid, thr, 0, s>>>(make_view(x), make_view(dx), cp, nrows, accumulate);
  else
    bn_relu_bwd_apply_multi_lds_kernel<T, NC><<<grid, thr, 0, s>>>(make_view(x), make_view(dx), cp, nrows,
                                                                   accumulate);
}

// y = x * scale + shift [relu] per channel (the standalone BatchNorm3d forward
// of the op-level modules; the generators fold it into the next conv instead)
template <typename T>
__global__ __launch_bounds__(256) void bn_apply_kernel(View x, View y, const float* __restrict__ scale,
                                                       const float* __restrict__ shift, int relu, int nrows) {
  constexpr int E = Chunk<T>::E;
  const int C = x.c;
  const int cpv = (C + E - 1) / E;
  const int vpb = blockDim.x / cpv;
  const int ch = threadIdx.x % cpv, vl = threadIdx.x / cpv;
  if (vl >= vpb) return;
  const int c0 = ch * E;
  const bool full = c0 + E <= C;
  float sc[E], sh[E];
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const int c = min(c0 + e, C - 1);
    sc[e] = scale[c];
    sh[e] = shift[c];
  }
  for (int r = blockIdx.x; r < nrows; r += gridDim.x) {
    const T* xr = reinterpret_cast<const T*>(x.ptr) + row_off(x, r) + c0;
    T* yr = reinterpret_cast<T*>(y.ptr) + row_off(y, r) + c0;
    for (int w = vl; w < x.w; w += vpb) {
      const T* px = xr + (int64_t)w * x.sw;
      T* py = yr + (int64_t)w * y.sw;
      float f[E];
      if (full) {
        Chunk<T>::unpack(*reinterpret_cast<const uint4*>(px), f);
      } else {
#pragma unroll
        for (int e = 0; e < E; ++e) f[e] = c0 + e < C ? to_f32<T>(px[e]) : 0.f;
      }
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const float t = fmaf(f[e], sc[e], sh[e]);
        f[e] = relu ? fmaxf(t, 0.f) : t;
      }
      if (full) {
        *reinterpret_cast<uint4*>(py) = Chunk<T>::pack(f);
      } else {
#pragma unroll
        for (int e = 0; e < E; ++e)
          if (c0 + e < C) py[e] = from_f32<T>(f[e]);
      }
    }
  }
}

int reduce_launch(int mode, const vsrk_tensor5* x, const vsrk_tensor5* dz, const float* scale, const float* shift,
                  const float* mean, const float* invstd, float* o1, float* o2, void* ws, size_t ws_bytes,
                  hipStream_t s, int groups = 1) {
  const int E = vsrk_is16(x->dtype) ? 8 : 4;
  const int cpv = ceil_div(x->c, E);
  VSRK_CHECK(cpv <= 256, "bn: too many channels (%d)", x->c);
  const int vpb = 256 / cpv;
  const int64_t nr64 = (int64_t)x->n * x->d * x->h;
  VSRK_CHECK(nr64 < (1ll << 31), "bn: too many rows");
  const int nrows = (int)nr64;
  VSRK_CHECK(groups >= 1 && groups <= RB && nrows % groups == 0, "bn: %d rows do not split into %d groups", nrows,
             groups);
  const int rpg = nrows / groups;
  const int bpg = std::max(1, std::min(rpg, RB / groups));  // blocks per group
  const int rpb = std::max(1, ceil_div(rpg, bpg));
  const int nblk = groups * bpg;
  const size_t need = (size_t)nblk * 2 * x->c * sizeof(float);
  VSRK_CHECK(ws && ws_bytes >= need, "bn: workspace %zu < %zu bytes", ws_bytes, need);
  VSRK_CHECK(x->shuffle <= 1 && (!dz || (dz->shuffle <= 1 && dz->n == x->n && dz->d == x->d && dz->h == x->h &&
                                         dz->w == x->w)),
             "bn: sub-pixel views / mismatched x, dz shapes are not supported");
  if (nrows == 0) return VSRK_OK;
  View vx = make_view(x);
  View vg = dz ? make_view(dz) : vx;
  float* part = (float*)ws;
  const int thr = cpv * vpb;
  if (x->dtype == VSRK_BF16) {
    if (mode == 0) chan_reduce_kernel<bf16, 0><<<nblk, thr, 0, s>>>(vx, vg, scale, shift, mean, invstd, rpg, bpg, rpb, part);
    else chan_reduce_kernel<bf16, 1><<<nblk, thr, 0, s>>>(vx, vg, scale, shift, mean, invstd, rpg, bpg, rpb, part);
  } else if (x->dtype == VSRK_F16) {
    if (mode == 0) chan_reduce_kernel<f16, 0><<<nblk, thr, 0, s>>>(vx, vg, scale, shift, mean, invstd, rpg, bpg, rpb, part);
    else chan_reduce_kernel<f16, 1><<<nblk, thr, 0, s>>>(vx, vg, scale, shift, mean, invstd, rpg, bpg, rpb, part);
  } else {
    if (mode == 0) chan_reduce_kernel<float, 0><<<nblk, thr, 0, s>>>(vx, vg, scale, shift, mean, invstd, rpg, bpg, rpb, part);
    else chan_reduce_kernel<float, 1><<<nblk, thr, 0, s>>>(vx, vg, scale, shift, mean, invstd, rpg, bpg, rpb, part);
  }
  VSRK_LAUNCH_CHECK("bn_reduce");
  chan_final_kernel<<<dim3(x->c, groups), 256, 0, s>>>(part, bpg, x->c, o1, o2);
  VSRK_LAUNCH_CHECK("bn_reduce_final");
  return VSRK_OK;
}

}  // namespace

extern "C" size_t vsrk_bn_workspace_size(int32_t channels) { return (size_t)RB * 2 * channels * sizeof(float); }

extern "C" int vsrk_bn_stats(const vsrk_tensor5* x, float* sum, float* sumsq, void* workspace,
                             size_t workspace_bytes, void* stream) {
  VSRK_CHECK(x && x->ptr && sum && sumsq, "bn_stats: null argument");
  return reduce_launch(0, x, nullptr, nullptr, nullptr, nullptr, nullptr, sum, sumsq, workspace, workspace_bytes,
                       (hipStream_t)stream);
}

extern "C" int vsrk_bn_stats_grouped(const vsrk_tensor5* x, int32_t groups, float* sum, float* sumsq,
                                     void* workspace, size_t workspace_bytes, void* stream) {
  VSRK_CHECK(x && x->ptr && sum && sumsq, "bn_stats_grouped: null argument");
  return reduce_launch(0, x, nullptr, nullptr, nullptr, nullptr, nullptr, sum, sumsq, workspace, workspace_bytes,
                       (hipStream_t)stream, groups);
}

extern "C" int vsrk_bn_finalize(const float* sum, const float* sumsq, double count, const float* gamma,
                                const float* beta, float eps, float momentum, float* running_mean,
                                float* running_var, float* scale, float* shift, float* mean, float* invstd,
                                int32_t channels, void* stream) {
  VSRK_CHECK(sum && sumsq && scale && shift && mean && invstd && count > 0, "bn_finalize: bad argument");
  bn_finalize_kernel<<<ceil_div(channels, 256), 256, 0, (hipStream_t)stream>>>(
      sum, sumsq, count, nullptr, gamma, beta, eps, momentum, running_mean, running_var, scale, shift, mean, invstd,
      channels);
  VSRK_LAUNCH_CHECK("bn_finalize");
  return VSRK_OK;
}

extern "C" int vsrk_bn_finalize_dcount(const float* sum, const float* sumsq, const double* count_dev,
                                       double count_mult, const float* gamma, const float* beta, float eps,
                                       float momentum, float* running_mean, float* running_var, float* scale,
                                       float* shift, float* mean, float* invstd, int32_t channels, void* stream) {
  VSRK_CHECK(sum && sumsq && count_dev && scale && shift && mean && invstd && count_mult > 0,
             "bn_finalize_dcount: bad argument");
  bn_finalize_kernel<<<ceil_div(channels, 256), 256, 0, (hipStream_t)stream>>>(
      sum, sumsq, count_mult, count_dev, gamma, beta, eps, momentum, running_mean, running_var, scale, shift, mean,
      invstd, channels);
  VSRK_LAUNCH_CHECK("bn_finalize_dcount");
  return VSRK_OK;
}

extern "C" int vsrk_bn_fold_running(const float* gamma, const float* beta, const float* running_mean,
                                    const float* running_var, float eps, float* scale, float* shift, float* mean,
                                    float* invstd, int32_t channels, void* stream) {
  VSRK_CHECK(running_mean && running_var && scale && shift, "bn_fold_running: null argument");
  bn_fold_running_kernel<<<ceil_div(channels, 256), 256, 0, (hipStream_t)stream>>>(
      gamma, beta, running_mean, running_var, eps, scale, shift, mean, invstd, channels);
  VSRK_LAUNCH_CHECK("bn_fold_running");
  return VSRK_OK;
}

extern "C" int vsrk_bn_relu_bwd_reduce(const vsrk_tensor5* x, const vsrk_tensor5* dz, const float* scale,
                                       const float* shift, const float* mean, const float* invstd, float* sum_dy,
                                       float* sum_dy_xhat, void* workspace, size_t workspace_bytes, void* stream) {
  VSRK_CHECK(x && dz && scale && shift && mean && invstd && sum_dy && sum_dy_xhat, "bn_relu_bwd_reduce: null");
  VSRK_CHECK(x->dtype == dz->dtype && x->c == dz->c, "bn_relu_bwd_reduce: x/dz mismatch");
  return reduce_launch(1, x, dz, scale, shift, mean, invstd, sum_dy, sum_dy_xhat, workspace, workspace_bytes,
                       (hipStream_t)stream);
}

extern "C" int vsrk_bn_relu_bwd_apply(const vsrk_tensor5* x, const vsrk_tensor5* dz, const float* scale,
                                      const float* shift, const float* mean, const float* invstd,
                                      const float* gamma, const float* sum_dy, const float* sum_dy_xhat,
                                      double count, const vsrk_tensor5* dx, int32_t accumulate, void* stream) {
  VSRK_CHECK(x && dz && dx && scale && shift && mean && invstd && sum_dy && sum_dy_xhat, "bn_relu_bwd_apply: null");
  VSRK_CHECK(x->dtype == dz->dtype && x->dtype == dx->dtype && x->c == dz->c && x->c == dx->c,
             "bn_relu_bwd_apply: view mismatch");
  const int E = vsrk_is16(x->dtype) ? 8 : 4;
  const int cpv = ceil_div(x->c, E);
  VSRK_CHECK(cpv <= 256, "bn_relu_bwd_apply: too many channels (%d)", x->c);
  VSRK_CHECK(dz->n == x->n && dz->d == x->d && dz->h == x->h && dz->w == x->w && dx->n == x->n &&
                 dx->d == x->d && dx->h == x->h && dx->w == x->w && x->shuffle <= 1 && dz->shuffle <= 1 &&
                 dx->shuffle <= 1,
             "bn_relu_bwd_apply: view shape mismatch");
  const int64_t nr64 = (int64_t)x->n * x->d * x->h;
  VSRK_CHECK(nr64 < (1ll << 31), "bn_relu_bwd_apply: too many rows");
  const int nrows = (int)nr64;
  const int thr = cpv * (256 / cpv);
  const int grid = std::min(nrows, 4096);
  hipStream_t s = (hipStream_t)stream;
  if (x->dtype == VSRK_BF16)
    bn_relu_bwd_apply_kernel<bf16><<<grid, thr, 0, s>>>(make_view(x), make_view(dz), make_view(dx), scale, shift,
                                                        mean, invstd, gamma, sum_dy, sum_dy_xhat,
                                                        (float)(1.0 / count), nrows, accumulate);
  else if (x->dtype == VSRK_F16)
    bn_relu_bwd_apply_kernel<f16><<<grid, thr, 0, s>>>(make_view(x), make_view(dz), make_view(dx), scale, shift,
                                                        mean, invstd, gamma, sum_dy, sum_dy_xhat,
                                                        (float)(1.0 / count), nrows, accumulate);
  else
    bn_relu_bwd_apply_kernel<float><<<grid, thr, 0, s>>>(make_view(x), make_view(dz), make_view(dx), scale, shift,
                                                         mean, invstd, gamma, sum_dy, sum_dy_xhat,
                                                         (float)(1.0 / count), nrows, accumulate);
  VSRK_LAUNCH_CHECK("bn_relu_bwd_apply");
  return VSRK_OK;
}

extern "C" int vsrk_bn_relu_bwd_apply_multi(const vsrk_tensor5* x, const vsrk_tensor5* dx, int32_t accumulate,
                                            int32_t n, const vsrk_bn_contrib* cs, void* stream) {
  VSRK_CHECK(x && dx && cs && n >= 1 && n <= VSRK_BN_MULTI_MAX, "bn_relu_bwd_apply_multi: bad argument");
  VSRK_CHECK(x->dtype == dx->dtype && x->c == dx->c && x->n == dx->n && x->d == dx->d && x->h == dx->h &&
                 x->w == dx->w && x->shuffle <= 1 && dx->shuffle <= 1,
             "bn_relu_bwd_apply_multi: x / dx mismatch");
  for (int i = 0; i < n; ++i) {
    const vsrk_bn_contrib& q = cs[i];
    VSRK_CHECK(q.dz.ptr && q.scale && q.shift && q.mean && q.invstd && q.sum_dy && q.sum_dy_xhat && q.count > 0,
               "bn_relu_bwd_apply_multi: contributor %d: null operand", i);
    VSRK_CHECK(q.dz.dtype == x->dtype && q.dz.c == x->c && q.dz.n == x->n && q.dz.h == x->h && q.dz.w == x->w &&
                   q.d0 >= 0 && q.d0 + q.dz.d <= x->d && q.dz.shuffle <= 1,
               "bn_relu_bwd_apply_multi: contributor %d does not fit the block", i);
  }
  const int E = vsrk_is16(x->dtype) ? 8 : 4;
  const int cpv = ceil_div(x->c, E);
  VSRK_CHECK(cpv <= 256, "bn_relu_bwd_apply_multi: too many channels (%d)", x->c);
  VSRK_CHECK(n <= 3 || cpv * E <= BN_MULTI_LDS_C,
             "bn_relu_bwd_apply_multi: more than 3 contributors need a block of <= %d channels (%d)", BN_MULTI_LDS_C,
             x->c);
  const int64_t nr64 = (int64_t)x->n * x->d * x->h;
  VSRK_CHECK(nr64 < (1ll << 31), "bn_relu_bwd_apply_multi: too many rows");
  const int nrows = (int)nr64;
  if (nrows == 0) return VSRK_OK;
  const int thr = cpv * (256 / cpv);
  const int grid = std::min(nrows, 4096);
  hipStream_t s = (hipStream_t)stream;
  auto go = [&](auto tag) {
    using T = decltype(tag);
    switch (n) {
      case 1: launch_apply_multi<T, 1>(x, dx, accumulate, cs, grid, thr, nrows, s); break;
      case 2: launch_apply_multi<T, 2>(x, dx, accumulate, cs, grid, thr, nrows, s); break;
      case 3: launch_apply_multi<T, 3>(x, dx, accumulate, cs, grid, thr, nrows, s); break;
      case 4: launch_apply_multi<T, 4>(x, dx, accumulate, cs, grid, thr, nrows, s); break;
      case 5: launch_apply_multi<T, 5>(x, dx, accumulate, cs, grid, thr, nrows, s); break;
      case 6: launch_apply_multi<T, 6>(x, dx, accumulate, cs, grid, thr, nrows, s); break;
      case 7: launch_apply_multi<T, 7>(x, dx, accumulate, cs, grid, thr, nrows, s); break;
      default: launch_apply_multi<T, 8>(x, dx, accumulate, cs, grid, thr, nrows, s); break;
    }
  };
  if (x->dtype == VSRK_BF16) go(bf16{});
  else if (x->dtype == VSRK_F16) go(f16{});
  else go(float{});
  VSRK_LAUNCH_CHECK("bn_relu_bwd_apply_multi");
  return VSRK_OK;
}

extern "C" int vsrk_bn_apply(const vsrk_tensor5* x, const float* scale, const float* shift, int32_t relu,
                             const vsrk_tensor5* y, void* stream) {
  VSRK_CHECK(x && y && x->ptr && y->ptr && scale && shift, "bn_apply: null argument");
  VSRK_CHECK(x->dtype == y->dtype && x->c == y->c && x->n == y->n && x->d == y->d && x->h == y->h && x->w == y->w &&
                 x->shuffle <= 1 && y->shuffle <= 1,
             "bn_apply: view mismatch");
  const int E = vsrk_is16(x->dtype) ? 8 : 4;
  const int cpv = ceil_div(x->c, E);
  VSRK_CHECK(cpv <= 256, "bn_apply: too many channels (%d)", x->c);
  const int64_t nr64 = (int64_t)x->n * x->d * x->h;
  VSRK_CHECK(nr64 < (1ll << 31), "bn_apply: too many rows");
  const int nrows = (int)nr64;
  if (nrows == 0) return VSRK_OK;
  const int thr = cpv * (256 / cpv);
  const int grid = std::min(nrows, 4096);
  hipStream_t s = (hipStream_t)stream;
  if (x->dtype == VSRK_BF16)
    bn_apply_kernel<bf16><<<grid, thr, 0, s>>>(make_view(x), make_view(y), scale, shift, relu, nrows);
  else if (x->dtype == VSRK_F16)
    bn_apply_kernel<f16><<<grid, thr, 0, s>>>(make_view(x), make_view(y), scale, shift, relu, nrows);
  else
    bn_apply_kernel<float><<<grid, thr, 0, s>>>(make_view(x), make_view(y), scale, shift, relu, nrows);
  VSRK_LAUNCH_CHECK("bn_apply");
  return VSRK_OK;
}
