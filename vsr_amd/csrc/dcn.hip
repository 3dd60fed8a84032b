// Modulated deformable convolution (DCNv2) and deformable convolution (DCNv1)
// sampling kernels for gfx950: the EDVR alignment op of the reference
// (edvr_net/dcn/src/deform_conv_cuda_kernel.cu:189-766, deform_conv.py:97-330).
//
// Split as the reference splits it -- sample (im2col), contraction, and the
// two backward scatters -- but laid out channels-last so the contraction is
// the library's MFMA 1x1 conv (cols (N, Ho, Wo, K*C) x W' (Cout, K*C)) and
// every sampling thread moves 16-byte channel vectors:
//   dcn_im2col:     cols[n,ho,wo,k*C+c] = m * bilinear(x[n,:,:,c], p_k + off)
//   dcn_col2im:     grad_x[n,y,x,c] += m * w_corner * gcols[n,ho,wo,k*C+c]
//                   (float atomics, as the reference's col2im: the one
//                   non-fixed-order sum of the library)
//   dcn_coord_grad: grad_off[n,(g*K+k)*2+{0,1},ho,wo] = sum_c gcols * m * d bilinear/d{h,w}
//                   grad_mask[n,g*K+k,ho,wo]        = sum_c gcols * bilinear
//                   (one thread per (n,ho,wo,g,k), channels in order: deterministic)
// Sampling rule (dmcn_im2col_bilinear, .cu:467-498 / :600-625): position
// h = ho*sh - ph + i*dh + off_h (w likewise); sampled when -1 < h < H and
// -1 < w < W, corners outside the image read as zero.  offset (N, G*2*K,
// Ho, Wo) and mask (N, G*K, Ho, Wo) keep the reference's NCHW layout; x,
// cols, grad_x, gcols are channels-last fp32.
#include "vsrk_common.h"
#include "../../include/vsrk_dcn.h"

namespace {

struct DcnGeom {
  int n, h, w, c, ho, wo, kh, kw, sh, sw, ph, pw, dh, dw, groups;  // groups = deformable groups
};

struct Sample {
  float hs, ws;  // sampling position
  float m;       // modulation (1 without a mask)
  bool ok;
};

__device__ __forceinline__ Sample sample_at(const DcnGeom& g, const float* __restrict__ off,
                                            const float* __restrict__ msk, int n, int oy, int ox, int grp, int k) {
  const int K = g.kh * g.kw, i = k / g.kw, j = k - (k / g.kw) * g.kw;
  const int64_t plane = (int64_t)g.ho * g.wo, pix = (int64_t)oy * g.wo + ox;
  const float* ob = off + ((int64_t)n * g.groups * 2 * K + (int64_t)(grp * K + k) * 2) * plane;
  Sample s;
  s.hs = (float)(oy * g.sh - g.ph + i * g.dh) + ob[pix];
  s.ws = (float)(ox * g.sw - g.pw + j * g.dw) + ob[plane + pix];
  s.m = msk ? msk[((int64_t)n * g.groups * K + grp * K + k) * plane + pix] : 1.f;
  s.ok = s.hs > -1.f && s.ws > -1.f && s.hs < (float)g.h && s.ws < (float)g.w;
  return s;
}

// bilinear corners: weights w[4] and in-image flags for (hl,wl),(hl,wh),(hh,wl),(hh,wh)
struct Corners {
  int hl, wl;
  float wt[4];
  bool in[4];
};

__device__ __forceinline__ Corners corners(float hs, float ws, int H, int W) {
  Corners c;
  c.hl = (int)floorf(hs);
  c.wl = (int)floorf(ws);
  const float lh = hs - c.hl, lw = ws - c.wl, hh = 1.f - lh, hw = 1.f - lw;
  c.wt[0] = hh * hw;
  c.wt[1] = hh * lw;
  c.wt[2] = lh * hw;
  c.wt[3] = lh * lw;
  c.in[0] = c.hl >= 0 && c.wl >= 0;
  c.in[1] = c.hl >= 0 && c.wl + 1 <= W - 1;
  c.in[2] = c.hl + 1 <= H - 1 && c.wl >= 0;
  c.in[3] = c.hl + 1 <= H - 1 && c.wl + 1 <= W - 1;
  return c;
}

__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }

// one thread per (n, ho, wo, k, 4-channel vector)
__global__ __launch_bounds__(256) void dcn_im2col_kernel(DcnGeom g, const float* __restrict__ x,
                                                         const float* __restrict__ off, const float* __restrict__ msk,
                                                         float* __restrict__ cols, int64_t total) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= total) return;
  const int C4 = g.c / 4, K = g.kh * g.kw;
  const int c4 = (int)(idx % C4);
  int64_t r = idx / C4;
  const int k = (int)(r % K);
  r /= K;
  const int ox = (int)(r % g.wo);
  r /= g.wo;
  const int oy = (int)(r % g.ho);
  const int n = (int)(r / g.ho);
  const int c = 4 * c4, grp = c / (g.c / g.groups);
  const Sample s = sample_at(g, off, msk, n, oy, ox, grp, k);
  float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
  if (s.ok) {
    const Corners q = corners(s.hs, s.ws, g.h, g.w);
    const float* xb = x + (int64_t)n * g.h * g.w * g.c + c;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      if (!q.in[t]) continue;
      const int yy = q.hl + (t >> 1), xx = q.wl + (t & 1);
      const float4 u = ld4(xb + ((int64_t)yy * g.w + xx) * g.c);
      v.x += q.wt[t] * u.x;
      v.y += q.wt[t] * u.y;
      v.z += q.wt[t] * u.z;
      v.w += q.wt[t] * u.w;
    }
  }
  v.x *= s.m;
  v.y *= s.m;
  v.z *= s.m;
  v.w *= s.m;
  *reinterpret_cast<float4*>(cols + ((((int64_t)n * g.ho + oy) * g.wo + ox) * K + k) * g.c + c) = v;
}

__global__ __launch_bounds__(256) void dcn_col2im_kernel(DcnGeom g, const float* __restrict__ gcols,
                                                         const float* __restrict__ off, const float* __restrict__ msk,
                                                         float* __restrict__ gx, int64_t total) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= total) return;
  const int C4 = g.c / 4, K = g.kh * g.kw;
  const int c4 = (int)(idx % C4);
  int64_t r = idx / C4;
  const int k = (int)(r % K);
  r /= K;
  const int ox = (int)(r % g.wo);
  r /= g.wo;
  const int oy = (int)(r % g.ho);
  const int n = (int)(r / g.ho);
  const int c = 4 * c4, grp = c / (g.c / g.groups);
  const Sample s = sample_at(g, off, msk, n, oy, ox, grp, k);
  if (!s.ok) return;
  const float4 gv = ld4(gcols + ((((int64_t)n * g.ho + oy) * g.wo + ox) * K + k) * g.c + c);
  const Corners q = corners(s.hs, s.ws, g.h, g.w);
  float* xb = gx + (int64_t)n * g.h * g.w * g.c + c;
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    if (!q.in[t]) continue;
    const int yy = q.hl + (t >> 1), xx = q.wl + (t & 1);
    const float f = q.wt[t] * s.m;
    float* p = xb + ((int64_t)yy * g.w + xx) * g.c;
    atomicAdd(p + 0, f * gv.x);
    atomicAdd(p + 1, f * gv.y);
    atomicAdd(p + 2, f * gv.z);
    atomicAdd(p + 3, f * gv.w);
  }
}

// one thread per (n, ho, wo, group, k): the offset and mask gradients of one sample
__global__ __launch_bounds__(256) void dcn_coord_grad_kernel(DcnGeom g, const float* __restrict__ x,
                                                             const float* __restrict__ gcols,
                                                             const float* __restrict__ off,
                                                             const float* __restrict__ msk,
                                                             float* __restrict__ goff, float* __restrict__ gmsk,
                                                             int64_t total) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= total) return;
  const int K = g.kh * g.kw;
  const int k = (int)(idx % K);
  int64_t r = idx / K;
  const int grp = (int)(r % g.groups);
  r /= g.groups;
  const int ox = (int)(r % g.wo);
  r /= g.wo;
  const int oy = (int)(r % g.ho);
  const int n = (int)(r / g.ho);
  const int cpg = g.c / g.groups;
  const Sample s = sample_at(g, off, msk, n, oy, ox, grp, k);
  float vh = 0.f, vw = 0.f, vm = 0.f;
  if (s.ok) {
    const Corners q = corners(s.hs, s.ws, g.h, g.w);
    const float lh = s.hs - q.hl, lw = s.ws - q.wl;
    // d w_t / d h and d w_t / d w for the four corners (dmcn_get_coordinate_weight)
    const float dwh[4] = {-(1.f - lw), -lw, 1.f - lw, lw};
    const float dww[4] = {-(1.f - lh), 1.f - lh, -lh, lh};
    const float* xb = x + (int64_t)n * g.h * g.w * g.c + grp * cpg;
    const float* gb = gcols + ((((int64_t)n * g.ho + oy) * g.wo + ox) * K + k) * g.c + grp * cpg;
    for (int c = 0; c < cpg; c += 4) {
      const float4 gv = ld4(gb + c);
      float4 bil = make_float4(0.f, 0.f, 0.f, 0.f), dh4 = bil, dw4 = bil;
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        if (!q.in[t]) continue;
        const int yy = q.hl + (t >> 1), xx = q.wl + (t & 1);
        const float4 u = ld4(xb + ((int64_t)yy * g.w + xx) * g.c + c);
        bil.x += q.wt[t] * u.x; bil.y += q.wt[t] * u.y; bil.z += q.wt[t] * u.z; bil.w += q.wt[t] * u.w;
        dh4.x += dwh[t] * u.x; dh4.y += dwh[t] * u.y; dh4.z += dwh[t] * u.z; dh4.w += dwh[t] * u.w;
        dw4.x += dww[t] * u.x; dw4.y += dww[t] * u.y; dw4.z += dww[t] * u.z; dw4.w += dww[t] * u.w;
      }
      vm += gv.x * bil.x + gv.y * bil.y + gv.z * bil.z + gv.w * bil.w;
      vh += gv.x * dh4.x + gv.y * dh4.y + gv.z * dh4.z + gv.w * dh4.w;
      vw += gv.x * dw4.x + gv.y * dw4.y + gv.z * dw4.z + gv.w * dw4.w;
    }
  }
  const int64_t plane = (int64_t)g.ho * g.wo, pix = (int64_t)oy * g.wo + ox;
  float* ob = goff + ((int64_t)n * g.groups * 2 * K + (int64_t)(grp * K + k) * 2) * plane;
  ob[pix] = vh * s.m;
  ob[plane + pix] = vw * s.m;
  if (gmsk) gmsk[((int64_t)n * g.groups * K + grp * K + k) * plane + pix] = vm;
}

int geom(const int32_t* shp, DcnGeom& g) {
  g = DcnGeom{shp[0], shp[1], shp[2], shp[3], shp[4], shp[5], shp[6], shp[7], shp[8], shp[9],
              shp[10], shp[11], shp[12], shp[13], shp[14]};
  VSRK_CHECK(g.n > 0 && g.h > 0 && g.w > 0 && g.c > 0 && g.ho > 0 && g.wo > 0 && g.kh > 0 && g.kw > 0 &&
                 g.sh > 0 && g.sw > 0 && g.dh > 0 && g.dw > 0 && g.groups > 0,
             "dcn: bad geometry");
  VSRK_CHECK(g.c % g.groups == 0 && (g.c / g.groups) % 4 == 0,
             "dcn: channels per deformable group (%d / %d) must be a multiple of 4", g.c, g.groups);
  return VSRK_OK;
}

int64_t blocks_for(int64_t total) { return (total + 255) / 256; }

}  // namespace

extern "C" int vsrk_dcn_im2col(const int32_t* geometry, const float* x, const float* offset, const float* mask,
                               float* cols, void* stream) {
  VSRK_CHECK(geometry && x && offset && cols, "dcn_im2col: null argument");
  DcnGeom g;
  if (int rc = geom(geometry, g)) return rc;
  const int64_t total = (int64_t)g.n * g.ho * g.wo * g.kh * g.kw * (g.c / 4);
  dcn_im2col_kernel<<<blocks_for(total), 256, 0, (hipStream_t)stream>>>(g, x, offset, mask, cols, total);
  VSRK_LAUNCH_CHECK("dcn_im2col");
  return VSRK_OK;
}

extern "C" int vsrk_dcn_col2im(const int32_t* geometry, const float* gcols, const float* offset, const float* mask,
                               float* grad_x, void* stream) {
  VSRK_CHECK(geometry && gcols && offset && grad_x, "dcn_col2im: null argument");
  DcnGeom g;
  if (int rc = geom(geometry, g)) return rc;
  const int64_t total = (int64_t)g.n * g.ho * g.wo * g.kh * g.kw * (g.c / 4);
  dcn_col2im_kernel<<<blocks_for(total), 256, 0, (hipStream_t)stream>>>(g, gcols, offset, mask, grad_x, total);
  VSRK_LAUNCH_CHECK("dcn_col2im");
  return VSRK_OK;
}

extern "C" int vsrk_dcn_coord_grad(const int32_t* geometry, const float* x, const float* gcols, const float* offset,
                                   const float* mask, float* grad_offset, float* grad_mask, void* stream) {
  VSRK_CHECK(geometry && x && gcols && offset && grad_offset, "dcn_coord_grad: null argument");
  DcnGeom g;
  if (int rc = geom(geometry, g)) return rc;
  const int64_t total = (int64_t)g.n * g.ho * g.wo * g.groups * g.kh * g.kw;
  dcn_coord_grad_kernel<<<blocks_for(total), 256, 0, (hipStream_t)stream>>>(g, x, gcols, offset, mask, grad_offset,
                                                                            grad_mask, total);
  VSRK_LAUNCH_CHECK("dcn_coord_grad");
  return VSRK_OK;
}
