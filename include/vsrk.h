/*
 * vsrk — C ABI of the MI355X (gfx950) kernels behind the cardiac cine-MRI
 * super-resolution train/eval step.
 *
 * Drop-in boundary.  The reference (yangsenwxy/VSR) builds its generators from
 * stock torch.nn modules and reaches native code only through the DCN
 * pybind11 module (src/model/nets/edvr_net/dcn/src/deform_conv_cuda.cpp:681-695).
 * Every entry point below replaces one torch.nn op the reference calls on the
 * hot path; the replaced call site is cited next to each declaration.
 *
 * Conventions
 *  - Plain C: pointers, sizes, a hipStream_t passed as void*.  No torch types.
 *  - The caller owns every buffer (device memory), including workspaces sized
 *    by the *_workspace_size queries.  Nothing here allocates or synchronises,
 *    so every call is safe inside hipGraph capture.
 *  - Every call returns 0 (VSRK_OK) or an error code; vsrk_last_error() gives
 *    the text for the calling thread.
 *  - Activations are channels-last (N, D, H, W, C) "views" (vsrk_tensor5) with
 *    element strides; 2-D maps use D = 1.  dtype is VSRK_F32 or VSRK_BF16 and
 *    applies to activations; weights handed in by the caller are fp32 in the
 *    torch layout, accumulation is always fp32.
 */
#ifndef VSRK_H
#define VSRK_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
  VSRK_OK = 0,
  VSRK_ERR_INVALID = 1,      /* bad argument / unsupported shape */
  VSRK_ERR_UNSUPPORTED = 2,  /* valid request this build does not implement */
  VSRK_ERR_LAUNCH = 3        /* HIP launch failure */
};

/* Element types of vsrk_tensor5 views and packed weights.  Every kernel
 * family computes in fp32 accumulators; 16-bit inputs use the MFMA of their
 * type (bf16 or fp16). */
enum { VSRK_F32 = 0, VSRK_BF16 = 1, VSRK_F16 = 2 };

enum { VSRK_PRO_NONE = 0, VSRK_PRO_RELU = 1, VSRK_PRO_AFFINE = 2, VSRK_PRO_AFFINE_RELU = 3 };
enum { VSRK_ACT_NONE = 0, VSRK_ACT_RELU = 1, VSRK_ACT_PRELU = 2 };

/* Channels-last view.  Element (n,d,h,w,c) lives at
 *   ptr + n*sn + d*sd + h*sh + w*sw + c                      (shuffle <= 1)
 * With shuffle = r > 1 the view is the sub-pixel (space-to-depth) image of a
 * physical tensor P of shape (n, d, h*r, w*r, c/(r*r)) whose strides are
 * sn..sw:  logical channel c = (i*r + j) * (c/(r*r)) + c' addresses
 * P[n, d, h*r + i, w*r + j, c'].  Writing a conv output through such a view
 * is a fused nn.PixelShuffle(r) (edsr_net.py:62, drf_net.py:142); reading
 * through one is the fused inverse.  The channel order differs from torch's
 * pixel_shuffle (c'*r*r + i*r + j); vsrk_conv_pack_weight(..., perm_r) and
 * vsrk_conv_wgrad(..., perm_r) translate. */
typedef struct vsrk_tensor5 {
  void* ptr;
  int32_t n, d, h, w, c;
  int64_t sn, sd, sh, sw;
  int32_t shuffle;
  int32_t dtype;
} vsrk_tensor5;

/* Stride-1 3-D convolution (2-D when kd = 1 and D = 1), zero padding.
 * out(n,do,ho,wo,co) = act(out_scale * (bias[co] + sum_{tap,ci} in(n, do+kd-pd,
 * ho+kh-ph, wo+kw-pw, ci) * W[co,ci,tap])) [* (mask > 0)] [+ residual] [+ out].
 * The input passes through the prologue first (per-channel scale/shift and/or
 * ReLU: a fused BatchNorm3d+ReLU, duf_net.py:198-203). */
typedef struct vsrk_conv_desc {
  int32_t kd, kh, kw;
  int32_t pd, ph, pw;
  int32_t prologue;   /* VSRK_PRO_* applied to every in-bounds input element */
  int32_t act;        /* VSRK_ACT_* */
  float out_scale;    /* multiplies (acc + bias) — EDSR res_scale (edsr_net.py:51) */
  int32_t accumulate; /* 1: out += result (gradient accumulation into concat buffers) */
  int32_t bias_perm_r; /* >1: bias is in torch pixel-shuffle order (see vsrk_conv_pack_weight perm_r) */
  const float* act_param;  /* device scalar, VSRK_ACT_PRELU: nn.PReLU(num_parameters=1) slope (drf_net.py:56) */
  const float* mask_slope; /* device scalar or NULL: where mask <= 0 the output is scaled by *mask_slope
                              instead of zeroed -- the PReLU backward dx = dy * (y > 0 ? 1 : a) */
  int32_t subpixel;   /* 0, or VSRK_SUBPIXEL(k, s, p, transposed, flipped): the weight is the
                         vsrk_subpixel_conv_weight image of nn.Conv2d / nn.ConvTranspose2d(k, stride s,
                         padding p) (drf_net.py:70-102), packed with mode `flipped`, and the shuffle-s
                         operand (x or y) carries its sub-pixel phase: taps whose weights are zero for a
                         whole phase may be skipped (4 of 9 at k = 8, s = 4, p = 2).  Results are those
                         of the dense weight. */
} vsrk_conv_desc;
#define VSRK_SUBPIXEL(k, s, p, transposed, flipped) \
  ((int32_t)((k) | ((s) << 8) | ((p) << 16) | ((transposed) ? 1 << 24 : 0) | ((flipped) ? 1 << 25 : 0)))

/* Repack an fp32 torch conv weight (cout, cin, kd, kh, kw) into the kernel
 * layout [kd][kh][kw][round_up(cout',128)][round_up(cin',32)] of `dtype`.
 * mode 0: forward (cout' = cout, cin' = cin).
 * mode 1: data-gradient (cout' = cin, cin' = cout, taps flipped): the packed
 *         weight turns vsrk_conv_fwd into dL/dinput of the forward conv with
 *         padding k-1-p.
 * perm_r > 1: the torch `cout` index is read in pixel-shuffle order so that a
 *         conv written through a shuffle-r output view equals torch's
 *         conv -> PixelShuffle(r).
 * packed must hold vsrk_conv_packed_elems(...) elements. */
size_t vsrk_conv_packed_elems(int32_t cout, int32_t cin, int32_t kd, int32_t kh, int32_t kw, int32_t mode);
int vsrk_conv_pack_weight(int32_t dtype, const float* w, int32_t cout, int32_t cin, int32_t kd,
                          int32_t kh, int32_t kw, int32_t mode, int32_t perm_r, void* packed,
                          void* stream);

/* Forward conv, nn.Conv2d / nn.Conv3d forward (edsr_net.py:28-64,
 * duf_net.py:35-49,116-214, drf_net.py:55-147).  Also the data-gradient of the
 * same conv when given a mode-1 packed weight and the gradient as `x`.
 * bias, pro_scale, pro_shift may be NULL; residual, mask may be NULL. */
int vsrk_conv_fwd(const vsrk_conv_desc* desc, const vsrk_tensor5* x, const void* w_packed,
                  const float* bias, const float* pro_scale, const float* pro_shift,
                  const vsrk_tensor5* residual, const vsrk_tensor5* mask,
                  const vsrk_tensor5* y, void* stream);

/* A pointwise (1x1x1) conv with a per-channel reduction of its stored output
 * fused into the store pass (DUF's dense units, duf_net.py:198-200):
 *   mode 1 (conv1 with the BN1+ReLU prologue): out_a = sum y, out_b = sum y^2
 *          -- the statistics of the following BatchNorm3d (bn2);
 *   mode 2 (the data gradient of conv1, no prologue): with dy' = y * (bnx *
 *          scale + shift > 0) and xhat = (bnx - mean) * invstd, out_a =
 *          sum dy', out_b = sum dy' * xhat -- vsrk_bn_relu_bwd_reduce of bn1
 *          without a second pass over y.
 * Square pointwise convs (cin = cout, 64..224 channels), no activation /
 * mask / residual / accumulate; and, mode 2 only, the data gradient of a
 * Conv3d 3x3x3 on the rolling kernel (a dense unit's conv2 feeding bn2's
 * backward, duf_net.py:198-203; bnx with y's geometry and strides).
 * VSRK_ERR_UNSUPPORTED otherwise (the caller runs vsrk_conv_fwd + the separate
 * reduction).  Fixed-order partials (deterministic); workspace
 * vsrk_conv_fwd_reduce_workspace(desc, y) bytes. */
size_t vsrk_conv_fwd_reduce_workspace(const vsrk_conv_desc* desc, const vsrk_tensor5* y);
int vsrk_conv_fwd_reduce(const vsrk_conv_desc* desc, const vsrk_tensor5* x, const void* w_packed,
                         const float* bias, const float* pro_scale, const float* pro_shift,
                         const vsrk_tensor5* y, int32_t mode, const vsrk_tensor5* bnx, const float* scale,
                         const float* shift, const float* mean, const float* invstd, float* out_a,
                         float* out_b, void* workspace, size_t workspace_bytes, void* stream);

/* A conv's output followed by the backward of the PReLU whose gradient it
 * is (DRF's chains, drf_net.py:55-106: the data gradient of a projection or
 * of a 1x1 conv feeding an earlier PReLU):
 *   t = conv(x) [+ y if desc->accumulate]
 *   y[c] = c >= c_lo ? t * (y_fwd > 0 ? 1 : a) : t
 *   *da [+]= sum_{c >= c_lo, y_fwd < 0} y * y_fwd / a^2
 * with a = *desc->mask_slope and y_fwd the PReLU's forward output (y's shape
 * and strides; only channels >= c_lo are read).  c_lo > 0 serves a consumer
 * that owns the tail slice of a concat gradient (its last contribution is
 * this conv).  Forms: the rolling 2-D kernel's (3x3 pad 1 over 64-channel
 * output blocks, plain or sub-pixel views, c_lo = 0) and the staged pointwise
 * kernel's (1x1, no bias); VSRK_ERR_UNSUPPORTED otherwise (the caller runs
 * vsrk_conv_fwd + vsrk_prelu_bwd).  Fixed-order per-wave partials and a
 * fixed-order final sum (deterministic); workspace
 * vsrk_conv_prelu_bwd_workspace() bytes.  da == NULL defers the slope
 * gradient: the partials stay in the workspace (see vsrk_slope_final_sum). */
size_t vsrk_conv_prelu_bwd_workspace(void);
int vsrk_conv_fwd_prelu_bwd(const vsrk_conv_desc* desc, const vsrk_tensor5* x, const void* w_packed,
                            const float* bias, const vsrk_tensor5* y_fwd, const vsrk_tensor5* y, int32_t c_lo,
                            float* da, int32_t accumulate_da, void* workspace, size_t workspace_bytes, void* stream);

/* Tuning knob for A/B measurement: -1 (default) = bf16 fast path when
 * eligible (env VSRK_CONV_FAST=0 disables), 0 = always the generic kernel,
 * 1 = fast path when eligible.  Results agree within bf16 rounding. */
int vsrk_conv_set_algo(int32_t mode);

/* Per-path switch for A/B measurement and tests: path "fast" (bf16 LDS-DMA
 * conv, default on), "pw"
 * (bf16 1x1x1 convs with cin = cout or cout a multiple of cin, cin <= 256:
 * forward, data gradient and weight gradient in one pass over HBM, default
 * on), "thin" (cin <= 4 / cout <= 3 kernels incl. their weight gradient,
 * default on), "wgrad_pipe" (pipelined 16-bit 3x3(x3) weight gradient, default
 * on), "wgrad_roll" (rolling-depth Conv3d 3x3x3 weight gradient), "wgrad_row"
 * (rolling-row Conv2d 3x3 weight gradient over 64 x 64 channel blocks,
 * default on), "roll_fold" (the depth-folded rolling forward of a Conv3d
 * 3x3x3 with one output depth from three slices, duf_net.py:214, default on;
 * env VSRK_ROLL_FOLD); mode -1 = default/environment (VSRK_CONV_FAST, VSRK_CONV_PW,
 * VSRK_CONV_ROLL, VSRK_CONV_THIN, VSRK_WGRAD_PIPE, VSRK_WGRAD_ROLL,
 * VSRK_WGRAD_ROW), 0 = off, 1 = on where eligible.  Every path computes the
 * same result as the generic kernels within bf16 rounding. */
int vsrk_conv_set_path(const char* path, int32_t mode);

/* Test knob: cap the persistent conv grids (forward / data-gradient kernels)
 * and the weight-gradient split at max_workgroups (0 = default: one
 * workgroup per CU and the split rule).  With a small cap a small shape runs
 * many tiles per workgroup, i.e. the same cross-tile pipeline (DMA ring,
 * deferred epilogue, next-tile prefetch) as the full-size shapes.  Results
 * are identical for every cap (the weight-gradient sums are re-associated
 * over a different split, so they agree within fp32 rounding). */
int vsrk_conv_set_grid_cap(int32_t max_workgroups);

/* Test knob of the rolling-depth Conv3d 3x3x3 path (path "roll" of
 * vsrk_conv_set_path: 16-bit forward / data gradient of DUF's dense-unit convs,
 * duf_net.py:203,214): output depths per tile, 0 = automatic (as many as keep
 * >= 2 tiles per CU).  Results are identical for every setting. */
int vsrk_conv_set_roll_depth(int32_t depths);

/* Weight/bias gradient (autograd of nn.Conv*d.weight/.bias in loss.backward(),
 * base_trainer.py:128).  dw is fp32 in torch layout (cout, cin, kd, kh, kw);
 * `perm_r` as in vsrk_conv_pack_weight.  Deterministic: per-workgroup fp32
 * partial slabs reduced in a fixed order (no float atomics).  dy_scale scales
 * both gradients; accumulate != 0 adds into dw / dbias.  dbias may be NULL. */
size_t vsrk_conv_wgrad_workspace_size(const vsrk_conv_desc* desc, const vsrk_tensor5* x,
                                      const vsrk_tensor5* dy);
int vsrk_conv_wgrad(const vsrk_conv_desc* desc, const vsrk_tensor5* x, const vsrk_tensor5* dy,
                    const float* pro_scale, const float* pro_shift, float dy_scale, int32_t perm_r,
                    float* dw, float* dbias, int32_t accumulate, void* workspace,
                    size_t workspace_bytes, void* stream);

/* Strided up/down projections of DRF's feedback block (drf_net.py:70-102):
 * nn.Conv2d(cin, cout, k, stride s, padding p) and nn.ConvTranspose2d(cin,
 * cout, k, s, p) with k <= p + 2s, p <= s (DRF: (6,2,2) (7,3,2) (8,4,2)
 * (12,8,2)) are exactly 3x3 / pad-1 convolutions on the sub-pixel grid:
 *  - the strided conv reads its high-res input through a shuffle-s view
 *    (s*s*cin logical channels) and is a plain 3x3 conv cin' = s*s*cin -> cout;
 *  - the transposed conv is a 3x3 conv cin -> s*s*cout written through a
 *    shuffle-s output view.
 * vsrk_subpixel_conv_weight builds that equivalent fp32 weight (torch layout,
 * view channel order; tap/sub-pixel pairs outside the k x k kernel are zero)
 * and bias; vsrk_subpixel_wgrad_fold maps the equivalent conv's weight/bias
 * gradient back onto the k x k weight (each entry has exactly one image) and
 * sums the transposed conv's bias gradient over sub-pixels in a fixed order.
 * transposed = 0: w (cout, cin, k, k) -> weq (cout, s*s*cin, 3, 3), beq (cout)
 * transposed = 1: w (cin, cout, k, k) -> weq (s*s*cout, cin, 3, 3), beq (s*s*cout) */
int vsrk_subpixel_conv_weight(const float* w, const float* bias, int32_t cin, int32_t cout, int32_t k, int32_t s,
                              int32_t p, int32_t transposed, float* weq, float* beq, void* stream);
int vsrk_subpixel_wgrad_fold(const float* dweq, const float* dbeq, int32_t cin, int32_t cout, int32_t k, int32_t s,
                             int32_t p, int32_t transposed, float* dw, float* db, int32_t accumulate, void* stream);

/* nn.PReLU(num_parameters=1) weight gradient (drf_net.py:56-102), from the
 * layer's output y and the gradient dx at its input (as the conv epilogues
 * produce it, dx = dy * (y > 0 ? 1 : a)):  da = sum_{y < 0} dx * y / a^2
 * (= sum_{x < 0} dy * x).  Deterministic two-pass reduction; *da is written
 * (accumulate = 0) or added to.  Workspace: vsrk_prelu_workspace_size(). */
size_t vsrk_prelu_workspace_size(void);
int vsrk_prelu_wgrad(const vsrk_tensor5* y, const vsrk_tensor5* dx, const float* a, float* da, int32_t accumulate,
                     void* workspace, size_t workspace_bytes, void* stream);

/* nn.PReLU backward in one pass: dx = (dy [+ dy2]) * (y > 0 ? 1 : a) for the
 * layer output y (dy2 may be NULL: a second gradient contribution, e.g. a
 * skip connection), and da [+]= sum_{y<0} dx * y / a^2.  dx may alias dy.
 * Workspace: vsrk_prelu_workspace_size(). */
int vsrk_prelu_bwd(const vsrk_tensor5* y, const vsrk_tensor5* dy, const vsrk_tensor5* dy2, const float* a,
                   const vsrk_tensor5* dx, float* da, int32_t accumulate_da, void* workspace, size_t workspace_bytes,
                   void* stream);

/* nn.PReLU backward from the layer INPUT x (the pre-activation, what
 * nn.PReLU itself saves; replaces drf_net.py:55-58,66,83-100's PReLU
 * autograd for ANY slope, a <= 0 included): dx = (dy [+ dy2]) * (x > 0 ? 1 :
 * a) and da [+]= sum_{x<0} (dy [+ dy2]) * x.  vsrk_prelu_bwd's output-based
 * form reads x < 0 as y < 0, exact only while a > 0 (it returns a NaN slope
 * gradient for a <= 0).  Same views, workspace and determinism. */
int vsrk_prelu_bwd_pre(const vsrk_tensor5* x, const vsrk_tensor5* dy, const vsrk_tensor5* dy2, const float* a,
                       const vsrk_tensor5* dx, float* da, int32_t accumulate_da, void* workspace,
                       size_t workspace_bytes, void* stream);

/* Deferred PReLU slope gradients (DRF: 12 PReLUs x 30 frames of backward
 * calls, one final sum each would be 360+ serial launches per step).  Each of
 * vsrk_conv_fwd_prelu_bwd / vsrk_prelu_bwd / _pre called with da == NULL
 * leaves its partials at the start of its workspace; given each call its own
 * slot of vsrk_slope_slot_doubles() doubles in one zero-filled region per
 * PReLU, vsrk_slope_final_sum over that region (nparts = slots x slot size)
 * is the slope gradient of all the calls, summed in slot order (fixed:
 * deterministic).  pre selects the partials' form (0: output-based, divided
 * by a^2; 1: pre-activation); one PReLU's calls must all use the same. */
size_t vsrk_slope_slot_doubles(void);
int vsrk_slope_final_sum(const double* part, int64_t nparts, const float* a, float* da, int32_t accumulate,
                         int32_t pre, void* stream);

/* Layout/dtype moves between torch's NC(D)HW fp32 tensors and channels-last
 * views: src is (n, c, d, h, w) fp32 contiguous; channels beyond c in dst are
 * zero-filled (input padding for the 1-channel head convs). */
int vsrk_ncdhw_to_view(const float* src, int32_t n, int32_t c, int32_t d, int32_t h, int32_t w,
                       const vsrk_tensor5* dst, void* stream);
int vsrk_view_to_ncdhw(const vsrk_tensor5* src, float* dst, int32_t c, void* stream);

/* Elementwise ReLU backward: dx = dy * (y > 0) (nn.ReLU, edsr_net.py:46). */
int vsrk_relu_bwd(const vsrk_tensor5* y, const vsrk_tensor5* dy, const vsrk_tensor5* dx, void* stream);

/* Sum of two views into a third (gradient merge at skip connections). */
int vsrk_add(const vsrk_tensor5* a, const vsrk_tensor5* b, const vsrk_tensor5* out, void* stream);

/* Losses (fp32, mean reduction): kind 0 = L1Loss, 1 = MSELoss, 2 = HuberLoss
 * (losses.py:5-20, param = delta), 3 = CharbonnierLoss (losses.py:23-34,
 * param = epsilon).  out/target are `count` contiguous fp32.  loss_fwd writes
 * the scalar to *loss (device).  loss_bwd writes dL/dout * (*gscale) with
 * gscale a device scalar (the upstream gradient) to `grad` in dtype. */
size_t vsrk_loss_workspace_size(int64_t count);
int vsrk_loss_fwd(int32_t kind, float param, const float* out, const float* target, int64_t count,
                  float* loss, void* workspace, size_t workspace_bytes, void* stream);
int vsrk_loss_bwd(int32_t kind, float param, const float* out, const float* target, int64_t count,
                  const float* gscale, void* grad, int32_t grad_dtype, void* stream);

/* [Denormalize +] PSNR (utils.py:1-20 then metrics.py:20-36): for each of the
 * `batch` samples of `per_sample` fp32 values, when denormalize != 0
 * x -> clamp(round(x*std+mean),0,255) (round half to even, as torch.round);
 * mse over the sample, psnr = 10*log10(max^2/(mse+1e-10)).  Writes per-sample
 * PSNR to psnr_per_sample[batch] and their mean to *psnr_mean (device). */
size_t vsrk_psnr_workspace_size(int32_t batch, int64_t per_sample);
int vsrk_psnr(const float* out, const float* target, int32_t batch, int64_t per_sample, int32_t denormalize,
              float mean, float std, float max_value, float* psnr_per_sample, float* psnr_mean, void* workspace,
              size_t workspace_bytes, void* stream);

/* [Denormalize +] SSIM (utils.py:1-20 then metrics.py:39-113, dim = 2): out and
 * target are (batch, channels, h, w) fp32 contiguous, h, w >= 11.  Per image
 * the five depthwise 11x11 Gaussian moments (valid convolution), the SSIM map
 * (c1 = (0.01 range)^2, c2 = (0.03 range)^2) and its mean: writes the
 * per-sample means (SSIM(size_average=False)) and their mean (size_average
 * = True).  Workspace: vsrk_ssim_workspace_size(). */
size_t vsrk_ssim_workspace_size(int32_t batch, int32_t channels, int32_t h, int32_t w);
int vsrk_ssim(const float* out, const float* target, int32_t batch, int32_t channels, int32_t h, int32_t w,
              int32_t denormalize, float mean, float std, float value_range, float* ssim_per_sample, float* ssim_mean,
              void* workspace, size_t workspace_bytes, void* stream);

/* SSIM(dim=3) of (N, C, D, H, W) fp32 volumes: the same Gaussian window
 * (metrics.py:66-79) as an 11x11x11 product, valid filtering; depth pass to
 * five moment volumes, then the separable in-plane pass.  Replaces
 * SSIM(dim=3).forward (metrics.py:86-113). */
size_t vsrk_ssim3d_workspace_size(int32_t batch, int32_t channels, int32_t d, int32_t h, int32_t w);
int vsrk_ssim3d(const float* out, const float* target, int32_t batch, int32_t channels, int32_t d, int32_t h,
                int32_t w, int32_t denormalize, float mean, float std, float value_range, float* ssim_per_sample,
                float* ssim_mean, void* workspace, size_t workspace_bytes, void* stream);

/* BatchNorm3d, training statistics (duf_net.py:116,198,201,209,212).  Split
 * so a data-parallel caller can all-reduce the per-channel sums between the
 * calls (SyncBatchNorm):
 *   vsrk_bn_stats:    sum, sumsq over every voxel of x (channels-last view)
 *   vsrk_bn_stats_grouped: the same per group of rows: x's (n, d, h) rows,
 *                     n outermost, split into `groups` equal runs; sum and
 *                     sumsq are [groups][C].  With x a depth-major view
 *                     (n := depth) this is the per-depth statistics of a
 *                     concat-buffer slice, which DUF's dense layer reuses
 *                     for every later BatchNorm over the same channels
 *                     (duf_net.py:122-128: concat channels never change)
 *   vsrk_bn_finalize: mean, biased var -> scale = gamma*invstd,
 *                     shift = beta - mean*scale (the fused conv prologue's
 *                     VSRK_PRO_AFFINE_RELU operands), running stats updated
 *                     with momentum and the unbiased variance (torch semantics)
 *   vsrk_bn_fold_running: eval mode (running statistics); mean / invstd
 *                     (may be NULL) receive running_mean, 1/sqrt(running_var + eps)
 *                     for the eval-mode backward (call the backward pair with
 *                     count = INFINITY: no batch-statistics terms)
 *   vsrk_bn_apply:    y = x * scale + shift [relu] (a materialised BatchNorm3d
 *                     output, for op-level use; the generators fold it into
 *                     the next conv instead)
 * Backward of BN followed by ReLU, given dz = dL/d relu(bn(x)) (a BN without
 * ReLU: pass scale = 0, shift = 1 -- the ReLU mask is x * scale + shift > 0):
 *   vsrk_bn_relu_bwd_reduce: sum_dy, sum_dy_xhat (= dbeta, dgamma)
 *   vsrk_bn_relu_bwd_apply:  dx [+]= gamma*invstd*(dy - sum_dy/M - xhat*sum_dy_xhat/M)
 * Workspace: vsrk_bn_workspace_size(channels) bytes. */
size_t vsrk_bn_workspace_size(int32_t channels);
int vsrk_bn_stats(const vsrk_tensor5* x, float* sum, float* sumsq, void* workspace, size_t workspace_bytes,
                  void* stream);
int vsrk_bn_stats_grouped(const vsrk_tensor5* x, int32_t groups, float* sum, float* sumsq, void* workspace,
                          size_t workspace_bytes, void* stream);
int vsrk_bn_finalize(const float* sum, const float* sumsq, double count, const float* gamma, const float* beta,
                     float eps, float momentum, float* running_mean, float* running_var, float* scale,
                     float* shift, float* mean, float* invstd, int32_t channels, void* stream);
/* vsrk_bn_finalize with the voxel count read on the device: count =
 * count_mult * *count_dev (one double).  SyncBatchNorm: count_dev is the
 * all-reduced N*H*W of the global batch, so no rank reads it on the host
 * (torch's SyncBatchNorm all-gathers the counts the same way; reference
 * BatchNorm3d, duf_net.py:116,198,201,209,212). */
int vsrk_bn_finalize_dcount(const float* sum, const float* sumsq, const double* count_dev, double count_mult,
                            const float* gamma, const float* beta, float eps, float momentum, float* running_mean,
                            float* running_var, float* scale, float* shift, float* mean, float* invstd,
                            int32_t channels, void* stream);
int vsrk_bn_fold_running(const float* gamma, const float* beta, const float* running_mean,
                         const float* running_var, float eps, float* scale, float* shift, float* mean,
                         float* invstd, int32_t channels, void* stream);
int vsrk_bn_apply(const vsrk_tensor5* x, const float* scale, const float* shift, int32_t relu, const vsrk_tensor5* y,
                  void* stream);
int vsrk_bn_relu_bwd_reduce(const vsrk_tensor5* x, const vsrk_tensor5* dz, const float* scale, const float* shift,
                            const float* mean, const float* invstd, float* sum_dy, float* sum_dy_xhat,
                            void* workspace, size_t workspace_bytes, void* stream);
int vsrk_bn_relu_bwd_apply(const vsrk_tensor5* x, const vsrk_tensor5* dz, const float* scale, const float* shift,
                           const float* mean, const float* invstd, const float* gamma, const float* sum_dy,
                           const float* sum_dy_xhat, double count, const vsrk_tensor5* dx, int32_t accumulate,
                           void* stream);
/* Every conv weight of a step repacked in ONE launch (the per-conv
 * vsrk_conv_pack_weight launches were ~4 us each, 73 per EDSR step).
 * descs: n records in DEVICE memory (built once by the caller and reused
 * every step: the weights are updated in place by the optimizer); record i
 * packs fp32 w (cout, cin, kd, kh, kw) into packed as vsrk_conv_pack_weight
 * would (mode, perm_r); max_elems = the largest vsrk_conv_packed_elems. */
typedef struct vsrk_pack_desc {
  const float* w;
  void* packed;
  int32_t cout, cin, kd, kh, kw, mode, perm_r;
  int32_t reserved;
} vsrk_pack_desc;
int vsrk_conv_pack_weights(int32_t dtype, int32_t n, const vsrk_pack_desc* descs, int64_t max_elems, void* stream);

/* Several BN+ReLU backward applies into ONE output block in one pass (DUF's
 * dense layer: every later unit's bn1 adds its input gradient to the same
 * concat channels, duf_net.py:122-128).  x, dx: the block (N, D, H, W, C);
 * contributor i: dz over depths [d0, d0 + dz.d) of the block and its BN's
 * per-channel operands (pointers at the block's first channel), as in
 * vsrk_bn_relu_bwd_apply.  dx [+]= sum_i apply_i: x and dx move once instead
 * of once per contributor.  1 <= n <= VSRK_BN_MULTI_MAX; more than 3
 * contributors need a block of at most 256 channels. */
#define VSRK_BN_MULTI_MAX 8
typedef struct vsrk_bn_contrib {
  vsrk_tensor5 dz;
  int32_t d0;
  const float *scale, *shift, *mean, *invstd, *gamma, *sum_dy, *sum_dy_xhat;
  double count;
} vsrk_bn_contrib;
int vsrk_bn_relu_bwd_apply_multi(const vsrk_tensor5* x, const vsrk_tensor5* dx, int32_t accumulate, int32_t n,
                                 const vsrk_bn_contrib* contribs, void* stream);

/* vsrk_conv_fwd_reduce mode 2 (a square 1x1x1 data gradient with the next
 * BatchNorm+ReLU backward's sums in its store pass) whose input is itself a
 * BN+ReLU backward apply, computed in the operand load: DUF's dense unit,
 * bn2's apply feeding conv1's data gradient (duf_net.py:198-201).
 *   x_out = vsrk_bn_relu_bwd_apply(bn_x, pre->dz, pre's BN)   (bitwise)
 *   y     = conv(x_out), (out_a, out_b) = bnx's BN+ReLU backward sums of y
 * pre->scale is not read: the mask uses gamma * invstd, which is
 * vsrk_bn_finalize's scale; pre->d0 is ignored.  bn_x, pre->dz and x_out
 * share one geometry (N, D, H, W, C with C % 32 == 0, 64..224); y may alias
 * pre->dz (each tile's rows are read before they are written).
 * VSRK_ERR_UNSUPPORTED when not eligible (nothing launched). */
int vsrk_conv_fwd_reduce_bnb(const vsrk_conv_desc* desc, const vsrk_tensor5* bn_x, const vsrk_bn_contrib* pre,
                             const vsrk_tensor5* x_out, const void* w_packed, const vsrk_tensor5* y,
                             const vsrk_tensor5* bnx, const float* scale, const float* shift, const float* mean,
                             const float* invstd, float* out_a, float* out_b, void* workspace,
                             size_t workspace_bytes, void* stream);

/* DUF dynamic upsampling (duf_net.py:67-97), fused: softmax over the k*k taps
 * of per-pixel logits (n, h, w, k*k*r*r) fp32 (tap-major, as the reference's
 * reshape), unfold of the centre frame x (n, h, w) fp32 with zero padding,
 * contraction, pixel shuffle and residual (n, h, w, r*r) add ->
 * out (n, r*h, r*w) fp32.  Backward writes d logits and d residual in
 * grad_dtype (x gets no gradient: it is input data). */
int vsrk_duf_dynfilter_fwd(const float* x, const float* logits, const float* residual, int32_t n, int32_t h,
                           int32_t w, int32_t size_filter, int32_t upscale, float* out, void* stream);
int vsrk_duf_dynfilter_bwd(const float* x, const float* logits, const float* grad_out, int32_t n, int32_t h,
                           int32_t w, int32_t size_filter, int32_t upscale, void* grad_logits, void* grad_residual,
                           int32_t grad_dtype, void* stream);

const char* vsrk_last_error(void);
const char* vsrk_version(void);

/* LR synthesis (acdc_preprocess.py:102-180, Downscale): cv2.resize with
 * INTER_CUBIC of n fp64 images (ih, iw) -> (oh, ow) (source coordinate
 * (d + 0.5) * ih / oh - 0.5, Keys cubic A = -0.75, border indices clamped),
 * then, with round_clip, np.clip(round(.), 0, 255). */
int vsrk_resize_bicubic(const double* src, int32_t n, int32_t ih, int32_t iw, int32_t oh, int32_t ow, double* dst,
                        int32_t round_clip, void* stream);

/* Measured device peaks (the roofline fractions are quoted
 * against the vendor peak; these give the measured ceiling beside it).
 *   vsrk_peak_mfma: vsrk_peak_mfma_blocks() workgroups of 4 waves, each wave
 *     iters x 4 v_mfma_f32_32x32x16_bf16 (32768 FLOP each) on register
 *     operands; out: blocks * 256 floats (keeps the loop live).
 *   vsrk_peak_copy: dst = src, 16-byte vectors, `bytes` a multiple of 16. */
int32_t vsrk_peak_mfma_blocks(void);
int vsrk_peak_mfma(int32_t iters, float* out, void* stream);
int vsrk_peak_copy(const void* src, void* dst, int64_t bytes, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* VSRK_H */
