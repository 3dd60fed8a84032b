// Internal (non-ABI) helpers shared between the kernel translation units.
#pragma once
#include <algorithm>
#include "vsrk_common.h"

// Per-channel sum (mode 0) or sum + sum of squares (mode 1) over every voxel of
// a view; perm_r maps view channel -> torch channel.  Needs workspace of
// vsrk_channel_reduce_ws_bytes(c) bytes.
size_t vsrk_channel_reduce_ws_bytes(int c);
int vsrk_channel_reduce_internal(const vsrk_tensor5* x, int mode, int perm_r, float scale, float* sum,
                                 float* sumsq, int accumulate, void* ws, size_t ws_bytes, hipStream_t s);

// bf16 fast path of vsrk_conv_fwd (conv_fast.hip): 1 = launched, 0 = not
// eligible (use the generic kernel), < 0 = -(error status).
int vsrk_conv_fwd_fast(const vsrk_conv_desc* d, const vsrk_tensor5* x, const void* w_packed, const float* bias,
                       const float* pro_scale, const float* pro_shift, const vsrk_tensor5* residual,
                       const vsrk_tensor5* mask, const vsrk_tensor5* y, hipStream_t s);
// thin-channel path of vsrk_conv_fwd (conv_thin.hip): cin <= 4 or cout <= 3;
// same return convention.
// one-input-channel 3x3 stencil (conv_stencil.hip): 1 = launched, 0 = not eligible, < 0 = -(error status)
int vsrk_conv_fwd_stencil(const vsrk_conv_desc* d, const vsrk_tensor5* x, const void* w_packed, const float* bias,
                          const vsrk_tensor5* residual, const vsrk_tensor5* mask, const vsrk_tensor5* y,
                          hipStream_t s);
int vsrk_conv_fwd_stencil_out(const vsrk_conv_desc* d, const vsrk_tensor5* x, const void* w_packed,
                              const float* bias, const vsrk_tensor5* residual, const vsrk_tensor5* mask,
                              const vsrk_tensor5* y, hipStream_t s);
void vsrk_conv_set_stencil_mode(int mode);
int vsrk_conv_fwd_thin(const vsrk_conv_desc* d, const vsrk_tensor5* x, const void* w_packed, const float* bias,
                       const float* pro_scale, const float* pro_shift, const vsrk_tensor5* residual,
                       const vsrk_tensor5* mask, const vsrk_tensor5* y, hipStream_t s);

// rolling-depth 16-bit Conv3d 3x3x3 (conv_roll.hip): forward / data gradient;
// same return convention; vsrk_conv_set_roll_mode: -1 env VSRK_CONV_ROLL, 0 off, 1 forced on, 2 automatic
// slope_ws != nullptr (2-D forms): mask is a PReLU output y_fwd with y's
// geometry and strides, desc->mask_slope its slope a: out = conv * (y_fwd > 0 ?
// 1 : a) and per-lane partials of sum_{y_fwd < 0} out * y_fwd into slope_ws
// (vsrk_roll_slope_ws_floats() floats); *slope_blocks = the grid.
// bnred (3-D form, no epilogue operands): the fused BN+ReLU backward reduce
// (bnx with y's geometry and strides; ws >= ntiles * 8 * 64 floats); on
// launch ntiles / ntn are filled for roll_bnred_final.
struct vsrk_roll_bnred {
  const vsrk_tensor5* bnx;
  const float *scale, *shift, *mean, *invstd;
  float* ws;
  size_t ws_floats;
  int ntiles, ntn;
};
// a fused PReLU backward's slope-gradient partials (one double per wave,
// vsrk_wave_sum) and their capacity; vsrk_slope_final sums them into *da
struct vsrk_slope_out {
  double* part;
  size_t cap;     // doubles
  int* nparts;    // out: partials written
};
void vsrk_slope_final(const double* part, int nparts, const float* a, float* da, int accumulate, int pre,
                      hipStream_t s);
int vsrk_conv_fwd_roll(const vsrk_conv_desc* d, const vsrk_tensor5* x, const void* w_packed, const float* bias,
                       const float* pro_scale, const float* pro_shift, const vsrk_tensor5* residual,
                       const vsrk_tensor5* mask, const vsrk_tensor5* y, hipStream_t s,
                       const vsrk_slope_out* slope = nullptr, vsrk_roll_bnred* bnred = nullptr);
// the fused reduce's final per-channel sums (roll_bnred_final_kernel)
int vsrk_roll_bnred_final(const vsrk_roll_bnred& r, int cout, float* sum_dy, float* sum_dy_xhat, hipStream_t s);
size_t vsrk_roll_bnred_ws_floats(const vsrk_tensor5* y);
size_t vsrk_roll_slope_ws_bytes();
void vsrk_conv_set_roll_mode(int mode);
void vsrk_conv_set_roll_wr_mode(int mode);
void vsrk_conv_set_roll_fold_mode(int mode);
// the depth-folded rolling forward (conv_roll_fold.hip): one output depth from
// three slices; 1 launched, 0 not eligible, < 0 -(error status)
int vsrk_conv_fwd_roll_fold(const vsrk_conv_desc* d, const vsrk_tensor5* x, const void* w_packed, const float* bias,
                            const float* pro_scale, const float* pro_shift, const vsrk_tensor5* y, hipStream_t s);

// pointwise (1x1x1) bf16 conv (conv_pw.hip): forward / data gradient and
// weight gradient; same return convention (the wgrad launches its own reduce)
int vsrk_conv_fwd_pw(const vsrk_conv_desc* d, const vsrk_tensor5* x, const void* w_packed, const float* bias,
                     const float* pro_scale, const float* pro_shift, const vsrk_tensor5* residual,
                     const vsrk_tensor5* mask, const vsrk_tensor5* y, hipStream_t s);
// wide pointwise convs (conv_pw_wide.hip: > 256 input channels or 256 -> >= 256)
int vsrk_conv_fwd_pw_wide(const vsrk_conv_desc* d, const vsrk_tensor5* x, const void* w_packed, const float* bias,
                          const vsrk_tensor5* residual, const vsrk_tensor5* mask, const vsrk_tensor5* y,
                          hipStream_t s);
int vsrk_conv_fwd_pw_pbwd(const vsrk_conv_desc* d, const vsrk_tensor5* x, const void* w_packed,
                          const vsrk_tensor5* mask, const vsrk_tensor5* y, int c_lo, const vsrk_slope_out* slope,
                          hipStream_t s);
size_t vsrk_pw_pbwd_ws_bytes();
size_t vsrk_conv_wgrad_pw_workspace(const vsrk_conv_desc* d, const vsrk_tensor5* x, const vsrk_tensor5* dy);
int vsrk_conv_wgrad_pw(const vsrk_conv_desc* d, const vsrk_tensor5* x, const vsrk_tensor5* dy,
                       const float* pro_scale, const float* pro_shift, float dy_scale, int32_t perm_r, float* dw,
                       float* dbias, int32_t accumulate, void* workspace, size_t workspace_bytes, hipStream_t s);

// path switches (vsrk_conv_set_path): -1 = from the environment, 0 off, 1 on
extern int vsrk_g_pw_mode;
extern int vsrk_g_thin_mode;
extern int vsrk_g_wgrad_pipe_mode;
// vsrk_conv_set_grid_cap: > 0 caps the workgroups of the persistent conv grids
// and of the weight-gradient split (tests drive the multi-tile loops with it)
extern int vsrk_g_grid_cap;
static inline int64_t vsrk_capped_grid(int64_t g) {
  return vsrk_g_grid_cap > 0 ? std::max<int64_t>(1, std::min<int64_t>(g, vsrk_g_grid_cap)) : g;
}
