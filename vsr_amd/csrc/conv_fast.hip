// Host entry of the bf16 fast path of the implicit-GEMM convolution (forward
// and data-gradient): eligibility, argument set-up and dispatch to the tile
// families instantiated in conv_fast_*.hip.  The kernel and its design notes
// are in conv_fast_impl.h.
#include <cstdlib>
#include <string>
#include "conv_fast_impl.h"

namespace {
using namespace vsrk_conv;

int g_fast_mode = -1;  // -1: from VSRK_CONV_FAST (default on), 0 off, 1 on

int num_cus_fast() {
  static int n = 0;
  if (n == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
  }
  return n;
}

}  // namespace

int vsrk_g_grid_cap = 0;  // vsrk_conv_set_grid_cap: 0 = one workgroup per CU

int vsrk_conv::fast_grid(int64_t ntiles) {
  int64_t g = std::min<int64_t>(ntiles, (int64_t)num_cus_fast());
  if (vsrk_g_grid_cap > 0) g = std::min<int64_t>(g, vsrk_g_grid_cap);
  return (int)std::max<int64_t>(g, 1);
}

extern "C" int vsrk_conv_set_algo(int32_t mode) {
  VSRK_CHECK(mode >= -1 && mode <= 1, "conv_set_algo: mode must be -1, 0 or 1");
  g_fast_mode = mode;
  return VSRK_OK;
}

extern int g_pw_wide_mode;  // conv_pw_wide.hip

extern "C" int vsrk_conv_set_path(const char* path, int32_t mode) {
  VSRK_CHECK(path, "conv_set_path: null path");
  const std::string p(path);
  VSRK_CHECK(mode >= -1 && mode <= (p == "wgrad_row" || p == "roll_wr" ? 2 : 1),
             "conv_set_path: mode must be -1, 0 or 1 (wgrad_row, roll_wr: 2)");
  if (p == "fast") g_fast_mode = mode;
  else if (p == "thin") vsrk_g_thin_mode = mode;
  else if (p == "wgrad_pipe") vsrk_g_wgrad_pipe_mode = mode;
  else if (p == "pw") vsrk_g_pw_mode = mode;
  else if (p == "roll") vsrk_conv_set_roll_mode(mode);
  else if (p == "wgrad_roll") vsrk_conv_set_wgrad_roll_mode(mode);
  else if (p == "wgrad_row") vsrk_conv_set_wgrad_row_mode(mode);
  else if (p == "roll_wr") vsrk_conv_set_roll_wr_mode(mode);
  else if (p == "roll_fold") vsrk_conv_set_roll_fold_mode(mode);
  else if (p == "stencil") vsrk_conv_set_stencil_mode(mode);
  else if (p == "pw_wide") g_pw_wide_mode = mode;
  else VSRK_CHECK(false, "conv_set_path: unknown path '%s' (fast, pw, roll, roll_wr, roll_fold, thin, wgrad_pipe, wgrad_roll, wgrad_row, stencil)",
                  path);
  return VSRK_OK;
}

extern "C" int vsrk_conv_set_grid_cap(int32_t max_workgroups) {
  VSRK_CHECK(max_workgroups >= 0, "conv_set_grid_cap: max_workgroups must be >= 0");
  vsrk_g_grid_cap = max_workgroups;
  return VSRK_OK;
}

// Returns 1 and launches when the fast path covers the request, 0 when the
// caller should use the generic kernel, <0 (negated status) on error.
int vsrk_conv_fwd_fast(const vsrk_conv_desc* d, const vsrk_tensor5* x, const void* w_packed, const float* bias,
                       const float* pro_scale, const float* pro_shift, const vsrk_tensor5* residual,
                       const vsrk_tensor5* mask, const vsrk_tensor5* y, hipStream_t s) {
  if (g_fast_mode < 0) {
    const char* e = getenv("VSRK_CONV_FAST");
    g_fast_mode = (e && e[0] == '0') ? 0 : 1;
  }
  if (g_fast_mode == 0) return 0;
  if (!vsrk_is16(x->dtype)) return 0;
  if (const int rl = vsrk_conv_fwd_roll(d, x, w_packed, bias, pro_scale, pro_shift, residual, mask, y, s)) return rl;
  if (!chunk_ok(x, 2) || x->c % 8 != 0) return 0;
  const int xr = x->shuffle > 1 ? x->shuffle : 1, yr = y->shuffle > 1 ? y->shuffle : 1;
  if (xr > 1 && (x->c / (xr * xr)) % 32 != 0) return 0;
  if (yr > 1 && ((y->c / (yr * yr)) % 32 != 0 || residual || mask)) return 0;
  if (xr > 1 && d->prologue) return 0;
  if (d->kh != d->kw || (d->kh != 1 && d->kh != 3)) return 0;
  // every 4-channel output group stored with one 8/16-byte access
  const int ye = vsrk_esize(y->dtype);
  if (((uintptr_t)y->ptr) % (4 * ye) != 0 || y->sn % 4 || y->sd % 4 || y->sh % 4 || y->sw % 4) return 0;
  if (y->c % 4 != 0 && !(y->c < 4 && !residual && !mask && !d->accumulate)) return 0;
  for (const vsrk_tensor5* t : {residual, mask}) {
    if (t && (((uintptr_t)t->ptr) % (4 * ye) != 0 || t->sn % 4 || t->sd % 4 || t->sh % 4 || t->sw % 4 ||
              t->shuffle > 1 || t->dtype != y->dtype))
      return 0;
  }
  FastArgs a;
  static int ablate = -1;
  if (ablate < 0) {
    const char* e = getenv("VSRK_FAST_ABLATE");
    ablate = e ? atoi(e) : 0;
  }
  a.ablate = ablate;
  a.x = make_view(x);
  a.y = make_view(y);
  a.res = residual ? make_view(residual) : a.y;
  a.msk = mask ? make_view(mask) : a.y;
  a.w = w_packed;
  a.bias = bias;
  a.pro_scale = pro_scale;
  a.pro_shift = pro_shift;
  a.cin = x->c;
  a.cout = y->c;
  a.cin_pad = round_up(x->c, 32);
  a.cout_pad = round_up(y->c, 128);
  a.kd = d->kd; a.pd = d->pd; a.ph = d->ph; a.pw = d->pw;
  a.prologue = d->prologue;
  a.act = d->act;
  a.accumulate = d->accumulate;
  a.has_res = residual != nullptr;
  a.has_mask = mask != nullptr;
  a.bias_r = d->bias_perm_r;
  a.out_scale = d->out_scale;
  a.act_param = d->act_param;
  a.mask_slope = d->mask_slope;
  a.tiles_w = ceil_div(y->w, TW);
  const int NT = y->c <= 32 ? 32 : (y->c <= 64 || d->kh == 3) ? 64 : 128;
  a.ntn = ceil_div(y->c, NT);
  const bool yf = y->dtype == VSRK_F32;
  const bool h16 = x->dtype == VSRK_F16;
  const bool ys = yr > 1, xs = xr > 1;
  int rc;
  if (d->kh == 1) {
    if (xs || ys) return 0;  // not instantiated (never requested)
    rc = fast_k1(a, NT, yf, h16, s);
  } else if (NT == 32) {
    if (xs || ys) return 0;
    rc = fast_k3_n32(a, yf, h16, s);
  } else if (!xs && !ys) {
    rc = fast_k3_n64(a, yf, h16, s);
  } else if (xs && !ys) {
    rc = fast_k3_n64_xs(a, yf, h16, s);
  } else if (!xs && ys) {
    rc = fast_k3_n64_ys(a, yf, h16, s);
  } else {
    return 0;
  }
  if (rc == kFastNotEligible) return 0;
  return rc == VSRK_OK ? 1 : -rc;
}
