// Host entry of the second-generation 3x3(x3) conv (conv_k3_impl.h):
// eligibility, argument set-up and dispatch to the tile families.
#include <cstdlib>
#include "conv_k3_impl.h"

namespace {
int num_cus_k3() {
  static int n = 0;
  if (n == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
  }
  return n;
}

bool aligned16(const vsrk_tensor5* t) {
  return ((uintptr_t)t->ptr) % 16 == 0 && t->sn % 8 == 0 && t->sd % 8 == 0 && t->sh % 8 == 0 && t->sw % 8 == 0;
}
}  // namespace

int vsrk_g_k3_mode = -1;  // -1: from VSRK_CONV_K3 (default off until it beats conv_fast), 0 off, 1 on (vsrk_conv_set_path "k3")

int vsrk_conv::k3_grid(int64_t ntiles) {
  return (int)vsrk_capped_grid(std::min<int64_t>(ntiles, 2 * (int64_t)num_cus_k3()));
}

// 1 = launched, 0 = not eligible (another kernel runs), < 0 = -(status)
int vsrk_conv_fwd_k3(const vsrk_conv_desc* d, const vsrk_tensor5* x, const void* w_packed, const float* bias,
                     const float* pro_scale, const float* pro_shift, const vsrk_tensor5* residual,
                     const vsrk_tensor5* mask, const vsrk_tensor5* y, hipStream_t s) {
  using namespace vsrk_conv;
  if (vsrk_g_k3_mode < 0) {
    const char* e = getenv("VSRK_CONV_K3");
    vsrk_g_k3_mode = (e && e[0] == '1') ? 1 : 0;
  }
  if (vsrk_g_k3_mode == 0) return 0;
  if (x->dtype != VSRK_BF16 || y->dtype != VSRK_BF16) return 0;
  if (d->kh != 3 || d->kw != 3) return 0;
  const int xr = x->shuffle > 1 ? x->shuffle : 1, yr = y->shuffle > 1 ? y->shuffle : 1;
  if (x->c % 16 != 0 || (xr > 1 && (x->c / (xr * xr)) % 16 != 0)) return 0;
  if (y->c % 8 != 0 || (yr > 1 && (y->c / (yr * yr)) % 8 != 0)) return 0;
  if (!aligned16(x) || !aligned16(y)) return 0;
  if (xr > 1 && (d->prologue || yr > 1)) return 0;
  if (yr > 1 && (residual || mask || (y->c / (yr * yr)) % 64 != 0)) return 0;
  for (const vsrk_tensor5* t : {residual, mask}) {
    if (t && (!aligned16(t) || t->shuffle > 1 || t->dtype != VSRK_BF16)) return 0;
  }
  K3Args a;
  a.x = make_view(x);
  a.y = make_view(y);
  a.res = residual ? make_view(residual) : a.y;
  a.msk = mask ? make_view(mask) : a.y;
  a.w = (const bf16*)w_packed;
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
  const int NT = y->c <= 32 ? 32 : 64;
  a.ntn = ceil_div(y->c, NT);
  int rc;
  if (xr > 1 || yr > 1) {
    if (NT != 64) return 0;
    rc = k3_n64_sub(a, xr > 1, yr > 1, s);
  } else if (NT == 32) {
    rc = k3_n32(a, d->prologue != 0, s);
  } else {
    rc = k3_n64(a, d->prologue != 0, s);
  }
  if (rc == kK3NotEligible) return 0;
  return rc == VSRK_OK ? 1 : -rc;
}
