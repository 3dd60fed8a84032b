// conv_fast family: 1x1(x1) pointwise convs (duf_net.py:40-49,200,211;
// drf_net.py:57,65,91,98,105), NT = 32 / 64 / 128 output channels per tile.
#define VSRK_FAST_KERNEL_TU
#include "conv_fast_impl.h"

int vsrk_conv::fast_k1(const FastArgs& a, int nt, bool yf, bool h16, hipStream_t s) {
  if (nt == 32) return fast_y<1, 32, 2, 0, 0>(a, yf, h16, s);
  if (nt == 64) return fast_y<1, 64, 2, 0, 0>(a, yf, h16, s);
  return fast_y<1, 128, 1, 0, 0>(a, yf, h16, s);
}
