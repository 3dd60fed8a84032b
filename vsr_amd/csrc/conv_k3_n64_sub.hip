// conv_k3 family: 3x3 convs through sub-pixel views -- a conv + nn.PixelShuffle
// store (edsr_net.py:61-62, drf_net.py:141-142) and the data gradient that
// reads the shuffled gradient back (x_shuffle).
#define VSRK_K3_KERNEL_TU
#include "conv_k3_impl.h"

int vsrk_conv::k3_n64_sub(const K3Args& a, int xs, int ys, hipStream_t s) {
  if (xs && !ys) return launch_k3<64, 1, 0, 0>(a, s);
  if (!xs && ys) return launch_k3<64, 0, 1, 0>(a, s);
  return kK3NotEligible;
}
