// conv_fast family: 3x3 convs reading a sub-pixel (space-to-depth) input view:
// the data gradient of a conv + PixelShuffle (edsr_net.py:61-62) and DRF's
// strided down projection (drf_net.py:93,100).
#define VSRK_FAST_KERNEL_TU
#include "conv_fast_impl.h"

int vsrk_conv::fast_k3_n64_xs(const FastArgs& a, bool yf, bool h16, hipStream_t s) { return fast_y<3, 64, 2, 1, 0>(a, yf, h16, s); }
