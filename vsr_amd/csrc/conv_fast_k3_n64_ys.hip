// conv_fast family: 3x3 convs storing through a sub-pixel output view: a fused
// conv + nn.PixelShuffle (edsr_net.py:61-62, drf_net.py:141-142) and DRF's
// transposed up projection (drf_net.py:81,86).
#define VSRK_FAST_KERNEL_TU
#include "conv_fast_impl.h"

int vsrk_conv::fast_k3_n64_ys(const FastArgs& a, bool yf, bool h16, hipStream_t s) { return fast_y<3, 64, 2, 0, 1>(a, yf, h16, s); }
