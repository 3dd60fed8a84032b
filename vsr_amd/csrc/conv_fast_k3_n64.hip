// conv_fast family: 3x3(x3) convs, 64 output channels per tile, plain views
// (EDSR body, edsr_net.py:41-53; DUF tail, duf_net.py:118).
#define VSRK_FAST_KERNEL_TU
#include "conv_fast_impl.h"

int vsrk_conv::fast_k3_n64(const FastArgs& a, bool yf, bool h16, hipStream_t s) { return fast_y<3, 64, 2, 0, 0>(a, yf, h16, s); }
