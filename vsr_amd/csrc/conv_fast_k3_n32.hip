// conv_fast family: 3x3(x3) convs with <= 32 output channels per tile (the DUF
// dense units' Conv3d(F, 32, 3), duf_net.py:203,214).
#define VSRK_FAST_KERNEL_TU
#include "conv_fast_impl.h"

int vsrk_conv::fast_k3_n32(const FastArgs& a, bool yf, bool h16, hipStream_t s) { return fast_y<3, 32, 2, 0, 0>(a, yf, h16, s); }
