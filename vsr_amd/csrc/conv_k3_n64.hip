// conv_k3 family: 3x3(x3) convs, 64 output channels per tile, plain views:
// the EDSR body (edsr_net.py:41-53), DUF's tail (duf_net.py:118) and the data
// gradients of the DUF units (duf_net.py:203,214).
#define VSRK_K3_KERNEL_TU
#include "conv_k3_impl.h"

int vsrk_conv::k3_n64(const K3Args& a, bool pro, hipStream_t s) {
  return pro ? launch_k3<64, 0, 0, 1>(a, s) : launch_k3<64, 0, 0, 0>(a, s);
}
