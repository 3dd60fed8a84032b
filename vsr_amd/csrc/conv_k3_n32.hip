// conv_k3 family: 3x3(x3) convs with <= 32 output channels per tile (the DUF
// dense units' Conv3d(F, 32, 3), duf_net.py:203,214, with the fused
// BatchNorm+ReLU prologue).
#define VSRK_K3_KERNEL_TU
#include "conv_k3_impl.h"

int vsrk_conv::k3_n32(const K3Args& a, bool pro, hipStream_t s) {
  return pro ? launch_k3<32, 0, 0, 1>(a, s) : launch_k3<32, 0, 0, 0>(a, s);
}
