/* vsrk deformable convolution (DCNv1 / DCNv2): the sampling and scatter
 * kernels of the reference's only native op (edvr_net/dcn/src/
 * deform_conv_cuda_kernel.cu:189-766, bound in deform_conv_cuda.cpp:681-695).
 * The contraction with the weights is the library's 1x1 conv (vsrk_conv_fwd /
 * vsrk_conv_wgrad in vsrk.h) over the sampled columns.
 *
 * geometry: int32[15] = {N, H, W, C, Ho, Wo, kh, kw, stride_h, stride_w,
 *   pad_h, pad_w, dil_h, dil_w, deformable_groups}; C / deformable_groups a
 *   multiple of 4.
 * x, grad_x: (N, H, W, C) fp32 channels-last.  cols, gcols: (N, Ho, Wo,
 *   kh*kw*C) fp32, column index k*C + c with k = i*kw + j.
 * offset, grad_offset: (N, G*2*kh*kw, Ho, Wo) fp32 (the reference's NCHW
 *   layout: channel (g*K + k)*2 + {0: h, 1: w}); mask, grad_mask: (N, G*kh*kw,
 *   Ho, Wo), mask NULL = DCNv1 (deform_conv), grad_mask may be NULL.
 *   vsrk_dcn_im2col:     cols = mask * bilinear(x, p + offset)
 *   vsrk_dcn_col2im:     grad_x += scatter of gcols (float atomics, as the
 *                        reference's col2im; grad_x must be zeroed first)
 *   vsrk_dcn_coord_grad: grad_offset, grad_mask (fixed-order per sample)
 * Same conventions as vsrk.h: int status, vsrk_last_error(), caller's stream. */
#ifndef VSRK_DCN_H
#define VSRK_DCN_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

int vsrk_dcn_im2col(const int32_t* geometry, const float* x, const float* offset, const float* mask, float* cols,
                    void* stream);
int vsrk_dcn_col2im(const int32_t* geometry, const float* gcols, const float* offset, const float* mask,
                    float* grad_x, void* stream);
int vsrk_dcn_coord_grad(const int32_t* geometry, const float* x, const float* gcols, const float* offset,
                        const float* mask, float* grad_offset, float* grad_mask, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* VSRK_DCN_H */
