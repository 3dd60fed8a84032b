"""TEST INFRASTRUCTURE ONLY (the checker, never the product path): a plain
torch (CPU, fp64-capable, autograd) restatement of the reference's modulated
deformable convolution, deform_conv_cuda_kernel.cu, for the GPU tests of
vsr_amd.dcn.

Followed line by line:
  * sampling position h = ho*stride - pad + i*dil + offset[(g*K+k)*2], w with
    offset[(g*K+k)*2+1]; sampled iff -1 < h < H and -1 < w < W
    (modulated_deformable_im2col_gpu_kernel, .cu:570-633);
  * bilinear interpolation with the out-of-image corners read as zero
    (dmcn_im2col_bilinear, .cu:467-498), value times the mask;
  * output = weight (Cout, C*K) x columns + bias (the addmm of
    deform_conv_cuda.cpp, modulated_deform_conv_cuda_forward).
Gradients come from torch autograd through this formulation: floor() is a
constant, so d/dh of the interpolation is the piecewise-linear derivative
the reference writes out in dmcn_get_coordinate_weight (.cu:524-567), and
the input gradient is its bilinear scatter (modulated_deformable_col2im).

The reference's CUDA extension cannot be built here (nvcc / CUDA absent,
SURVEY §8c), so this restatement is pinned to the reference's source only:
parity unpinned by reference outputs.
"""
from __future__ import annotations

import torch


def modulated_deform_conv_ref(x, offset, mask, weight, bias=None, stride=1, padding=0, dilation=1,
                              deformable_groups=1):
    if isinstance(stride, int):
        stride = (stride, stride)
    if isinstance(padding, int):
        padding = (padding, padding)
    if isinstance(dilation, int):
        dilation = (dilation, dilation)
    n, c, h, w = x.shape
    co, _, kh, kw = weight.shape
    K, dg = kh * kw, deformable_groups
    cpg = c // dg
    ho = (h + 2 * padding[0] - (dilation[0] * (kh - 1) + 1)) // stride[0] + 1
    wo = (w + 2 * padding[1] - (dilation[1] * (kw - 1) + 1)) // stride[1] + 1
    dt = x.dtype
    off = offset.view(n, dg, K, 2, ho, wo)
    ki = torch.arange(K) // kw
    kj = torch.arange(K) % kw
    base_h = (torch.arange(ho) * stride[0] - padding[0]).view(1, 1, 1, ho, 1).to(dt) + \
        (ki * dilation[0]).view(1, 1, K, 1, 1).to(dt)
    base_w = (torch.arange(wo) * stride[1] - padding[1]).view(1, 1, 1, 1, wo).to(dt) + \
        (kj * dilation[1]).view(1, 1, K, 1, 1).to(dt)
    hs = base_h + off[:, :, :, 0]  # (n, dg, K, ho, wo)
    ws = base_w + off[:, :, :, 1]
    valid = ((hs > -1) & (ws > -1) & (hs < h) & (ws < w)).to(dt)
    hl, wl = torch.floor(hs), torch.floor(ws)
    lh, lw = hs - hl, ws - wl
    hl, wl = hl.long(), wl.long()
    xg = x.reshape(n, dg, cpg, h * w)
    val = torch.zeros((n, dg, cpg, K, ho, wo), dtype=dt)
    for dy, dx, wt in ((0, 0, (1 - lh) * (1 - lw)), (0, 1, (1 - lh) * lw), (1, 0, lh * (1 - lw)), (1, 1, lh * lw)):
        yy, xx = hl + dy, wl + dx
        inb = ((yy >= 0) & (yy <= h - 1) & (xx >= 0) & (xx <= w - 1)).to(dt)
        idx = (yy.clamp(0, h - 1) * w + xx.clamp(0, w - 1)).view(n, dg, 1, K * ho * wo).expand(n, dg, cpg, K * ho * wo)
        v = torch.gather(xg, 3, idx).view(n, dg, cpg, K, ho, wo)
        val = val + (wt * inb).unsqueeze(2) * v
    val = val * valid.unsqueeze(2)
    if mask is not None:
        val = val * mask.view(n, dg, K, ho, wo).unsqueeze(2)
    cols = val.reshape(n, c * K, ho * wo)  # channel-major (c*K + k), as weight.view(co, c*K)
    out = torch.einsum("ok,nkp->nop", weight.reshape(co, c * K), cols).view(n, co, ho, wo)
    if bias is not None:
        out = out + bias.view(1, co, 1, 1)
    return out
