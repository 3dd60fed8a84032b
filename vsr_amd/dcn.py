"""Deformable convolution v1 / v2 on HIP: the reference's EDVR alignment op
(src/model/nets/edvr_net/dcn/deform_conv.py:15-330 over
deform_conv_cuda_kernel.cu:189-766), with the same functions, modules,
constructor arguments, parameter names and NCHW fp32 tensors:

  deform_conv(x, offset, weight, stride, padding, dilation, groups, deformable_groups)
  modulated_deform_conv(x, offset, mask, weight, bias, stride, padding, dilation, groups, deformable_groups)
  DeformConv, DeformConvPack, ModulatedDeformConv, ModulatedDeformConvPack

How it runs: the sampling is vsrk_dcn_im2col (include/vsrk_dcn.h) into
channels-last columns (N, Ho, Wo, kh*kw*C); the contraction with the weights
is the library's MFMA 1x1 conv over those columns (bias fused in its
epilogue), its data gradient gives the column gradient and its weight
gradient the weight / bias gradients; vsrk_dcn_col2im and
vsrk_dcn_coord_grad return the input, offset and mask gradients.  Conv
groups other than 1 are not supported (EDVR uses 1).
"""
from __future__ import annotations

import ctypes as C
import logging
import math

import torch
import torch.nn as nn
from torch.nn.modules.utils import _pair

from . import _native as N
from . import functional as F
from .modules import HipConv2d

logger = logging.getLogger(__name__)
K1, P0 = (1, 1, 1), (0, 0, 0)


def _geometry(x, weight, stride, padding, dilation, dg):
    n, c, h, w = x.shape
    kh, kw = weight.shape[2:]
    sh, sw = stride
    ph, pw = padding
    dh, dw = dilation
    ho = (h + 2 * ph - (dh * (kh - 1) + 1)) // sh + 1
    wo = (w + 2 * pw - (dw * (kw - 1) + 1)) // sw + 1
    return (C.c_int32 * 15)(n, h, w, c, ho, wo, kh, kw, sh, sw, ph, pw, dh, dw, dg), ho, wo


class _DcnFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, offset, mask, weight, bias, stride, padding, dilation, groups, dg):
        if groups != 1:
            raise NotImplementedError("vsr_amd DCN: conv groups other than 1")
        if not x.is_cuda:
            raise NotImplementedError  # deform_conv.py:106-107: CUDA only, here HIP only
        x, offset = x.float().contiguous(), offset.float().contiguous()
        mask = mask.float().contiguous() if mask is not None else None
        lib = N.load()
        geo, ho, wo = _geometry(x, weight, stride, padding, dilation, dg)
        n, c = x.shape[:2]
        co, _, kh, kw = weight.shape
        K = kh * kw
        if offset.shape != (n, dg * 2 * K, ho, wo) or (mask is not None and mask.shape != (n, dg * K, ho, wo)):
            raise ValueError("offset / mask shape does not match the conv geometry")
        xcl = x.permute(0, 2, 3, 1).contiguous()
        cols = torch.empty((n, 1, ho, wo, K * c), dtype=torch.float32, device=x.device)
        sp = N.stream_ptr(x.device)
        N.check(lib.vsrk_dcn_im2col(geo, xcl.data_ptr(), offset.data_ptr(), N.ptr(mask), cols.data_ptr(), sp),
                "dcn_im2col")
        w1 = weight.float().permute(0, 2, 3, 1).reshape(co, K * c, 1, 1).contiguous()
        y = torch.empty((n, 1, ho, wo, co), dtype=torch.float32, device=x.device)
        F.conv(cols, F.pack_weight(w1, 0, torch.float32), y, K1, P0,
               bias=bias.float() if bias is not None else None)
        ctx.save_for_backward(xcl, offset, mask, w1, cols)
        ctx.geo, ctx.shape, ctx.has_bias = geo, (n, c, co, kh, kw, ho, wo), bias is not None
        ctx.has_mask = mask is not None
        return y.view(n, ho, wo, co).permute(0, 3, 1, 2).contiguous()

    @staticmethod
    def backward(ctx, gy):
        xcl, offset, mask, w1, cols = ctx.saved_tensors
        n, c, co, kh, kw, ho, wo = ctx.shape
        K = kh * kw
        lib = N.load()
        sp = N.stream_ptr(gy.device)
        g = gy.float().permute(0, 2, 3, 1).contiguous().view(n, 1, ho, wo, co)
        gcols = torch.empty_like(cols)
        F.conv(g, F.pack_weight(w1, 1, torch.float32), gcols, K1, P0)
        dw = torch.empty((co, K * c, 1, 1, 1), dtype=torch.float32, device=gy.device)
        db = torch.empty(co, dtype=torch.float32, device=gy.device) if ctx.has_bias else None
        F.conv_wgrad(cols, g, K1, P0, dw, db)
        grad_w = dw.view(co, kh, kw, c).permute(0, 3, 1, 2).contiguous()
        gx = torch.zeros_like(xcl)
        N.check(lib.vsrk_dcn_col2im(ctx.geo, gcols.data_ptr(), offset.data_ptr(), N.ptr(mask), gx.data_ptr(), sp),
                "dcn_col2im")
        goff = torch.empty_like(offset)
        gmask = torch.empty_like(mask) if mask is not None else None
        N.check(lib.vsrk_dcn_coord_grad(ctx.geo, xcl.data_ptr(), gcols.data_ptr(), offset.data_ptr(), N.ptr(mask),
                                        goff.data_ptr(), N.ptr(gmask), sp), "dcn_coord_grad")
        return (gx.permute(0, 3, 1, 2).contiguous(), goff, gmask, grad_w, db, None, None, None, None, None)


def modulated_deform_conv(x, offset, mask, weight, bias=None, stride=1, padding=0, dilation=1, groups=1,
                          deformable_groups=1):
    """ModulatedDeformConvFunction.apply (deform_conv.py:97-158)."""
    return _DcnFunction.apply(x, offset, mask, weight, bias, _pair(stride), _pair(padding), _pair(dilation), groups,
                              deformable_groups)


def deform_conv(x, offset, weight, stride=1, padding=0, dilation=1, groups=1, deformable_groups=1):
    """DeformConvFunction.apply (deform_conv.py:15-94): DCNv1 = no modulation, no bias."""
    return _DcnFunction.apply(x, offset, None, weight, None, _pair(stride), _pair(padding), _pair(dilation), groups,
                              deformable_groups)


class DeformConv(nn.Module):
    """deform_conv.py:161-197."""

    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0, dilation=1, groups=1,
                 deformable_groups=1, bias=False):
        super().__init__()
        assert not bias
        assert in_channels % groups == 0, f"in_channels {in_channels} cannot be divisible by groups {groups}"
        assert out_channels % groups == 0, f"out_channels {out_channels} cannot be divisible by groups {groups}"
        self.in_channels = in_channels
        self.out_channels = out_channels
        self.kernel_size = _pair(kernel_size)
        self.stride = _pair(stride)
        self.padding = _pair(padding)
        self.dilation = _pair(dilation)
        self.groups = groups
        self.deformable_groups = deformable_groups
        self.weight = nn.Parameter(torch.Tensor(out_channels, in_channels // self.groups, *self.kernel_size))
        self.reset_parameters()

    def reset_parameters(self):
        n = self.in_channels
        for k in self.kernel_size:
            n *= k
        stdv = 1. / math.sqrt(n)
        self.weight.data.uniform_(-stdv, stdv)

    def forward(self, x, offset):
        return deform_conv(x, offset, self.weight, self.stride, self.padding, self.dilation, self.groups,
                           self.deformable_groups)


class DeformConvPack(DeformConv):
    """deform_conv.py:200-219: the offsets from a zero-initialised conv of x."""

    def __init__(self, *args, **kwargs):
        super().__init__(*args, **kwargs)
        self.conv_offset = HipConv2d(self.in_channels, self.deformable_groups * 2 * self.kernel_size[0] *
                                     self.kernel_size[1], kernel_size=self.kernel_size, stride=_pair(self.stride),
                                     padding=_pair(self.padding), bias=True)
        self.init_offset()

    def init_offset(self):
        self.conv_offset.weight.data.zero_()
        self.conv_offset.bias.data.zero_()

    def forward(self, x):
        offset = self.conv_offset(x)
        return deform_conv(x, offset, self.weight, self.stride, self.padding, self.dilation, self.groups,
                           self.deformable_groups)


class ModulatedDeformConv(nn.Module):
    """deform_conv.py:222-258."""

    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0, dilation=1, groups=1,
                 deformable_groups=1, bias=True):
        super().__init__()
        self.in_channels = in_channels
        self.out_channels = out_channels
        self.kernel_size = _pair(kernel_size)
        self.stride = stride
        self.padding = padding
        self.dilation = dilation
        self.groups = groups
        self.deformable_groups = deformable_groups
        self.with_bias = bias
        self.weight = nn.Parameter(torch.Tensor(out_channels, in_channels // groups, *self.kernel_size))
        if bias:
            self.bias = nn.Parameter(torch.Tensor(out_channels))
        else:
            self.register_parameter("bias", None)
        self.reset_parameters()

    def reset_parameters(self):
        n = self.in_channels
        for k in self.kernel_size:
            n *= k
        stdv = 1. / math.sqrt(n)
        self.weight.data.uniform_(-stdv, stdv)
        if self.bias is not None:
            self.bias.data.zero_()

    def forward(self, x, offset, mask):
        return modulated_deform_conv(x, offset, mask, self.weight, self.bias, self.stride, self.padding,
                                     self.dilation, self.groups, self.deformable_groups)


class ModulatedDeformConvPack(ModulatedDeformConv):
    """deform_conv.py:261-300 (EDVR's DCNv2Pack): offsets and sigmoid masks from
    a zero-initialised conv of x (or of the features x[1] with extra_offset_mask)."""

    def __init__(self, *args, extra_offset_mask=False, **kwargs):
        super().__init__(*args, **kwargs)
        self.extra_offset_mask = extra_offset_mask
        self.conv_offset_mask = HipConv2d(self.in_channels, self.deformable_groups * 3 * self.kernel_size[0] *
                                          self.kernel_size[1], kernel_size=self.kernel_size,
                                          stride=_pair(self.stride), padding=_pair(self.padding), bias=True)
        self.init_offset()

    def init_offset(self):
        self.conv_offset_mask.weight.data.zero_()
        self.conv_offset_mask.bias.data.zero_()

    def forward(self, x):
        if self.extra_offset_mask:
            out = self.conv_offset_mask(x[1])
            x = x[0]
        else:
            out = self.conv_offset_mask(x)
        o1, o2, mask = torch.chunk(out, 3, dim=1)
        offset = torch.cat((o1, o2), dim=1)
        mask = torch.sigmoid(mask)
        offset_mean = torch.mean(torch.abs(offset))
        if offset_mean > 100:
            logger.warning("Offset mean is %s, larger than 100.", offset_mean)
        return modulated_deform_conv(x, offset, mask, self.weight, self.bias, self.stride, self.padding,
                                     self.dilation, self.groups, self.deformable_groups)
