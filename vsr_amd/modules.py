"""Op-level drop-in modules over ``torch.ops.vsrk`` (vsr_amd.ops).

Each class subclasses the torch.nn layer it replaces, so parameters, buffers,
``state_dict`` keys and constructor arguments are unchanged; only forward()
runs the HIP kernels.  ``swap_modules(net)`` replaces every supported layer
of an existing network in place -- e.g. a reference generator built from its
own source (src/model/nets/*.py) keeps its forward code and weights and runs
its convolutions / batch norms on MI355X:

  nn.Conv2d / nn.Conv3d (kernel 1 or 3 in h, w; stride 1; zero padding)  -> HipConv2d / HipConv3d
  nn.Conv2d(k, stride s, padding p), k <= p + 2s, p <= s (DRF's down
      projections, drf_net.py:93,100)                                   -> HipConv2d (sub-pixel form)
  nn.ConvTranspose2d(k, s, p) (DRF's up projections, drf_net.py:81,86)  -> HipConvTranspose2d
  nn.BatchNorm3d (duf_net.py:116,198,201)                               -> HipBatchNorm3d

Activations, PixelShuffle and tensor plumbing stay torch ops.  The fused
generators in vsr_amd.nets are the fast path; these modules trade a layout
conversion per op for drop-in generality.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from . import ops  # noqa: F401  (registers torch.ops.vsrk)


def _supported_conv(m: nn.Module) -> bool:
    k = m.kernel_size
    return (m.groups == 1 and m.dilation == (1,) * len(k) and m.padding_mode == "zeros"
            and all(s == 1 for s in m.stride) and k[-1] == k[-2] and k[-1] in (1, 3)
            and isinstance(m.padding, tuple))


def _subpixel_ok(k: int, s: int, p: int) -> bool:
    return s > 1 and k <= p + 2 * s and p <= s


class HipConv2d(nn.Conv2d):
    """nn.Conv2d on vsrk::conv (stride 1, kernel 1/3), or -- for a strided
    kernel k with stride s -- a 3x3 conv over the s x s sub-pixel view."""

    def forward(self, x):
        s = self.stride[0]
        if s > 1:
            weq, beq = torch.ops.vsrk.subpixel_weight(self.weight, self.bias, self.kernel_size[0], s,
                                                      self.padding[0], False)
            return torch.ops.vsrk.conv(x, weq, beq if self.bias is not None else None, [1, 1], "none", s, 1)
        return torch.ops.vsrk.conv(x, self.weight, self.bias, list(self.padding), "none", 1, 1)


class HipConv3d(nn.Conv3d):
    def forward(self, x):
        return torch.ops.vsrk.conv(x, self.weight, self.bias, list(self.padding), "none", 1, 1)


class HipConvTranspose2d(nn.ConvTranspose2d):
    """nn.ConvTranspose2d(k, stride s, padding p) as a 3x3 conv storing through
    an s x s sub-pixel output view (exact: every output sub-pixel is one 3x3
    window of the low-resolution input)."""

    def forward(self, x, output_size=None):
        k, s, p = self.kernel_size[0], self.stride[0], self.padding[0]
        weq, beq = torch.ops.vsrk.subpixel_weight(self.weight, self.bias, k, s, p, True)
        return torch.ops.vsrk.conv(x, weq, beq if self.bias is not None else None, [1, 1], "none", 1, s, True)


class HipBatchNorm3d(nn.BatchNorm3d):
    def forward(self, x):
        if self.training and self.track_running_stats and self.num_batches_tracked is not None:
            self.num_batches_tracked.add_(1)
        use_batch = self.training or not self.track_running_stats
        rm = self.running_mean if self.running_mean is not None else torch.zeros(self.num_features, device=x.device)
        rv = self.running_var if self.running_var is not None else torch.ones(self.num_features, device=x.device)
        st = torch.ops.vsrk.batch_norm_stats(x.detach(), self.weight.detach() if self.weight is not None else None,
                                             self.bias.detach() if self.bias is not None else None, rm, rv,
                                             use_batch, self.momentum if self.momentum is not None else 0.1,
                                             self.eps)
        return torch.ops.vsrk.batch_norm(x, self.weight, self.bias, st, use_batch, False)


def _convert(m: nn.Module) -> nn.Module | None:
    if type(m) is nn.Conv2d:
        if _supported_conv(m):
            new = HipConv2d.__new__(HipConv2d)
        elif (m.groups == 1 and m.kernel_size[0] == m.kernel_size[1] and m.stride[0] == m.stride[1]
              and m.padding[0] == m.padding[1] and _subpixel_ok(m.kernel_size[0], m.stride[0], m.padding[0])):
            new = HipConv2d.__new__(HipConv2d)
        else:
            return None
    elif type(m) is nn.Conv3d and _supported_conv(m):
        new = HipConv3d.__new__(HipConv3d)
    elif (type(m) is nn.ConvTranspose2d and m.groups == 1 and m.output_padding == (0, 0)
          and m.kernel_size[0] == m.kernel_size[1] and m.stride[0] == m.stride[1]
          and _subpixel_ok(m.kernel_size[0], m.stride[0], m.padding[0])):
        new = HipConvTranspose2d.__new__(HipConvTranspose2d)
    elif type(m) is nn.BatchNorm3d:
        new = HipBatchNorm3d.__new__(HipBatchNorm3d)
    else:
        return None
    new.__dict__ = m.__dict__  # same parameters, buffers and hyper-parameters
    return new


def swap_modules(net: nn.Module) -> nn.Module:
    """Replace every supported layer of `net` (recursively, in place) by its
    Hip* counterpart; returns net (or its replacement when net itself is a
    supported layer).  Unsupported layers are left as they are."""
    new = _convert(net)
    if new is not None:
        return new
    for name, child in list(net.named_children()):
        new = _convert(child)
        if new is not None:
            setattr(net, name, new)
        else:
            swap_modules(child)
    return net
