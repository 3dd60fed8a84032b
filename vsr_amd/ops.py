"""PyTorch custom operators over the vsrk C ABI: ``torch.ops.vsrk.*``.

The generators (vsr_amd.nets) run fused HIP pipelines with hand-written
backward passes.  This module exposes the same kernels one op at a time, as
torch.library custom operators with autograd formulas, for code that builds
its own networks from torch.nn-style layers (the precedent in the reference
is its DCN extension: pybind ops with autograd Functions,
src/model/nets/edvr_net/dcn/src/deform_conv_cuda.cpp:681-695 and
deform_conv.py:15-154).  Tensors are the reference's NC(D)HW layout at the
op boundary; internally the kernels work on channels-last views, so each op
converts in and out (the fused generators avoid that).

  vsrk::conv(x, weight, bias, padding, act, x_shuffle, y_shuffle, view_order)
      nn.Conv2d / nn.Conv3d (kernel 1 or 3 in h, w; any kd), fused ReLU,
      sub-pixel input / output views (a fused PixelShuffle: y_shuffle = r)
  vsrk::subpixel_weight(weight, bias, k, s, p, transposed)
      the 3x3 sub-pixel form of DRF's ConvTranspose2d / strided Conv2d
  vsrk::batch_norm_stats(x, weight, bias, running_mean, running_var,
                         training, momentum, eps) -> (scale, shift, mean, invstd)
  vsrk::batch_norm(x, weight, bias, stats, training, relu)
      nn.BatchNorm3d (+ nn.ReLU): statistics (running statistics updated in
      training), then the normalisation with its autograd formula
  vsrk::duf_dynfilter(x, logits, residual, k, r)   DUF dynamic upsampling
  vsrk::loss(out, target, kind, param)             L1 / MSE / Huber / Charbonnier
  vsrk::psnr(out, target, mean, std, max_value, denormalize) -> per-sample
  vsrk::ssim(out, target, mean, std, value_range, denormalize) -> per-sample

Every op launches HIP kernels on torch's current stream and raises when the
native library is missing: there is no CPU or ATen fallback.
"""
from __future__ import annotations

from typing import List, Optional, Tuple

import torch
from torch import Tensor

from . import functional as F

_ACTS = {"none": F.ACT_NONE, "relu": F.ACT_RELU}


# ----------------------------------------------------------------- layout --
def _to_cl(x: Tensor, dtype: torch.dtype) -> Tensor:
    """(N, C, [D,] H, W) -> channels-last (N, D, H, W, C) in dtype; 1..7-channel
    maps live in 8-channel zero-padded storage (the kernels read 16 B chunks)."""
    c = x.shape[1]
    cpad = 8 if c < 8 else None
    return F.to_view(x.float() if x.dtype != torch.float32 else x, dtype, cpad=cpad)[..., :c]


def _empty_cl(lead, c: int, dtype: torch.dtype, device) -> Tensor:
    """Uninitialised channels-last (*lead, c) view; c < 8 in 8-channel storage."""
    return torch.empty((*lead, 8 if c < 8 else c), dtype=dtype, device=device)[..., :c]


def _from_cl(v: Tensor, two_d: bool, dtype: torch.dtype) -> Tensor:
    out = F.from_view(v, two_d=two_d)
    return out if dtype == torch.float32 else out.to(dtype)


def _k3(w: Tensor) -> Tuple[int, int, int]:
    return tuple(w.shape[2:]) if w.dim() == 5 else (1, w.shape[2], w.shape[3])


def _pad3(padding: List[int], two_d: bool) -> Tuple[int, int, int]:
    return (0, padding[0], padding[1]) if two_d else (padding[0], padding[1], padding[2])


def _out_shape(x: Tensor, w: Tensor, padding, x_shuffle: int, y_shuffle: int):
    two_d = x.dim() == 4
    k = _k3(w)
    p = _pad3(padding, two_d)
    n = x.shape[0]
    d = 1 if two_d else x.shape[2]
    h, ww = x.shape[-2] // x_shuffle, x.shape[-1] // x_shuffle
    do = d + 2 * p[0] - k[0] + 1
    cout = w.shape[0] // (y_shuffle * y_shuffle)
    ho, wo = h * y_shuffle, ww * y_shuffle
    return (n, cout, ho, wo) if two_d else (n, cout, do, ho, wo)


# ------------------------------------------------------------------- conv --
@torch.library.custom_op("vsrk::conv", mutates_args=())
def conv(x: Tensor, weight: Tensor, bias: Optional[Tensor], padding: List[int], act: str = "none",
         x_shuffle: int = 1, y_shuffle: int = 1, view_order: bool = False) -> Tensor:
    """y = act(conv(x, weight) + bias), optionally read through a sub-pixel
    input view (x_shuffle: logical channels = C * s^2) and / or stored through a
    sub-pixel output view (y_shuffle = r: conv -> nn.PixelShuffle(r)).  The
    output channels of weight are in nn.PixelShuffle order (c*r*r + i*r + j)
    unless view_order (sub-pixel-major, as vsrk::subpixel_weight makes them)."""
    two_d = x.dim() == 4
    k = _k3(weight)
    p = _pad3(padding, two_d)
    cd = x.dtype
    xv = _to_cl(x, cd)
    shape = _out_shape(x, weight, padding, x_shuffle, y_shuffle)
    n, cout = shape[0], shape[1]
    do = 1 if two_d else shape[2]
    yv = _empty_cl((n, do, shape[-2], shape[-1]), cout, cd, x.device)
    perm = 1 if view_order else y_shuffle
    wp = F.pack_weight(weight.float(), 0, cd, perm_r=perm)
    F.conv(xv, wp, yv, k, p, bias=bias.float() if bias is not None else None, act=_ACTS[act],
           x_shuffle=x_shuffle, y_shuffle=y_shuffle, bias_r=perm)
    return _from_cl(yv, two_d, cd)


@conv.register_fake
def _(x, weight, bias, padding, act="none", x_shuffle=1, y_shuffle=1, view_order=False):
    return x.new_empty(_out_shape(x, weight, padding, x_shuffle, y_shuffle))


@torch.library.custom_op("vsrk::conv_backward", mutates_args=())
def conv_backward(grad: Tensor, x: Tensor, weight: Tensor, y: Tensor, padding: List[int], act: str,
                  x_shuffle: int, y_shuffle: int, view_order: bool,
                  need_bias: bool) -> Tuple[Tensor, Tensor, Tensor]:
    """(grad_x, grad_weight, grad_bias) of vsrk::conv.  The ReLU mask comes
    from the saved output y (fused into the data-gradient epilogue; the weight
    gradient reads the masked gradient)."""
    two_d = x.dim() == 4
    k = _k3(weight)
    p = _pad3(padding, two_d)
    cd = x.dtype
    gv = _to_cl(grad, cd)
    if act == "relu":
        yv = _to_cl(y, cd)
        masked = _empty_cl(gv.shape[:-1], gv.shape[-1], cd, x.device)
        F.relu_bwd(yv, gv, masked)
        gv = masked
    xv = _to_cl(x, cd)
    dpad = tuple(kk - 1 - pp for kk, pp in zip(k, p))
    dxv = _empty_cl(xv.shape[:-1], xv.shape[-1], cd, x.device)
    perm = 1 if view_order else y_shuffle
    F.conv(gv, F.pack_weight(weight.float(), 1, cd, perm_r=perm), dxv, k, dpad, x_shuffle=y_shuffle,
           y_shuffle=x_shuffle)
    gw = torch.empty(weight.shape, dtype=torch.float32, device=x.device)
    gb = torch.empty(weight.shape[0], dtype=torch.float32, device=x.device)
    w5 = gw if gw.dim() == 5 else gw.view(*gw.shape[:2], 1, *gw.shape[2:])
    F.conv_wgrad(xv, gv, k, p, w5, gb if need_bias else None, perm_r=perm, x_shuffle=x_shuffle,
                 dy_shuffle=y_shuffle)
    return _from_cl(dxv, two_d, cd), gw.to(weight.dtype), gb.to(weight.dtype)


@conv_backward.register_fake
def _(grad, x, weight, y, padding, act, x_shuffle, y_shuffle, view_order, need_bias):
    return x.new_empty(x.shape), weight.new_empty(weight.shape), weight.new_empty(weight.shape[0])


def _conv_setup(ctx, inputs, output):
    x, weight, bias, padding, act, x_shuffle, y_shuffle, view_order = inputs
    ctx.save_for_backward(x, weight, output)
    ctx.cfg = (list(padding), act, x_shuffle, y_shuffle, view_order, bias is not None)


def _conv_bwd(ctx, grad):
    x, weight, y = ctx.saved_tensors
    padding, act, xs, ys, vo, has_bias = ctx.cfg
    gx, gw, gb = conv_backward(grad.contiguous(), x, weight, y, padding, act, xs, ys, vo, has_bias)
    return gx, gw, (gb if has_bias else None), None, None, None, None, None


conv.register_autograd(_conv_bwd, setup_context=_conv_setup)


# ----------------------------------------------------- sub-pixel weights --
@torch.library.custom_op("vsrk::subpixel_weight", mutates_args=())
def subpixel_weight(weight: Tensor, bias: Optional[Tensor], k: int, s: int, p: int,
                    transposed: bool) -> Tuple[Tensor, Tensor]:
    """The exact 3x3 sub-pixel weight / bias of nn.Conv2d or nn.ConvTranspose2d
    (k, stride s, padding p) -- drf_net.py:70-102 (see vsrk_subpixel_conv_weight)."""
    return F.subpixel_conv_weight(weight, bias, k, s, p, transposed)


@subpixel_weight.register_fake
def _(weight, bias, k, s, p, transposed):
    if transposed:
        cin, cout = weight.shape[:2]
        return weight.new_empty((s * s * cout, cin, 3, 3)), weight.new_empty(s * s * cout)
    cout, cin = weight.shape[:2]
    return weight.new_empty((cout, s * s * cin, 3, 3)), weight.new_empty(cout)


def _spw_setup(ctx, inputs, output):
    weight, bias, k, s, p, transposed = inputs
    ctx.cfg = (weight.shape, bias is not None, k, s, p, transposed)


def _spw_bwd(ctx, gweq, gbeq):
    shape, has_bias, k, s, p, transposed = ctx.cfg
    dw = torch.empty(shape, dtype=torch.float32, device=gweq.device)
    db = torch.empty(shape[1] if transposed else shape[0], dtype=torch.float32, device=gweq.device)
    F.subpixel_wgrad_fold(gweq.float().contiguous(), gbeq.float().contiguous(), dw, db if has_bias else None,
                          k, s, p, transposed)
    return dw, (db if has_bias else None), None, None, None, None


subpixel_weight.register_autograd(_spw_bwd, setup_context=_spw_setup)


# ------------------------------------------------------------- batch norm --
@torch.library.custom_op("vsrk::batch_norm_stats", mutates_args=("running_mean", "running_var"))
def batch_norm_stats(x: Tensor, weight: Optional[Tensor], bias: Optional[Tensor], running_mean: Tensor,
                     running_var: Tensor, training: bool, momentum: float, eps: float) -> Tensor:
    """nn.BatchNorm3d statistics -> (4, C) fp32: scale = gamma*invstd, shift,
    mean, invstd.  Training: batch statistics of x, running statistics
    updated in place (momentum, unbiased variance, torch semantics).  Eval:
    running statistics.  (Mutating, so no autograd formula of its own: the
    gradient through the batch statistics is part of vsrk::batch_norm's.)"""
    if training:
        xv = _to_cl(x, x.dtype)
        sums = F.bn_stats(xv)
        count = xv.shape[0] * xv.shape[1] * xv.shape[2] * xv.shape[3]
        return F.bn_finalize(sums, count, weight, bias, eps, momentum, running_mean, running_var)
    return F.bn_fold_running(weight, bias, running_mean, running_var, eps)


@batch_norm_stats.register_fake
def _(x, weight, bias, running_mean, running_var, training, momentum, eps):
    return x.new_empty((4, x.shape[1]), dtype=torch.float32)


@torch.library.custom_op("vsrk::batch_norm", mutates_args=())
def batch_norm(x: Tensor, weight: Optional[Tensor], bias: Optional[Tensor], stats: Tensor, training: bool,
               relu: bool) -> Tensor:
    """y = x * scale + shift [relu] with stats from vsrk::batch_norm_stats."""
    xv = _to_cl(x, x.dtype)
    yv = _empty_cl(xv.shape[:-1], xv.shape[-1], x.dtype, x.device)
    F.bn_apply(xv, stats[0].contiguous(), stats[1].contiguous(), relu, yv)
    return _from_cl(yv, x.dim() == 4, x.dtype)


@batch_norm.register_fake
def _(x, weight, bias, stats, training, relu):
    return x.new_empty(x.shape)


@torch.library.custom_op("vsrk::batch_norm_backward", mutates_args=())
def batch_norm_backward(grad: Tensor, x: Tensor, weight: Optional[Tensor], stats: Tensor, training: bool,
                        relu: bool) -> Tuple[Tensor, Tensor, Tensor]:
    """(grad_x, grad_weight, grad_bias).  Without ReLU the mask operands are
    (scale 0, shift 1); in eval mode the batch-statistics terms vanish
    (count = inf)."""
    xv, gv = _to_cl(x, x.dtype), _to_cl(grad, x.dtype)
    st = stats
    if not relu:
        st = stats.clone()
        st[0].zero_()
        st[1].fill_(1.0)
    red = F.bn_relu_bwd_reduce(xv, gv, st)
    count = xv.shape[0] * xv.shape[1] * xv.shape[2] * xv.shape[3] if training else float("inf")
    dxv = _empty_cl(xv.shape[:-1], xv.shape[-1], x.dtype, x.device)
    F.bn_relu_bwd_apply(xv, gv, st, weight, red, count, dxv)
    return _from_cl(dxv, x.dim() == 4, x.dtype), red[1].clone(), red[0].clone()


@batch_norm_backward.register_fake
def _(grad, x, weight, stats, training, relu):
    c = x.shape[1]
    return x.new_empty(x.shape), stats.new_empty(c), stats.new_empty(c)


def _bn_setup(ctx, inputs, output):
    x, weight, bias, stats, training, relu = inputs
    ctx.save_for_backward(x, weight, stats)
    ctx.cfg = (training, relu, weight is not None, bias is not None)


def _bn_bwd(ctx, gy):
    x, weight, stats = ctx.saved_tensors
    training, relu, hw, hb = ctx.cfg
    gx, gw, gb = batch_norm_backward(gy.contiguous(), x, weight, stats, training, relu)
    return gx, (gw if hw else None), (gb if hb else None), None, None, None


batch_norm.register_autograd(_bn_bwd, setup_context=_bn_setup)


# ----------------------------------------------------------- DUF filter --
@torch.library.custom_op("vsrk::duf_dynfilter", mutates_args=())
def duf_dynfilter(x: Tensor, logits: Tensor, residual: Tensor, k: int, r: int) -> Tensor:
    """duf_net.py:67-97: softmax over the k*k taps of per-pixel logits (N, k*k*r*r,
    H, W) (tap-major), unfold of x (N, 1, H, W), contraction, pixel shuffle and
    the residual (N, r*r, H, W) added -> (N, 1, r*H, r*W)."""
    n, _, h, w = x.shape
    lg = logits.float().permute(0, 2, 3, 1).contiguous()
    rs = residual.float().permute(0, 2, 3, 1).contiguous()
    return F.duf_dynfilter_fwd(x.float().reshape(n, h, w).contiguous(), lg, rs, k, r)


@duf_dynfilter.register_fake
def _(x, logits, residual, k, r):
    n, _, h, w = x.shape
    return x.new_empty((n, 1, h * r, w * r), dtype=torch.float32)


def _duf_setup(ctx, inputs, output):
    x, logits, residual, k, r = inputs
    ctx.save_for_backward(x, logits)
    ctx.cfg = (k, r)


def _duf_bwd(ctx, g):
    x, logits = ctx.saved_tensors
    k, r = ctx.cfg
    n, _, h, w = x.shape
    lg = logits.float().permute(0, 2, 3, 1).contiguous()
    dl, dr = F.duf_dynfilter_bwd(x.float().reshape(n, h, w).contiguous(), lg, g, k, r, torch.float32)
    return None, dl.permute(0, 3, 1, 2).to(logits.dtype), dr.permute(0, 3, 1, 2), None, None


duf_dynfilter.register_autograd(_duf_bwd, setup_context=_duf_setup)


# ------------------------------------------------------------ losses etc --
@torch.library.custom_op("vsrk::loss", mutates_args=())
def loss(out: Tensor, target: Tensor, kind: int, param: float) -> Tensor:
    """Mean-reduced loss: kind 0 L1, 1 MSE, 2 Huber(delta), 3 Charbonnier(eps)
    (losses.py:5-34)."""
    return F.loss_fwd(kind, param, out.float(), target.float())


@loss.register_fake
def _(out, target, kind, param):
    return out.new_empty((), dtype=torch.float32)


def _loss_setup(ctx, inputs, output):
    out, target, kind, param = inputs
    ctx.save_for_backward(out, target)
    ctx.cfg = (kind, param)


def _loss_bwd(ctx, g):
    out, target = ctx.saved_tensors
    kind, param = ctx.cfg
    gi = F.loss_bwd(kind, param, out.float(), target.float(), g.detach().reshape(()), torch.float32)
    return gi.to(out.dtype), None, None, None


loss.register_autograd(_loss_bwd, setup_context=_loss_setup)


@torch.library.custom_op("vsrk::psnr", mutates_args=())
def psnr(out: Tensor, target: Tensor, mean: float, std: float, max_value: float, denormalize: bool) -> Tensor:
    """Per-sample PSNR [of denormalized images] (utils.py:1-20, metrics.py:20-36)."""
    return F.psnr(out, target, mean, std, max_value, denormalize)[1]


@psnr.register_fake
def _(out, target, mean, std, max_value, denormalize):
    return out.new_empty(out.shape[0], dtype=torch.float32)


@torch.library.custom_op("vsrk::ssim", mutates_args=())
def ssim(out: Tensor, target: Tensor, mean: float, std: float, value_range: float, denormalize: bool) -> Tensor:
    """Per-sample 2-D SSIM [of denormalized images] (metrics.py:39-113)."""
    return F.ssim(out, target, mean, std, value_range, denormalize)[1]


@ssim.register_fake
def _(out, target, mean, std, value_range, denormalize):
    return out.new_empty(out.shape[0], dtype=torch.float32)
