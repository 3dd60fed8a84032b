"""EDSR-style 2-D generator on fused HIP kernels.

Same constructor, module tree and state_dict keys as the reference
EDSRNet (src/model/nets/edsr_net.py:8-67), so reference checkpoints load and
the same seed gives the same initial weights:

    head.0                        conv3x3 in -> F            (edsr_net.py:28)
    body.{i}.body.conv1 / conv2   resblock conv3x3 F -> F    (edsr_net.py:41-53)
    body.conv                     conv3x3 F -> F, + head     (edsr_net.py:30,36)
    tail.0.conv{j}                conv3x3 F -> s^2 F, PixelShuffle(s)  (edsr_net.py:56-67)
    tail.conv                     conv3x3 F -> out           (edsr_net.py:32)

Fusions (one HIP conv launch each): ReLU in conv1's epilogue, the
``res.mul(res_scale) += x`` residual in conv2's epilogue, the global skip in
body.conv's epilogue, nn.PixelShuffle as the sub-pixel output view of the up
convs.  Backward fuses the ReLU mask and res_scale into the data-gradient
epilogues and accumulates skip gradients in place.
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn

from .. import functional as F
from .base_net import BaseNet

K3 = (1, 3, 3)
P1 = (0, 1, 1)


def _up_steps(r: int) -> list[int]:
    if math.log(r, 2) % 1 == 0:
        return [2] * int(math.log(r, 2))
    if r == 3:
        return [3]
    raise NotImplementedError(f"upscale factor {r}")


class _ResBlock(nn.Module):
    def __init__(self, f: int, res_scale: float):
        super().__init__()
        self.body = nn.Sequential()
        self.body.add_module("conv1", nn.Conv2d(f, f, 3, padding=1))
        self.body.add_module("relu1", nn.ReLU())
        self.body.add_module("conv2", nn.Conv2d(f, f, 3, padding=1))
        self.res_scale = res_scale


class _UpBlock(nn.Sequential):
    def __init__(self, f: int, r: int):
        super().__init__()
        for j, s in enumerate(_up_steps(r), start=1):
            self.add_module(f"conv{j}", nn.Conv2d(f, s * s * f, 3, padding=1))
            self.add_module(f"deconv{j}", nn.PixelShuffle(s))


class EDSRNet(BaseNet):
    """Enhanced Deep Residual Network (SISR: (B,C,h,w) -> (B,C,rh,rw))."""

    def __init__(self, in_channels, out_channels, num_resblocks, num_features, upscale_factor, res_scale=0.1):
        super().__init__()
        self.in_channels = in_channels
        self.out_channels = out_channels
        self.num_resblocks = num_resblocks
        self.num_features = num_features
        self.upscale_factor = upscale_factor
        self.res_scale = res_scale
        f = num_features
        self.head = nn.Sequential(nn.Conv2d(in_channels, f, 3, padding=1))
        self.body = nn.Sequential(*[_ResBlock(f, res_scale) for _ in range(num_resblocks)])
        self.body.add_module("conv", nn.Conv2d(f, f, 3, padding=1))
        self.tail = nn.Sequential(_UpBlock(f, upscale_factor))
        self.tail.add_module("conv", nn.Conv2d(f, out_channels, 3, padding=1))

    # ------------------------------------------------------------------
    def _blocks(self):
        return [m for m in self.body if isinstance(m, _ResBlock)]

    def _ups(self):
        up = self.tail[0]
        steps = _up_steps(self.upscale_factor)
        return [(getattr(up, f"conv{j}"), s) for j, s in enumerate(steps, start=1)]

    def _run(self, x: torch.Tensor, tape: dict | None):
        cd = self.compute_dtype
        dev = x.device
        b, cin, h, w = x.shape
        f = self.num_features
        new = lambda hh, ww, c: torch.empty((b, 1, hh, ww, c), dtype=cd, device=dev)  # noqa: E731
        xv = F.to_view(x, cd, cpad=8)[..., :cin]  # chunk-aligned storage for the 1-channel input
        head = self.head[0]
        specs = [(head.weight, 0, 1)] + [(c.weight, 0, 1) for blk in self._blocks()
                                         for c in (blk.body.conv1, blk.body.conv2)]
        specs += [(self.body.conv.weight, 0, 1)] + [(c.weight, 0, s) for c, s in self._ups()]
        specs += [(self.tail.conv.weight, 0, 1)]
        pk = self._pack_weights(specs)  # every forward weight in one launch

        def P(conv, perm=1):
            return pk[(id(conv.weight), 0, perm)]

        h0 = F.conv(xv, P(head), new(h, w, f), K3, P1, bias=head.bias)
        saved = []
        cur = h0
        for blk in self._blocks():
            c1, c2 = blk.body.conv1, blk.body.conv2
            t = F.conv(cur, P(c1), new(h, w, f), K3, P1, bias=c1.bias, act=F.ACT_RELU)
            nxt = F.conv(t, P(c2), new(h, w, f), K3, P1, bias=c2.bias,
                         out_scale=blk.res_scale, residual=cur)
            saved.append((cur, t))
            cur = nxt
        bc = self.body.conv
        body_out = F.conv(cur, P(bc), new(h, w, f), K3, P1, bias=bc.bias, residual=h0)
        ups_in = []
        u, hh, ww = body_out, h, w
        for conv, s in self._ups():
            nxt = torch.empty((b, 1, hh * s, ww * s, f), dtype=cd, device=dev)
            F.conv(u, P(conv, s), nxt, K3, P1, bias=conv.bias, y_shuffle=s)
            ups_in.append(u)
            u, hh, ww = nxt, hh * s, ww * s
        tc = self.tail.conv
        y = torch.empty((b, self.out_channels, hh, ww), dtype=torch.float32, device=dev)
        yv = y.view(b, 1, hh, ww, 1) if self.out_channels == 1 else None
        if yv is not None:
            F.conv(u, P(tc), yv, K3, P1, bias=tc.bias)
        else:
            tmp = F.conv(u, P(tc), torch.empty((b, 1, hh, ww, self.out_channels),
                                                                         dtype=torch.float32, device=dev),
                         K3, P1, bias=tc.bias)
            y = F.from_view(tmp)
        if tape is not None:
            tape.update(xv=xv, saved=saved, last=cur, ups_in=ups_in, tail_in=u, hw=(h, w))
        return y

    def _backward(self, tape: dict, gy: torch.Tensor) -> dict:
        cd = self.compute_dtype
        dev = gy.device
        b = gy.shape[0]
        f = self.num_features
        h, w = tape["hw"]
        grads: dict = {}

        def wgrad(conv, x, dy, **kw):
            dw = self._grad_buffer(conv.weight)
            db = self._grad_buffer(conv.bias)
            self._on_wgrad_stream(
                lambda: F.conv_wgrad(x, dy, K3, P1, dw.view(*dw.shape[:2], 1, *dw.shape[2:]), db, **kw), x, dy)
            self._grad_done(grads, conv.weight, dw)
            self._grad_done(grads, conv.bias, db)

        specs = [(self.tail.conv.weight, 1, 1)] + [(c.weight, 1, s) for c, s in self._ups()]
        specs += [(self.body.conv.weight, 1, 1)] + [(c.weight, 1, 1) for blk in self._blocks()
                                                    for c in (blk.body.conv1, blk.body.conv2)]
        pk = self._pack_weights(specs)  # every data-gradient weight in one launch

        def dgrad(conv, dy, out, perm_r=1, **kw):
            return F.conv(dy, pk[(id(conv.weight), 1, perm_r)], out, K3, P1, **kw)

        # tail conv
        u = tape["tail_in"]
        hh, ww = u.shape[2], u.shape[3]
        g = F.to_view(gy, cd, cpad=8)[..., :self.out_channels]  # (b,1,H,W,out), chunk-aligned storage
        tc = self.tail.conv
        wgrad(tc, u, g)
        du = dgrad(tc, g, torch.empty((b, 1, hh, ww, f), dtype=cd, device=dev))
        # up convs (reverse)
        for (conv, s), uin in reversed(list(zip(self._ups(), tape["ups_in"]))):
            wgrad(conv, uin, du, perm_r=s, dy_shuffle=s)
            hh, ww = hh // s, ww // s
            du = dgrad(conv, du, torch.empty((b, 1, hh, ww, f), dtype=cd, device=dev), perm_r=s, x_shuffle=s)
        d_body = du  # grad of body output == grad of the global skip into head
        bc = self.body.conv
        wgrad(bc, tape["last"], d_body)
        gcur = dgrad(bc, d_body, torch.empty((b, 1, h, w, f), dtype=cd, device=dev))
        blocks = self._blocks()
        for i in range(len(blocks) - 1, -1, -1):
            blk = blocks[i]
            xin, t = tape["saved"][i]
            c1, c2 = blk.body.conv1, blk.body.conv2
            wgrad(c2, t, gcur, dy_scale=blk.res_scale)
            dpre = dgrad(c2, gcur, torch.empty_like(t), out_scale=blk.res_scale, mask=t)
            wgrad(c1, xin, dpre)
            if i == 0:
                # dL/dhead = block-0 input grad + global skip grad, accumulated in
                # place -- into d_body, which the body conv's weight gradient reads
                self._join_wgrad()
                gcur = dgrad(c1, dpre, d_body, residual=gcur, accumulate=True)
            else:
                gcur = dgrad(c1, dpre, torch.empty_like(xin), residual=gcur)
        if not blocks:
            gcur = F.add(gcur, d_body, torch.empty_like(gcur))
        wgrad(self.head[0], tape["xv"], gcur)
        return grads
