"""DUF 3-D generator on fused HIP kernels (the Conv3d 3x3x3 / BatchNorm3d path).

Same constructor, module tree and state_dict keys as the reference DUFNet
(src/model/nets/duf_net.py:9-214): denseLayer.conv{i}.{bn1,conv1,bn2,conv2},
denseLayer.tail.{bn,conv}, head, filterNet.{conv1,conv2},
residualNet.{conv1,conv2}; same construction order, so one seed gives the
same initial weights.

Layout: one channels-last concat buffer C (N, T, H, W, F0 + units*G) holds
the head output and every unit's output.  The reference's
``torch.cat((concat[:, :, 1:-1], x), 1)`` (duf_net.py:122-128) is free: a
depth-valid unit reads the depth window [lo, hi) of C and writes its output
at depth [lo+1, hi-1), channels [F, F+G).  Every BatchNorm3d+ReLU is folded
into the consuming conv's staging prologue (scale/shift from the batch
statistics), so normalised activations are never stored.  The dynamic
upsampling filter (softmax, unfold, contraction, pixel shuffle, residual
add) is one kernel.  Backward accumulates into a concat-gradient buffer dC
of the same layout.

SyncBatchNorm: with ``self.bn_allreduce`` set (vsr_amd.ddp), the per-channel
sums of every BN are all-reduced across ranks before they are used, forward
and backward, so multi-GPU statistics equal single-GPU statistics of the
global batch.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from .. import functional as F
from .base_net import BaseNet

_BACKBONES = {"_DenseLayer16": (32, 3, 256), "_DenseLayer28": (16, 9, 256), "_DenseLayer52": (16, 21, 448)}
ARF = F.PRO_AFFINE_RELU


def _unit(cin: int, growth: int, depth_pad: int) -> nn.Sequential:
    """_denseBlock1 (depth_pad 1) / _denseBlock2 (depth_pad 0), duf_net.py:195-214."""
    u = nn.Sequential()
    u.add_module("bn1", nn.BatchNorm3d(cin))
    u.add_module("relu1", nn.ReLU())
    u.add_module("conv1", nn.Conv3d(cin, cin, kernel_size=1))
    u.add_module("bn2", nn.BatchNorm3d(cin))
    u.add_module("relu2", nn.ReLU())
    u.add_module("conv2", nn.Conv3d(cin, growth, kernel_size=3, padding=(depth_pad, 1, 1)))
    return u


class _DenseLayer(nn.Module):
    """_DenseLayer16/28/52 (duf_net.py:102-192)."""

    def __init__(self, growth: int, n_keep: int, tail_in: int):
        super().__init__()
        self.growth, self.n_keep, self.n_units = growth, n_keep, n_keep + 3
        f = 64
        for i in range(self.n_units):
            setattr(self, f"conv{i}", _unit(f, growth, 1 if i < n_keep else 0))
            f += growth
        assert f == tail_in
        self.tail = nn.Sequential()
        self.tail.add_module("bn", nn.BatchNorm3d(tail_in))
        self.tail.add_module("relu", nn.ReLU())
        self.tail.add_module("conv", nn.Conv3d(tail_in, 256, kernel_size=(1, 3, 3), padding=(0, 1, 1)))


class _ScaledWork:
    """A SyncBN backward all-reduce in flight: wait() orders the stream after
    it and then divides the summed (sum_dy, sum_dy_xhat) by the global count
    on the device, so the apply runs with count 1.  The divisor is formed in
    double (the count is a device float64, as the single-process path's
    qinv_count) and rounded once; a second wait() does nothing."""

    def __init__(self, work, red, count_dev, mult):
        self.work, self.red, self.count_dev, self.mult = work, red, count_dev, mult
        self.done = False

    def wait(self):
        if self.done:
            return
        self.done = True
        self.work.wait()
        self.red.div_((self.count_dev.to(torch.float64) * self.mult).to(self.red.dtype))


class DUFNet(BaseNet):
    """Dynamic Upsampling Filter network (MISR: list of T (B,C,h,w) -> (B,C,rh,rw))."""

    def __init__(self, in_channels, out_channels, num_frames, size_filter, upscale_factor, backbone):
        super().__init__()
        if backbone not in _BACKBONES:
            raise AssertionError(f"backbone {backbone}")
        self.num_frames = num_frames
        self.size_filter = size_filter
        self.upscale_factor = upscale_factor
        self.in_channels = in_channels
        g, n_keep, tail_in = _BACKBONES[backbone]
        self.denseLayer = _DenseLayer(g, n_keep, tail_in)
        self.head = nn.Conv2d(in_channels, 64, kernel_size=3, padding=1)
        k2r2 = size_filter ** 2 * upscale_factor ** 2
        self.filterNet = nn.Sequential()
        for name, mod in (("relu1", nn.ReLU()), ("conv1", nn.Conv3d(256, 512, 1)), ("relu2", nn.ReLU()),
                          ("conv2", nn.Conv3d(512, k2r2, 1))):
            self.filterNet.add_module(name, mod)
        self.residualNet = nn.Sequential()
        for name, mod in (("relu1", nn.ReLU()), ("conv1", nn.Conv3d(256, 256, 1)), ("relu2", nn.ReLU()),
                          ("conv2", nn.Conv3d(256, in_channels * upscale_factor ** 2, 1))):
            self.residualNet.add_module(name, mod)
        self.bn_allreduce = None  # SyncBN hook: callable(tensor) all-reducing in place (sum)

    def _centre(self) -> int:
        n = self.num_frames
        return n // 2 if n % 2 == 1 else n // 2 - 1  # duf_net.py:53

    # -- BatchNorm helpers ------------------------------------------------
    def _bn_forward(self, bn: nn.BatchNorm3d, x: torch.Tensor, sums: torch.Tensor | None = None) -> torch.Tensor:
        """(4, C) = scale, shift, mean, invstd for the fused BN+ReLU prologue.
        sums: x's per-channel (sum, sumsq) when the caller already has them."""
        if not self.training:
            # running statistics; the backward (a gradient taken through an
            # eval-mode net) then has no batch-statistics terms: count = inf
            st = F.bn_fold_running(bn.weight, bn.bias, bn.running_mean, bn.running_var, bn.eps)
            st.count = float("inf")
            return st
        if sums is None:
            sums = F.bn_stats(x)
        else:
            sums = sums.clone()  # the SyncBN hook all-reduces in place
        count, count_dev = x.shape[0] * x.shape[1] * x.shape[2] * x.shape[3], None
        if self.bn_allreduce is not None:
            self.bn_allreduce(sums)
            # depth x the N*H*W of every rank, a device scalar (no host read)
            count, count_dev = x.shape[1], self._global_nhw
        st = F.bn_finalize(sums, count, bn.weight, bn.bias, bn.eps, bn.momentum if bn.momentum is not None else 0.1,
                           bn.running_mean if bn.track_running_stats else None,
                           bn.running_var if bn.track_running_stats else None, count_dev=count_dev)
        if bn.track_running_stats and bn.num_batches_tracked is not None:
            bn.num_batches_tracked.add_(1)
        # the backward's apply takes 1 / count: SyncBN hands it sums already
        # divided by the device count (_bn_backward_reduce) and count 1
        st.count = count if count_dev is None else 1.0
        st.count_dev = (count_dev, float(count)) if count_dev is not None else None
        return st

    def _bn_backward_reduce(self, bn, x, dz, st, grads, red=None):
        """The reduce half of the BN+ReLU backward: writes dgamma / dbeta and
        returns (the (sum_dy, sum_dy_xhat) that feed the input gradient, the
        work handle of their SyncBN all-reduce or None).  The all-reduce is
        asynchronous: the caller queues independent work (a weight gradient)
        before waiting on the handle.  red: the sums when the producing conv
        already reduced them (F.conv_reduce)."""
        if red is None:
            red = F.bn_relu_bwd_reduce(x, dz, st)
        # dgamma / dbeta are this rank's local sums: the data-parallel gradient
        # average (GradSync) combines them across ranks, as torch's
        # SyncBatchNorm does.  Only the copy that feeds the input gradient is
        # all-reduced (sum over the global batch, with the global count).
        gw = self._grad_buffer(bn.weight)
        gb = self._grad_buffer(bn.bias)
        gw.copy_(red[1])
        gb.copy_(red[0])
        work = None
        if self.bn_allreduce is not None and st.count != float("inf"):
            red = red.clone()
            work = _ScaledWork(self.bn_allreduce.start(red), red, *st.count_dev)
        self._grad_done(grads, bn.weight, gw)
        self._grad_done(grads, bn.bias, gb)
        return red, work

    # ----------------------------------------------------------------------
    def _run(self, inputs, tape: dict | None):
        if len(inputs) != self.num_frames:
            raise ValueError(f"expected {self.num_frames} frames, got {len(inputs)}")
        cd = self.compute_dtype
        dl = self.denseLayer
        n, cin, h, w = inputs[0].shape
        if cin != 1:
            raise NotImplementedError("the fused DUF path supports in_channels == 1")
        dev = inputs[0].device
        T, k, r, g = self.num_frames, self.size_filter, self.upscale_factor, dl.growth
        ctot = 64 + dl.n_units * g
        if T - 2 * 3 != 1:
            # the reference's residual branch squeezes depth 1 (duf_net.py:94-96) and only works for T = 7
            raise RuntimeError(f"DUFNet needs num_frames = 7 (got {T}): depth after the dense layer must be 1")
        if self.training and self.bn_allreduce is not None:
            self._global_nhw = self.bn_allreduce.global_count(n * h * w, dev)  # SyncBN: the global batch
        frames = torch.stack(inputs, dim=2)  # (n, cin, T, h, w) fp32
        xv = F.to_view(frames, cd, cpad=8)[..., :cin]  # (n, T, h, w, cin), chunk-aligned storage
        C = torch.empty((n, T, h, w, ctot), dtype=cd, device=dev)
        F.conv(xv, F.pack_weight(self.head.weight, 0, cd), C[..., :64], (1, 3, 3), (0, 1, 1), bias=self.head.bias)
        # Per-depth (sum, sumsq) of every channel of C, taken once when the
        # channel slice is written: the concat channels never change, so each
        # unit's bn1 (and the tail bn) over a depth window of C[..., :f] is a
        # sum of these rows instead of another pass over f channels.
        S = None
        if self.training:
            S = torch.empty((T, 2, ctot), dtype=torch.float32, device=dev)
            S[:, :, :64] = F.bn_stats_depth(C[..., :64])

        def window_sums(lo_, hi_, c_):
            return None if S is None else S[lo_:hi_, :, :c_].double().sum(0).float()

        units = []
        lo, hi, f = 0, T, 64
        for i in range(dl.n_units):
            u = getattr(dl, f"conv{i}")
            keep = i < dl.n_keep
            R = C[:, lo:hi, :, :, :f]
            st1 = self._bn_forward(u.bn1, R, window_sums(lo, hi, f))
            t1 = torch.empty((n, hi - lo, h, w, f), dtype=cd, device=dev)
            w1 = F.pack_weight(u.conv1.weight, 0, cd)
            # bn2's statistics come out of conv1's store pass (no second read of t1)
            sums2 = F.conv_reduce(R, w1, t1, bias=u.conv1.bias, prologue=ARF, pro_scale=st1[0],
                                  pro_shift=st1[1]) if self.training else None
            if sums2 is None:
                F.conv(R, w1, t1, (1, 1, 1), (0, 0, 0), bias=u.conv1.bias, prologue=ARF, pro_scale=st1[0],
                       pro_shift=st1[1])
            st2 = self._bn_forward(u.bn2, t1, sums2)
            olo, ohi = (lo, hi) if keep else (lo + 1, hi - 1)
            pad = (1, 1, 1) if keep else (0, 1, 1)
            F.conv(t1, F.pack_weight(u.conv2.weight, 0, cd), C[:, olo:ohi, :, :, f:f + g], (3, 3, 3), pad,
                   bias=u.conv2.bias, prologue=ARF, pro_scale=st2[0], pro_shift=st2[1])
            if S is not None:
                S[olo:ohi, :, f:f + g] = F.bn_stats_depth(C[:, olo:ohi, :, :, f:f + g])
            units.append((lo, hi, olo, ohi, f, pad, st1, st2, t1))
            lo, hi, f = olo, ohi, f + g
        Rt = C[:, lo:hi, :, :, :ctot]  # depth window [3, 4) for T = 7
        stt = self._bn_forward(dl.tail.bn, Rt, window_sums(lo, hi, ctot))
        feat = torch.empty((n, 1, h, w, 256), dtype=cd, device=dev)
        F.conv(Rt, F.pack_weight(dl.tail.conv.weight, 0, cd), feat, (1, 3, 3), (0, 1, 1), bias=dl.tail.conv.bias,
               prologue=ARF, pro_scale=stt[0], pro_shift=stt[1])
        fn, rn = self.filterNet, self.residualNet
        h1 = torch.empty((n, 1, h, w, 512), dtype=cd, device=dev)
        F.conv(feat, F.pack_weight(fn.conv1.weight, 0, cd), h1, (1, 1, 1), (0, 0, 0), bias=fn.conv1.bias,
               prologue=F.PRO_RELU, act=F.ACT_RELU)
        logits = torch.empty((n, 1, h, w, k * k * r * r), dtype=torch.float32, device=dev)
        F.conv(h1, F.pack_weight(fn.conv2.weight, 0, cd), logits, (1, 1, 1), (0, 0, 0), bias=fn.conv2.bias)
        r1 = torch.empty((n, 1, h, w, 256), dtype=cd, device=dev)
        F.conv(feat, F.pack_weight(rn.conv1.weight, 0, cd), r1, (1, 1, 1), (0, 0, 0), bias=rn.conv1.bias,
               prologue=F.PRO_RELU, act=F.ACT_RELU)
        res = torch.empty((n, 1, h, w, r * r), dtype=torch.float32, device=dev)
        F.conv(r1, F.pack_weight(rn.conv2.weight, 0, cd), res, (1, 1, 1), (0, 0, 0), bias=rn.conv2.bias)
        centre = inputs[self._centre()].float().contiguous().view(n, h, w)
        out = F.duf_dynfilter_fwd(centre, logits.view(n, h, w, -1), res.view(n, h, w, -1), k, r)
        if tape is not None:
            tape.update(xv=xv, C=C, units=units, tail=(lo, hi, stt), feat=feat, h1=h1, logits=logits, r1=r1,
                        centre=centre, shape=(n, h, w))
        return out

    def _backward(self, tape: dict, gy: torch.Tensor) -> dict:
        cd = self.compute_dtype
        dl, fn, rn = self.denseLayer, self.filterNet, self.residualNet
        n, h, w = tape["shape"]
        k, r, g = self.size_filter, self.upscale_factor, dl.growth
        dev = gy.device
        grads: dict = {}

        def wgrad(conv, x, dy, ksz, pad, **kw):
            dw = self._grad_buffer(conv.weight)
            db = self._grad_buffer(conv.bias)
            w5 = dw if dw.dim() == 5 else dw.view(*dw.shape[:2], 1, *dw.shape[2:])
            self._on_wgrad_stream(lambda: F.conv_wgrad(x, dy, ksz, pad, w5, db, **kw), x, dy)
            self._grad_done(grads, conv.weight, dw)
            self._grad_done(grads, conv.bias, db)

        def dgrad(conv, dy, out, ksz, pad, **kw):
            dpad = tuple(kk - 1 - p for kk, p in zip(ksz, pad))
            return F.conv(dy, F.pack_weight(conv.weight, 1, cd), out, ksz, dpad, **kw)

        K1, P0 = (1, 1, 1), (0, 0, 0)
        dlog, dres = F.duf_dynfilter_bwd(tape["centre"], tape["logits"].view(n, h, w, -1), gy, k, r, cd)
        dlog = dlog.view(n, 1, h, w, -1)
        dres = dres.view(n, 1, h, w, -1)
        feat, h1, r1 = tape["feat"], tape["h1"], tape["r1"]
        # residual branch: relu -> conv1 -> relu -> conv2
        wgrad(rn.conv2, r1, dres, K1, P0)
        dr1 = dgrad(rn.conv2, dres, torch.empty_like(r1), K1, P0, mask=r1)
        wgrad(rn.conv1, feat, dr1, K1, P0, prologue=F.PRO_RELU)
        dfeat = dgrad(rn.conv1, dr1, torch.empty_like(feat), K1, P0, mask=feat)
        # filter branch
        wgrad(fn.conv2, h1, dlog, K1, P0)
        dh1 = dgrad(fn.conv2, dlog, torch.empty_like(h1), K1, P0, mask=h1)
        wgrad(fn.conv1, feat, dh1, K1, P0, prologue=F.PRO_RELU)
        dgrad(fn.conv1, dh1, dfeat, K1, P0, mask=feat, accumulate=True)
        # tail: BN+ReLU -> conv (1,3,3)
        C = tape["C"]
        lo, hi, stt = tape["tail"]
        ctot = C.shape[-1]
        Rt = C[:, lo:hi, :, :, :ctot]
        wgrad(dl.tail.conv, Rt, dfeat, (1, 3, 3), (0, 1, 1), prologue=ARF, pro_scale=stt[0], pro_shift=stt[1])
        dzt = dgrad(dl.tail.conv, dfeat, torch.empty_like(Rt), (1, 3, 3), (0, 1, 1))
        # dC needs no zero fill: every block window is first written whole by
        # its flush (accumulate off: rows no contributor covers become zero)
        dC = torch.empty_like(C)
        # Each unit's bn1 input gradient lands in every concat channel below
        # its f.  Instead of a read-modify-write of dC[..., :f] per unit, the
        # units' (dz1, statistics) are kept and a channel block is summed in
        # one pass over x / dC (up to F.BN_MULTI_MAX contributors per pass)
        # right before the unit that needs it -- the head block at the end.
        # (lo, hi, f, dz, st, gamma, red, count) of the BNs done so far: the
        # tail's bn over every channel at the last depth, then each unit's bn1
        red_t, work_t = self._bn_backward_reduce(dl.tail.bn, Rt, dzt, stt, grads)
        pending = [(lo, hi, ctot, dzt, stt, dl.tail.bn.weight, red_t, stt.count)]
        works = [work_t]  # SyncBN all-reduces in flight (waited before their sums are used)

        def flush(dlo, dhi, c0, c1):
            for wk in works:
                if wk is not None:
                    wk.wait()
            works.clear()
            xs, out = C[:, dlo:dhi, :, :, c0:c1], dC[:, dlo:dhi, :, :, c0:c1]
            cs = [(dz[..., c0:c1], plo - dlo, st[:, c0:c1], gm[c0:c1] if gm is not None else None, red[:, c0:c1], cnt)
                  for plo, phi, pf, dz, st, gm, red, cnt in pending]
            for j in range(0, len(cs), F.BN_MULTI_MAX):
                F.bn_relu_bwd_apply_multi(xs, out, j > 0, cs[j:j + F.BN_MULTI_MAX])

        for i in range(dl.n_units - 1, -1, -1):
            u = getattr(dl, f"conv{i}")
            lo, hi, olo, ohi, f, pad, st1, st2, t1 = tape["units"][i]
            R = C[:, lo:hi, :, :, :f]
            flush(olo, ohi, f, f + g)
            dx_i = dC[:, olo:ohi, :, :, f:f + g]
            # each weight gradient is queued between a BatchNorm reduce and the
            # use of its (SyncBN all-reduced) sums, so it hides the collective
            # bn2's backward reduce comes out of conv2's data-gradient epilogue
            dz2 = torch.empty_like(t1)
            dpad = tuple(kk - 1 - p for kk, p in zip((3, 3, 3), pad))
            pre2 = F.conv_reduce(dx_i, F.pack_weight(u.conv2.weight, 1, cd), dz2, bnx=t1, st=st2, k=(3, 3, 3),
                                 pad=dpad)
            if pre2 is None:
                dgrad(u.conv2, dx_i, dz2, (3, 3, 3), pad)
            red2, work2 = self._bn_backward_reduce(u.bn2, t1, dz2, st2, grads, red=pre2)
            wgrad(u.conv2, t1, dx_i, (3, 3, 3), pad, prologue=ARF, pro_scale=st2[0], pro_shift=st2[1])
            if work2 is not None:
                work2.wait()
            dt1 = torch.empty_like(t1)
            # dz1 reuses dz2's storage; bn2's backward apply is computed in
            # conv1's data-gradient operand load (dt1 stored once, for the
            # weight gradient) and bn1's backward reduce comes out of its
            # store pass, where the shape allows
            dz1 = dz2
            w1t = F.pack_weight(u.conv1.weight, 1, cd)
            pre1 = F.conv_reduce_bnb(t1, dz2, st2, u.bn2.weight, red2, st2.count, dt1, w1t, dz1, bnx=R, st=st1)
            if pre1 is None:
                F.bn_relu_bwd_apply(t1, dz2, st2, u.bn2.weight, red2, st2.count, dt1, False)
                pre1 = F.conv_reduce(dt1, w1t, dz1, bnx=R, st=st1)
            if pre1 is None:
                dgrad(u.conv1, dt1, dz1, K1, P0)
            red1, work1 = self._bn_backward_reduce(u.bn1, R, dz1, st1, grads, red=pre1)
            works.append(work1)
            wgrad(u.conv1, R, dt1, K1, P0, prologue=ARF, pro_scale=st1[0], pro_shift=st1[1])
            pending.append((lo, hi, f, dz1, st1, u.bn1.weight, red1, st1.count))
        flush(0, C.shape[1], 0, 64)
        wgrad(self.head, tape["xv"], dC[..., :64], (1, 3, 3), (0, 1, 1))
        return grads

    def forward(self, inputs):
        return super().forward(list(inputs))
