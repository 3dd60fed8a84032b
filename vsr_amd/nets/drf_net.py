"""DRF (Deep Recurrent Feedback) generators on fused HIP kernels.

Same constructors, module trees and state_dict keys as the reference
DRFNet (src/model/nets/drf_net.py:8-147, VSR: list of T frames -> list of T
outputs) and DRFSISRNet (src/model/nets/drf_sisr_net.py:8-50, SISR: one image
fed num_steps times -> list of num_steps outputs), built in the same order so
one seed gives the same initial weights:

    in_block.{conv1, prelu1, conv2, prelu2}                    (drf_net.py:52-58)
    f_block.in_block.{conv, prelu}                              (:64-66)
    f_block.up_blocks.{0: deconv, prelu | i: conv1, prelu1, deconv2, prelu2}
    f_block.down_blocks.{0: conv, prelu | i: conv1, prelu1, conv2, prelu2}  (:78-102)
    f_block.out_block.{conv, prelu}                             (:104-106)
    out_block.{conv1, pixelshuffle1, ..., conv<n>}              (:136-147)

How it runs (one HIP conv launch per reference conv, PReLU fused into its
epilogue):
  * Concatenations are never materialised: [in_features, hidden] (X0), the
    low-res feature list (L, (G+1)*F channels) and the high-res feature list
    (Hc, G*F channels) are preallocated channels-last buffers; every conv
    writes its channel slice and consumers read channel-prefix views.
  * The feedback hidden state of frame t is written by f_block.out_block's
    conv straight into X0 of frame t+1.
  * ConvTranspose2d / Conv2d(k, stride s, pad p) are 3x3 sub-pixel convs
    (vsrk_subpixel_conv_weight): the deconv writes through a shuffle-s view
    of its Hc slice, the strided conv reads its high-res input through one.
  * Backward is hand-written (frames in reverse): every PReLU output's
    gradient is accumulated from all its consumers into the matching slice of
    a gradient buffer of the concat layout, then one fused pass applies the
    PReLU derivative and reduces its slope gradient.
  * Weight gradients over runs of frames: the weights are shared by all T
    frames (drf_net.py:38-49), so a conv's weight gradient over K frames is
    ONE launch over K*B samples.  Every operand a weight gradient reads --
    forward activations and backward output gradients -- is frame t of a
    frame-major (T, B, h, w, C) sequence buffer, so frames t..t+K-1 are K*B
    consecutive samples of one view.  As the reverse-time backward finishes
    frame t = 0 (mod K) the run's weight gradients are launched on the side
    stream, overlapping the data-gradient chain of the frames still to go;
    the runs accumulate in a fixed order (deterministic).  K keeps every
    view's element offsets within 32 bits (7 at cfg 3), so the pipelined
    kernels stay eligible.  The backward's own sequence buffers are
    allocated in chunks of Kg frames and dropped as soon as every run over a
    chunk is launched: Kg keeps them within VSR_DRF_SEQ_BUDGET_GB (default
    16 GiB; at cfg 3 one frame of them is ~1.2 GB, so Kg = 13 instead of all
    30 frames, ~37 GB).  VSR_DRF_SEQ_WGRAD=0: one launch per frame.
"""
from __future__ import annotations

import math
import os

import torch
import torch.nn as nn

from .. import functional as F
from .base_net import BaseNet

K1, P0 = (1, 1, 1), (0, 0, 0)
K3, P1 = (1, 3, 3), (0, 1, 1)
_PROJ = {2: (6, 2, 2), 3: (7, 3, 2), 4: (8, 4, 2), 8: (12, 8, 2)}  # drf_net.py:70-77


def _prelu():
    return nn.PReLU(num_parameters=1, init=0.2)


class _InBlock(nn.Sequential):
    def __init__(self, in_channels, out_channels):
        super().__init__()
        self.add_module("conv1", nn.Conv2d(in_channels, 4 * out_channels, kernel_size=3, padding=1))
        self.add_module("prelu1", _prelu())
        self.add_module("conv2", nn.Conv2d(4 * out_channels, out_channels, kernel_size=1))
        self.add_module("prelu2", _prelu())


class _FBlock(nn.Module):
    def __init__(self, num_features, num_groups, upscale_factor):
        super().__init__()
        f = num_features
        self.in_block = nn.Sequential()
        self.in_block.add_module("conv", nn.Conv2d(f * 2, f, kernel_size=1))
        self.in_block.add_module("prelu", _prelu())
        self.up_blocks = nn.ModuleList()
        self.down_blocks = nn.ModuleList()
        k, s, p = _PROJ[upscale_factor]
        for i in range(num_groups):
            up, down = nn.Sequential(), nn.Sequential()
            if i == 0:
                up.add_module("deconv", nn.ConvTranspose2d(f, f, kernel_size=k, stride=s, padding=p))
                up.add_module("prelu", _prelu())
                self.up_blocks.append(up)
                down.add_module("conv", nn.Conv2d(f, f, kernel_size=k, stride=s, padding=p))
                down.add_module("prelu", _prelu())
                self.down_blocks.append(down)
            else:
                up.add_module("conv1", nn.Conv2d(f * (i + 1), f, kernel_size=1))
                up.add_module("prelu1", _prelu())
                up.add_module("deconv2", nn.ConvTranspose2d(f, f, kernel_size=k, stride=s, padding=p))
                up.add_module("prelu2", _prelu())
                self.up_blocks.append(up)
                down.add_module("conv1", nn.Conv2d(f * (i + 1), f, kernel_size=1))
                down.add_module("prelu1", _prelu())
                down.add_module("conv2", nn.Conv2d(f, f, kernel_size=k, stride=s, padding=p))
                down.add_module("prelu2", _prelu())
                self.down_blocks.append(down)
        self.out_block = nn.Sequential()
        self.out_block.add_module("conv", nn.Conv2d(f * num_groups, f, kernel_size=1))
        self.out_block.add_module("prelu", _prelu())
        self._hidden_state = None

    @property
    def hidden_state(self):  # API parity (drf_net.py:110-116); the fused path keeps it in X0 buffers
        return self._hidden_state

    @hidden_state.setter
    def hidden_state(self, state):
        self._hidden_state = state


def _up_steps(r: int) -> list[int]:
    if math.log(r, 2) % 1 == 0:
        return [2] * int(math.log(r, 2))
    if r == 3:
        return [3]
    raise ValueError(f"upscale factor {r}")


class _OutBlock(nn.Sequential):
    def __init__(self, in_channels, out_channels, upscale_factor):
        super().__init__()
        steps = _up_steps(upscale_factor)
        for i, s in enumerate(steps):
            self.add_module(f"conv{i + 1}", nn.Conv2d(in_channels, s * s * in_channels, kernel_size=3, padding=1))
            self.add_module(f"pixelshuffle{i + 1}", nn.PixelShuffle(s))
        self.add_module(f"conv{len(steps) + 1}", nn.Conv2d(in_channels, out_channels, kernel_size=3, padding=1))


def _seq_view(views: list) -> torch.Tensor | None:
    """Consecutive frames of one frame-major sequence buffer as a single
    (K*B, 1, h, w, C) view, given the per-frame (B, 1, h, w, C) views in frame
    order; None when they are not consecutive sample blocks of one buffer."""
    v0 = views[0]
    b, _, h, w, c = v0.shape
    sn = v0.stride(0)
    es = v0.element_size()
    for t, v in enumerate(views):
        if v.shape != v0.shape or v.stride() != v0.stride() or v.data_ptr() != v0.data_ptr() + t * b * sn * es:
            return None
    return torch.as_strided(v0, (len(views) * b, 1, h, w, c), v0.stride(), v0.storage_offset())


class _DRFBase(BaseNet):
    _OVERLAP_WGRAD = True  # per-frame launches leave CUs idle: weight gradients fill them
    # weight gradients batched over the sequence (see the module docstring)
    SEQ_WGRAD = os.environ.get("VSR_DRF_SEQ_WGRAD", "1") != "0"
    # the PReLU backwards over concat-gradient slices fused into their last
    # producer (round 5; VSR_DRF_FUSE_SLICES=0 for A/B)
    FUSE_SLICES = os.environ.get("VSR_DRF_FUSE_SLICES", "1") != "0"
    # training: the in_block convs once over all frames (VSR_DRF_BATCH_IN=0 for A/B)
    BATCH_IN_BLOCK = os.environ.get("VSR_DRF_BATCH_IN", "1") != "0"
    # eager training: every PReLU backward call leaves its slope partials in a
    # per-(PReLU, frame) slot, one fixed-order sum per PReLU after the
    # recurrence (VSR_DRF_DEFER_SLOPES=0: one final per call)
    DEFER_SLOPES = os.environ.get("VSR_DRF_DEFER_SLOPES", "1") != "0"
    def __init__(self, in_channels, out_channels, num_features, num_groups, upscale_factor):
        super().__init__()
        self._sp_tmp: dict = {}  # side-stream scratch of the sub-pixel weight gradients
        self.in_channels = in_channels
        self.out_channels = out_channels
        self.num_features = num_features
        self.num_groups = num_groups
        if upscale_factor not in [2, 3, 4, 8]:
            raise ValueError(f"The upscale factor should be 2, 3, 4 or 8. Got {upscale_factor}.")
        self.upscale_factor = upscale_factor
        self.in_block = _InBlock(in_channels, num_features)
        self.f_block = _FBlock(num_features, num_groups, upscale_factor)
        self.out_block = _OutBlock(num_features, out_channels, upscale_factor)

    def _returns_list(self) -> bool:
        return True

    def _frames(self, inputs) -> list:
        raise NotImplementedError

    # -- weights prepared once per forward (shared by all frames and the backward)
    def _packer(self):
        cd = self.compute_dtype
        cache: dict = {}

        def pw(conv, mode=0, perm_r=1):
            key = ("w", id(conv.weight), mode, perm_r)
            if key not in cache:
                cache[key] = F.pack_weight(conv.weight, mode, cd, perm_r=perm_r)
            return cache[key]

        def sp(conv, transposed, mode=0):
            k, s, p = _PROJ[self.upscale_factor]
            key = ("eq", id(conv.weight))
            if key not in cache:
                cache[key] = F.subpixel_conv_weight(conv.weight, conv.bias, k, s, p, transposed)
            weq, beq = cache[key]
            pkey = ("sp", id(conv.weight), mode)
            if pkey not in cache:
                cache[pkey] = F.pack_weight(weq, mode, cd)
            return cache[pkey], beq

        return pw, sp

    def _slopes_async(self):
        """The PReLU slopes, copied to the host without a sync: the backward
        reads them (the copy long done by then) to choose, per PReLU, the
        output-based backward (exact while a > 0) or the pre-activation one
        (nn.PReLU's own, any slope; the pre-activation is recomputed from the
        tape).  Inside graph capture nothing is copied (the replays may run
        with other slopes): every PReLU then takes the pre-activation form."""
        if torch.cuda.is_current_stream_capturing():
            return None
        prelus = [m for m in self.modules() if isinstance(m, nn.PReLU)]
        sl = torch.cat([m.weight.detach().reshape(-1) for m in prelus])
        host = torch.empty(sl.shape, dtype=sl.dtype, pin_memory=True)
        host.copy_(sl, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(sl.device))  # the stream the copy was queued on
        idx, i = {}, 0
        for m in prelus:
            idx[id(m)] = (i, m.weight.numel())
            i += m.weight.numel()
        return host, ev, idx

    def _ups(self):
        steps = _up_steps(self.upscale_factor)
        return [(getattr(self.out_block, f"conv{j}"), s) for j, s in enumerate(steps, start=1)]

    def _last_conv(self):
        return getattr(self.out_block, f"conv{len(_up_steps(self.upscale_factor)) + 1}")

    # ------------------------------------------------------------------
    def _run(self, inputs, tape: dict | None):
        frames = self._frames(inputs)
        cd = self.compute_dtype
        f, G = self.num_features, self.num_groups
        k, s, p = _PROJ[self.upscale_factor]
        b, cin, h, w = frames[0].shape
        dev = frames[0].device
        H, W = h * s, w * s
        PR = F.ACT_PRELU
        pw, sp = self._packer()
        ib, fb = self.in_block, self.f_block

        def new(hh, ww, c):
            return torch.empty((b, 1, hh, ww, c), dtype=cd, device=dev)

        # training (tape): every tensor a weight gradient reads is frame t of
        # a sequence buffer (B, T[+1], h, w, C); inference: per-frame buffers
        T = len(frames)
        seqs: dict | None = {} if tape is not None else None

        def buf(name, t, hh, ww, c, nfr=T):
            if seqs is None:
                return new(hh, ww, c)
            big = seqs.get(name)
            if big is None:
                big = seqs[name] = torch.empty((nfr, b, hh, ww, c), dtype=cd, device=dev)
            return big[t].unsqueeze(1)

        XV = None
        if seqs is not None:  # all input frames in one layout move, frame-major
            XV = F.to_view(torch.cat([x.float() for x in frames]), cd, cpad=8)[..., :cin]  # (T*b, 1, h, w, cin)
        outs, recs = [], []
        X0 = buf("X0", 0, h, w, 2 * f, T + 1)
        batched = seqs is not None and self.BATCH_IN_BLOCK
        if batched:
            # in_features = in_block(x_t) does not depend on the recurrence
            # (drf_net.py:40-41): both in_block convs run once over all T
            # frames of the sequence buffers (per frame they were 2 x T small
            # latency-bound launches)
            buf("u1", 0, h, w, 4 * f)  # creates the (T, B, h, w, 4F) sequence buffer
            U1 = seqs["u1"].view(T * b, 1, h, w, 4 * f)
            F.conv(XV, pw(ib.conv1), U1, K3, P1, bias=ib.conv1.bias, act=PR, act_param=ib.prelu1.weight)
            X0s = seqs["X0"][:T].view(T * b, 1, h, w, 2 * f)
            F.conv(U1, pw(ib.conv2), X0s[..., :f], K1, P0, bias=ib.conv2.bias, act=PR, act_param=ib.prelu2.weight)
        for t, x in enumerate(frames):
            xv = XV[t * b:(t + 1) * b] if XV is not None else F.to_view(x, cd, cpad=8)[..., :cin]
            u1 = buf("u1", t, h, w, 4 * f)
            if not batched:
                F.conv(xv, pw(ib.conv1), u1, K3, P1, bias=ib.conv1.bias, act=PR, act_param=ib.prelu1.weight)
                F.conv(u1, pw(ib.conv2), X0[..., :f], K1, P0, bias=ib.conv2.bias, act=PR,
                       act_param=ib.prelu2.weight)
            if t == 0:  # hidden_state = in_features (drf_net.py:42-43)
                F.conv(u1, pw(ib.conv2), X0[..., f:], K1, P0, bias=ib.conv2.bias, act=PR,
                       act_param=ib.prelu2.weight)
            L = buf("L", t, h, w, (G + 1) * f)
            F.conv(X0, pw(fb.in_block.conv), L[..., :f], K1, P0, bias=fb.in_block.conv.bias, act=PR,
                   act_param=fb.in_block.prelu.weight)
            Hc = buf("Hc", t, H, W, G * f)
            t1s, t2s = [None] * G, [None] * G
            for i in range(G):
                up, dn = fb.up_blocks[i], fb.down_blocks[i]
                if i == 0:
                    src, dec, dpr = L[..., :f], up.deconv, up.prelu
                else:
                    src = buf(f"t1_{i}", t, h, w, f)
                    F.conv(L[..., :(i + 1) * f], pw(up.conv1), src, K1, P0, bias=up.conv1.bias, act=PR,
                           act_param=up.prelu1.weight)
                    t1s[i], dec, dpr = src, up.deconv2, up.prelu2
                wq, bq = sp(dec, True)
                F.conv(src, wq, Hc[..., i * f:(i + 1) * f], K3, P1, bias=bq, bias_r=1, y_shuffle=s, act=PR,
                       act_param=dpr.weight, subpixel=F.subpixel_code(k, s, p, True, False))
                if i == 0:
                    hsrc, cv, cpr = Hc[..., :f], dn.conv, dn.prelu
                else:
                    hsrc = buf(f"t2_{i}", t, H, W, f)
                    F.conv(Hc[..., :(i + 1) * f], pw(dn.conv1), hsrc, K1, P0, bias=dn.conv1.bias, act=PR,
                           act_param=dn.prelu1.weight)
                    t2s[i], cv, cpr = hsrc, dn.conv2, dn.prelu2
                wq, bq = sp(cv, False)
                F.conv(hsrc, wq, L[..., (i + 1) * f:(i + 2) * f], K3, P1, bias=bq, x_shuffle=s, act=PR,
                       act_param=cpr.weight, subpixel=F.subpixel_code(k, s, p, False, False))
            X0n = buf("X0", t + 1, h, w, 2 * f, T + 1)
            ffeat = X0n[..., f:]  # f_features = next frame's hidden state (drf_net.py:45)
            F.conv(L[..., f:], pw(fb.out_block.conv), ffeat, K1, P0, bias=fb.out_block.conv.bias, act=PR,
                   act_param=fb.out_block.prelu.weight)
            feat = F.add(X0[..., :f], ffeat, buf("feat", t, h, w, f))  # global residual skip (drf_net.py:46)
            u, hh, ww, ups_in = feat, h, w, []
            for j, (conv, st) in enumerate(self._ups()):
                nxt = buf(f"up{j}", t, hh * st, ww * st, f)
                F.conv(u, pw(conv, perm_r=st), nxt, K3, P1, bias=conv.bias, y_shuffle=st)
                ups_in.append(u)
                u, hh, ww = nxt, hh * st, ww * st
            tc = self._last_conv()
            co = self.out_channels
            if co == 1:
                y = torch.empty((b, 1, hh, ww), dtype=torch.float32, device=dev)
                F.conv(u, pw(tc), y.view(b, 1, hh, ww, 1), K3, P1, bias=tc.bias)
            else:
                tmp = torch.empty((b, 1, hh, ww, co), dtype=torch.float32, device=dev)
                y = F.from_view(F.conv(u, pw(tc), tmp, K3, P1, bias=tc.bias))
            outs.append(y)
            if tape is not None:
                recs.append(dict(xv=xv, u1=u1, X0=X0, L=L, Hc=Hc, t1s=t1s, t2s=t2s, ffeat=ffeat, ups_in=ups_in,
                                 tail_in=u))
            X0 = X0n
        if tape is not None:
            tape.update(recs=recs, shape=(b, h, w), packer=(pw, sp), slopes=self._slopes_async())
        return outs

    def _backward(self, tape: dict, gys) -> dict:
        cd = self.compute_dtype
        f, G = self.num_features, self.num_groups
        k, s, p = _PROJ[self.upscale_factor]
        b, h, w = tape["shape"]
        H, W = h * s, w * s
        pw, sp = tape["packer"]
        ib, fb = self.in_block, self.f_block
        # PReLUs with a slope <= 0 take the pre-activation backward; so does
        # every PReLU when the slopes are unknown (graph capture)
        if tape.get("slopes") is not None:
            host, ev, idx = tape["slopes"]
            ev.synchronize()
            nonpos = {k for k, (i, n) in idx.items() if bool((host[i:i + n] <= 0).any())}
        else:
            nonpos = {id(m) for m in self.modules() if isinstance(m, nn.PReLU)}
        recs = tape["recs"]
        dev = recs[0]["X0"].device
        if not isinstance(gys, (tuple, list)):
            gys = [gys]
        grads: dict = {}
        bufs: dict = {}  # id(param) -> gradient buffer (accumulated over frames)

        def new(hh, ww, c):
            return torch.empty((b, 1, hh, ww, c), dtype=cd, device=dev)

        T = len(recs)
        seq = self.SEQ_WGRAD
        seqs: dict = {}
        # Sequence buffers come in chunks of Kg frames ([r Kg, (r+1) Kg)),
        # each dropped once every run over its frames is launched (the side
        # stream keeps the storage alive through record_stream): the extra
        # memory over per-frame buffers is at most VSR_DRF_SEQ_BUDGET_GB
        # (default 16) instead of T frames of every buffer (~37 GB at cfg 3).
        Kg = T
        if seq:
            HH0, WW0 = recs[0]["tail_in"].shape[2], recs[0]["tail_in"].shape[3]
            fe = HH0 * WW0 * f  # dup{len(ups)}
            hh0, ww0 = HH0, WW0
            for _, st_ in reversed(self._ups()):
                hh0, ww0 = hh0 // st_, ww0 // st_
                fe += hh0 * ww0 * f  # dup{j}
            fe += (2 * G + 2) * h * w * f + h * w * 4 * f  # gout, dL ((G + 1) f), dt1_*, gin, du_u1
            fe += (2 * G - 1) * H * W * f  # dHc (G f), dt2_*
            frame_bytes = fe * b * torch.empty((), dtype=cd).element_size()
            budget = float(os.environ.get("VSR_DRF_SEQ_BUDGET_GB", "16")) * 2 ** 30
            Kg = max(1, min(T, int(budget // max(frame_bytes, 1))))
            if torch.cuda.is_current_stream_capturing():
                # under HIP-graph capture no chunk is freed mid-backward: a
                # block freed during capture can go to a later captured
                # allocation while the side stream's weight-gradient runs
                # still read it (record_stream does not defer it there) --
                # the captured cfg 3 step diverged from the eager one
                # (tools/diag/graph_drf_cfg3.py); the graph pool holds all T
                Kg = T
        self._seq_run_frames = Kg  # (tests / bench records)

        def sbuf(name, t, hh, ww, c):
            """frame t of a backward sequence buffer (an output gradient a
            weight gradient reads); per-frame buffers without SEQ_WGRAD"""
            if not seq:
                return new(hh, ww, c)
            r = t // Kg
            big = seqs.get((name, r))
            if big is None:
                big = seqs[(name, r)] = torch.empty((min(Kg, T - r * Kg), b, hh, ww, c), dtype=cd, device=dev)
            return big[t - r * Kg].unsqueeze(1)

        # deferred weight gradients: key -> (param, launch(x, dy, accumulate),
        # {frame: (x, dy)}, runs launched, frames per run K)
        pend: dict = {}

        run_k: dict = {}  # weight name -> frames per run (tests / bench records)
        self._seq_run_k = run_k
        pnames = {id(p_): n_ for n_, p_ in self.named_parameters()}

        def run_frames(x, dy, name="") -> int:
            """K for a weight: the run's view must keep 32-bit element offsets
            (B x the frame's span of the wider operand, per frame).  Runs
            start at every K-th frame of a sequence-buffer chunk and stop at
            its end, so K need not divide Kg (round 5 lowered K until it did:
            at cfg 3, Kg = 13 is prime and the high-res projection weights
            fell back to single-frame runs)"""
            span = max(v.stride(0) * b for v in (x, dy))
            k_ = max(1, min(Kg, (2 ** 31 - 1) // max(span, 1) - 1))
            cap = int(os.environ.get("VSR_DRF_RUN_FRAMES", "0"))  # test knob: a shorter run
            if cap > 0:
                k_ = min(k_, cap)
            run_k[name] = k_
            return k_

        def launch_runs(t):
            """frame t just finished: launch every deferred weight gradient
            whose run [t, t + K) is complete on the side stream (accumulating
            after its first run)"""
            if not seq:
                return
            r0 = (t // Kg) * Kg  # the chunk [r0, r0 + Kg) frame t belongs to
            for key, (prm, launch, frs, nrun, K) in list(pend.items()):
                if (t - r0) % K != 0:
                    continue
                t1 = min(t + K, r0 + Kg, T)
                xs = _seq_view([frs[u][0] for u in range(t, t1)])
                dys = _seq_view([frs[u][1] for u in range(t, t1)])
                if xs is not None and dys is not None:
                    self._on_wgrad_stream(lambda: launch(xs, dys, nrun > 0), xs, dys)
                    nrun += 1
                else:  # operands not in sequence buffers: per frame
                    for u in range(t, t1):
                        x_, dy_ = frs[u]
                        self._on_wgrad_stream(lambda: launch(x_, dy_, nrun > 0), x_, dy_)
                        nrun += 1
                for u in range(t, t1):
                    del frs[u]
                pend[key] = (prm, launch, frs, nrun, K)
            if t % Kg == 0:  # every run over chunk t // Kg is launched: drop its buffers
                for key in [k_ for k_ in seqs if k_[1] == t // Kg]:
                    del seqs[key]

        def gbuf(prm):
            key = id(prm)
            if key in bufs:
                return bufs[key][1], True
            g = self._grad_buffer(prm)
            bufs[key] = (prm, g)
            return g, False

        def defer(key, t, x, dy, launch, acc):
            """per frame: launch now (acc: accumulate onto the frames done so
            far); SEQ_WGRAD: record frame t's operands, launched once over
            the sequence"""
            if not seq:
                self._on_wgrad_stream(lambda: launch(x, dy, acc), x, dy)
                return
            ent = pend.get(id(key))
            if ent is None:
                ent = pend[id(key)] = (key, launch, {}, 0, run_frames(x, dy, pnames.get(id(key), "")))
            ent[2][t] = (x, dy)

        def wgrad(conv, x, dy, ksz, pad, t, **kw):
            dw, acc = gbuf(conv.weight)
            db, _ = gbuf(conv.bias)
            defer(conv.weight, t, x, dy,
                  lambda x_, dy_, acc_: F.conv_wgrad(x_, dy_, ksz, pad, dw.view(*dw.shape[:2], 1, *dw.shape[2:]), db,
                                                     accumulate=acc_, **kw), acc)

        def sp_wgrad(conv, x, dy, transposed, t):
            k_, s_, p_ = k, s, p
            cop = s_ * s_ * f if transposed else f
            cip = f if transposed else s_ * s_ * f
            dw, acc = gbuf(conv.weight)
            db, _ = gbuf(conv.bias)

            def run(x_, dy_, acc_):  # the sub-pixel wgrad and its fold
                # (persistent side-stream scratch: inside a graph capture a
                # block freed on one stream can go to the next captured
                # allocation on the other one while kernels still use it)
                tk = (cop, cip, dev)
                if tk not in self._sp_tmp:
                    self._sp_tmp[tk] = (torch.empty((cop, cip, 1, 3, 3), dtype=torch.float32, device=dev),
                                        torch.empty(cop, dtype=torch.float32, device=dev))
                dweq, dbeq = self._sp_tmp[tk]
                spc = F.subpixel_code(k_, s_, p_, transposed, False)
                if transposed:
                    F.conv_wgrad(x_, dy_, K3, P1, dweq, dbeq, dy_shuffle=s_, subpixel=spc)
                else:
                    F.conv_wgrad(x_, dy_, K3, P1, dweq, dbeq, x_shuffle=s_, subpixel=spc)
                F.subpixel_wgrad_fold(dweq, dbeq, dw, db, k_, s_, p_, transposed, accumulate=acc_)

            defer(conv.weight, t, x, dy, run, acc)

        # PReLU slope gradients, deferred: every PReLU backward call of frame
        # t leaves its partials in slot t of its PReLU's zero-filled region;
        # one fixed-order sum per PReLU after the loop (12 launches per step
        # instead of one final per call, 540 at cfg 3)
        S = F.slope_slot_doubles()
        regions: dict = {}  # id(prelu) -> (prelu, (T, S) float64, frames taken)
        cur = [T - 1]

        # Inside a graph capture the slope gradients are not deferred: with
        # the slot regions the captured step's slope gradients come out wrong
        # while every other gradient stays bitwise equal to the eager step's
        # (tools/diag/graph_drf_grads.py; persistent slot regions, persistent
        # side-stream scratch and kept workspaces did not change it: cause
        # open) -- the per-call finals are what the captured-vs-eager test
        # holds equal
        defer_slopes = self.DEFER_SLOPES and not torch.cuda.is_current_stream_capturing()

        def slot_row(pr):
            reg = regions.get(id(pr))
            if reg is None:
                reg = regions[id(pr)] = (pr, torch.zeros((T, S), dtype=torch.float64, device=dev), set())
            if cur[0] in reg[2]:
                raise RuntimeError("DRF backward: two slope-gradient calls of one PReLU in one frame")
            reg[2].add(cur[0])
            return reg[1][cur[0]]

        def slot(pr):
            """(da, accumulate_da, slot) of a PReLU backward call: deferred,
            the call's slot row; else its slope gradient buffer"""
            if defer_slopes:
                return None, False, slot_row(pr)
            da, acc = gbuf(pr.weight)
            return da, acc, None

        def fuse(pr, call) -> bool:
            """the PReLU pr's backward fused into its gradient's last producer:
            call(slot) -> launched (F.conv_prelu_bwd); never for a slope <= 0
            (the fused epilogues read the PReLU output)"""
            if id(pr) in nonpos or not self.FUSE_SLICES or not defer_slopes:
                return False
            if call(slot_row(pr)):
                return True
            regions[id(pr)][2].discard(cur[0])  # nothing launched: the slot stays free (and zero)
            return False

        def prelu(y, dy, pr, out, dy2=None, pre=None):
            """PReLU backward from its output y; for a slope <= 0 from the
            pre-activation that pre() recomputes from the tape (the producing
            conv without its activation), as nn.PReLU does (drf_net.py:55-58)"""
            da_, acc_, sl_ = slot(pr)
            if id(pr) in nonpos:
                return F.prelu_bwd(pre(), dy, pr.weight, out, da_, acc_, dy2=dy2, pre=True, slot=sl_)
            return F.prelu_bwd(y, dy, pr.weight, out, da_, acc_, dy2=dy2, slot=sl_)

        co = self.out_channels
        HH, WW = recs[0]["tail_in"].shape[2], recs[0]["tail_in"].shape[3]
        gfull = [gys[t] if t < len(gys) and gys[t] is not None else
                 torch.zeros((b, co, HH, WW), dtype=torch.float32, device=dev) for t in range(T)]
        GV = F.to_view(torch.cat([g_.float() for g_ in gfull]), cd, cpad=8)[..., :co]  # (T*b, 1, HH, WW, co)
        d_hidden = None  # grad of the previous frame's f_features (X0_t[..., f:])
        for t in range(T - 1, -1, -1):
            cur[0] = t
            rc = recs[t]
            u = rc["tail_in"]
            hh, ww = u.shape[2], u.shape[3]
            g = GV[t * b:(t + 1) * b]
            tc = self._last_conv()
            wgrad(tc, u, g, K3, P1, t)
            ups = list(zip(self._ups(), rc["ups_in"]))
            du = F.conv(g, pw(tc, 1), sbuf(f"dup{len(ups)}", t, hh, ww, f), K3, P1)
            for j in range(len(ups) - 1, -1, -1):
                (conv, st), uin = ups[j]
                wgrad(conv, uin, du, K3, P1, t, perm_r=st, dy_shuffle=st)
                hh, ww = hh // st, ww // st
                du = F.conv(du, pw(conv, 1, perm_r=st), sbuf(f"dup{j}", t, hh, ww, f), K3, P1, x_shuffle=st)
            gfeat = du  # grad of features = in_features + f_features
            L, Hc, X0 = rc["L"], rc["Hc"], rc["X0"]
            # f_block out: f_features feeds the skip and the next frame's hidden state
            gout = prelu(rc["ffeat"], gfeat, fb.out_block.prelu, sbuf("gout", t, h, w, f), dy2=d_hidden,
                         pre=lambda: F.conv(L[..., f:], pw(fb.out_block.conv), new(h, w, f), K1, P0,
                                            bias=fb.out_block.conv.bias))
            wgrad(fb.out_block.conv, L[..., f:], gout, K1, P0, t)
            # Concat gradients without zero fills (the high-res one is 0.5 GB
            # per frame at cfg 3): the first contributor to a slice writes it,
            # later ones accumulate.  dL[..., f:] is first written by the
            # out_block's data gradient; dHc (every slice) by the last group's
            # 1x1 down-projection gradient (group 0's strided conv when G = 1);
            # dL[..., :f] has mixed first contributors and is zeroed.
            # The concat gradients are sequence buffers too: each PReLU
            # backward over a slice runs in place, fused into the slice's last
            # producer where it can (the slice is the producer's tail channels,
            # c_lo), and the weight gradients read the slices.
            dL = sbuf("dL", t, h, w, (G + 1) * f)
            dL[..., :f].zero_()
            dHc = sbuf("dHc", t, H, W, G * f)
            done = set()  # slices whose PReLU backward ran fused: ("l", i) / ("h", i) / "g0"

            def dnpr(i_):  # the PReLU after down projection i_ (lr_{i_+1})
                return fb.down_blocks[i_].prelu if i_ == 0 else fb.down_blocks[i_].prelu2

            def uppr(i_):  # the PReLU after up projection i_ (hr_{i_})
                return fb.up_blocks[i_].prelu if i_ == 0 else fb.up_blocks[i_].prelu2

            wo = pw(fb.out_block.conv, 1)
            if fuse(dnpr(G - 1), lambda sl_: F.conv_prelu_bwd(
                    gout, wo, dL[..., f:], K1, P0, L[..., f:], dnpr(G - 1).weight, None, False, c_lo=(G - 1) * f, slot=sl_)):
                done.add(("l", G - 1))
            else:
                F.conv(gout, wo, dL[..., f:], K1, P0)
            for i in range(G - 1, -1, -1):
                up, dn = fb.up_blocks[i], fb.down_blocks[i]
                # down projection -> lr_{i+1} = L[..., (i+1)f:(i+2)f]
                cv, cpr = (dn.conv, dn.prelu) if i == 0 else (dn.conv2, dn.prelu2)
                sl = slice((i + 1) * f, (i + 2) * f)
                hsrc = Hc[..., :f] if i == 0 else rc["t2s"][i]
                gl = dL[..., sl]
                if ("l", i) not in done:
                    prelu(L[..., sl], gl, cpr, gl,
                          pre=lambda cv=cv, hsrc=hsrc: F.conv(
                              hsrc, sp(cv, False)[0], new(h, w, f), K3, P1, bias=sp(cv, False)[1], x_shuffle=s,
                              subpixel=F.subpixel_code(k, s, p, False, False)))
                sp_wgrad(cv, hsrc, gl, False, t)
                wq1, _ = sp(cv, False, 1)
                spc = F.subpixel_code(k, s, p, False, True)
                if i == 0:
                    if fuse(uppr(0), lambda sl_: F.conv_prelu_bwd(
                            gl, wq1, dHc[..., :f], K3, P1, Hc[..., :f], uppr(0).weight, None, False, y_shuffle=s,
                            subpixel=spc, accumulate=G > 1, slot=sl_)):
                        done.add(("h", 0))
                    else:
                        F.conv(gl, wq1, dHc[..., :f], K3, P1, y_shuffle=s, accumulate=G > 1, subpixel=spc)
                else:
                    dt2 = sbuf(f"dt2_{i}", t, H, W, f)
                    da2, acc2, sl2 = slot(dn.prelu1)
                    if id(dn.prelu1) in nonpos:  # slope <= 0: from the recomputed pre-activation
                        F.conv(gl, wq1, dt2, K3, P1, y_shuffle=s, subpixel=spc)
                        x2 = F.conv(Hc[..., :(i + 1) * f], pw(dn.conv1), new(H, W, f), K1, P0, bias=dn.conv1.bias)
                        F.prelu_bwd(x2, dt2, dn.prelu1.weight, dt2, da2, acc2, pre=True, slot=sl2)
                    elif not F.conv_prelu_bwd(gl, wq1, dt2, K3, P1, rc["t2s"][i], dn.prelu1.weight, da2, acc2,
                                              y_shuffle=s, subpixel=spc, slot=sl2):
                        F.conv(gl, wq1, dt2, K3, P1, y_shuffle=s, subpixel=spc)
                        F.prelu_bwd(rc["t2s"][i], dt2, dn.prelu1.weight, dt2, da2, acc2, slot=sl2)
                    wgrad(dn.conv1, Hc[..., :(i + 1) * f], dt2, K1, P0, t)
                    wd1 = pw(dn.conv1, 1)
                    if fuse(uppr(i), lambda sl_: F.conv_prelu_bwd(
                            dt2, wd1, dHc[..., :(i + 1) * f], K1, P0, Hc[..., :(i + 1) * f], uppr(i).weight, None, False,
                            accumulate=i != G - 1, c_lo=i * f, slot=sl_)):
                        done.add(("h", i))
                    else:
                        F.conv(dt2, wd1, dHc[..., :(i + 1) * f], K1, P0, accumulate=i != G - 1)
                # up projection -> hr_i = Hc[..., i f:(i+1) f]
                dec, dpr = (up.deconv, up.prelu) if i == 0 else (up.deconv2, up.prelu2)
                sh = slice(i * f, (i + 1) * f)
                src = L[..., :f] if i == 0 else rc["t1s"][i]
                gh = dHc[..., sh]
                if ("h", i) not in done:
                    prelu(Hc[..., sh], gh, dpr, gh,
                          pre=lambda dec=dec, src=src: F.conv(
                              src, sp(dec, True)[0], new(H, W, f), K3, P1, bias=sp(dec, True)[1], bias_r=1,
                              y_shuffle=s, subpixel=F.subpixel_code(k, s, p, True, False)))
                sp_wgrad(dec, src, gh, True, t)
                wq1, _ = sp(dec, True, 1)
                spc = F.subpixel_code(k, s, p, True, True)
                if i == 0:
                    ipr = fb.in_block.prelu
                    if fuse(ipr, lambda sl_: F.conv_prelu_bwd(
                            gh, wq1, dL[..., :f], K3, P1, L[..., :f], ipr.weight, None, False, x_shuffle=s,
                            subpixel=spc, accumulate=True, slot=sl_)):
                        done.add("g0")
                    else:
                        F.conv(gh, wq1, dL[..., :f], K3, P1, x_shuffle=s, accumulate=True, subpixel=spc)
                else:
                    dt1 = sbuf(f"dt1_{i}", t, h, w, f)
                    da1, acc1, sl1 = slot(up.prelu1)
                    if id(up.prelu1) in nonpos:  # slope <= 0: from the recomputed pre-activation
                        F.conv(gh, wq1, dt1, K3, P1, x_shuffle=s, subpixel=spc)
                        x1 = F.conv(L[..., :(i + 1) * f], pw(up.conv1), new(h, w, f), K1, P0, bias=up.conv1.bias)
                        F.prelu_bwd(x1, dt1, up.prelu1.weight, dt1, da1, acc1, pre=True, slot=sl1)
                    elif not F.conv_prelu_bwd(gh, wq1, dt1, K3, P1, rc["t1s"][i], up.prelu1.weight, da1, acc1,
                                              x_shuffle=s, subpixel=spc, slot=sl1):
                        F.conv(gh, wq1, dt1, K3, P1, x_shuffle=s, subpixel=spc)
                        F.prelu_bwd(rc["t1s"][i], dt1, up.prelu1.weight, dt1, da1, acc1, slot=sl1)
                    wgrad(up.conv1, L[..., :(i + 1) * f], dt1, K1, P0, t)
                    wu1 = pw(up.conv1, 1)
                    # the last contribution to lr_i's gradient (slice i of dL)
                    if fuse(dnpr(i - 1), lambda sl_: F.conv_prelu_bwd(
                            dt1, wu1, dL[..., :(i + 1) * f], K1, P0, L[..., :(i + 1) * f], dnpr(i - 1).weight, None,
                            False, accumulate=True, c_lo=i * f, slot=sl_)):
                        done.add(("l", i - 1))
                    else:
                        F.conv(dt1, wu1, dL[..., :(i + 1) * f], K1, P0, accumulate=True)
            g0 = dL[..., :f]
            if "g0" not in done:
                prelu(L[..., :f], g0, fb.in_block.prelu, g0,
                      pre=lambda: F.conv(X0, pw(fb.in_block.conv), new(h, w, f), K1, P0, bias=fb.in_block.conv.bias))
            wgrad(fb.in_block.conv, X0, g0, K1, P0, t)
            dX0 = F.conv(g0, pw(fb.in_block.conv, 1), new(h, w, 2 * f), K1, P0)
            if t == 0:  # the first hidden state is in_features itself
                F.add(dX0[..., :f], dX0[..., f:], dX0[..., :f])
                d_hidden = None
            else:
                d_hidden = dX0[..., f:]
            gin = prelu(X0[..., :f], gfeat, ib.prelu2, sbuf("gin", t, h, w, f), dy2=dX0[..., :f],
                        pre=lambda: F.conv(rc["u1"], pw(ib.conv2), new(h, w, f), K1, P0, bias=ib.conv2.bias))
            wgrad(ib.conv2, rc["u1"], gin, K1, P0, t)
            du1 = sbuf("du_u1", t, h, w, 4 * f)
            wi2 = pw(ib.conv2, 1)
            if not fuse(ib.prelu1, lambda sl_: F.conv_prelu_bwd(gin, wi2, du1, K1, P0, rc["u1"], ib.prelu1.weight,
                                                                    None, False, slot=sl_)):
                F.conv(gin, wi2, du1, K1, P0)
                prelu(rc["u1"], du1, ib.prelu1, du1,
                      pre=lambda: F.conv(rc["xv"], pw(ib.conv1), new(h, w, 4 * f), K3, P1, bias=ib.conv1.bias))
            wgrad(ib.conv1, rc["xv"], du1, K3, P1, t)
            launch_runs(t)
        for pr, reg, _ in regions.values():  # the slope gradients, one fixed-order sum per PReLU
            da, acc = gbuf(pr.weight)
            F.slope_final_sum(reg, pr.weight, da, acc, id(pr) in nonpos)
        for prm, g in bufs.values():
            self._grad_done(grads, prm, g)
        return grads


class DRFNet(_DRFBase):
    """Deep Recurrent Feedback Network, VSR (drf_net.py:8-49): list of T (B,C,h,w) -> list of T (B,C,rh,rw)."""

    def _frames(self, inputs):
        return list(inputs)

    def forward(self, inputs):
        return super().forward(list(inputs))


class DRFSISRNet(_DRFBase):
    """DRFN for SISR (drf_sisr_net.py:8-50): (B,C,h,w) -> list of num_steps (B,C,rh,rw)."""

    def __init__(self, in_channels, out_channels, num_steps, num_features, num_groups, upscale_factor):
        super().__init__(in_channels, out_channels, num_features, num_groups, upscale_factor)
        self.num_steps = num_steps

    def _frames(self, inputs):
        return [inputs] * self.num_steps
