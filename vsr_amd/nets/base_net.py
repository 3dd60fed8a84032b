"""Base class of the fused generators.

Mirrors src/model/nets/base_net.py:5-13 (BaseNet.__repr__ reports trainable
parameters and fp32 size) and adds the bridge between torch autograd and the
hand-written backward passes: a net's forward runs HIP kernels directly and
records a tape; one autograd.Function replays the tape in reverse, writing
every parameter gradient with the deterministic wgrad kernels.
"""
from __future__ import annotations

import os

import torch
import torch.nn as nn

from .. import functional as F

_COMPUTE_DTYPES = {"bf16": torch.bfloat16, "bfloat16": torch.bfloat16, "fp16": torch.float16,
                   "float16": torch.float16, "fp32": torch.float32, "float32": torch.float32}


class BaseNet(nn.Module):
    """Base of every vsr_amd generator (reference: base_net.py:5-13)."""

    # Side-stream weight gradients (see _on_wgrad_stream), measured on one
    # MI355X at cfg 2 / 3 (profiles/r2e_side_stream_ab.txt): DRF -4.5 %
    # (its per-frame convs leave CUs idle), EDSR -2.3 % but every conv's own
    # launch time (the roofline) stretched by the sharing, DUF 86 -> 255 ms
    # (the persistent one-workgroup-per-CU conv grids stall behind resident
    # wgrad workgroups).  On for DRF only.
    _OVERLAP_WGRAD = False

    def __init__(self):
        super().__init__()
        self.compute_dtype = torch.bfloat16
        self._grad_sink = None  # vsr_amd.ddp.GradSync when data-parallel
        # fp16 loss scale: None = dynamic (see _loss_scale / step_ok), else a fixed float
        self.loss_scale = None
        self._scale = None       # current dynamic fp16 scale (set at the first fp16 backward)
        self._good_steps = 0     # finite steps since the last change of _scale
        self.scale_growth_interval = 2000
        self._found_inf = None   # device flag: the last fp16 backward produced an inf/NaN gradient
        # weight gradients on a second stream, overlapped with the data-gradient
        # chain: per net class (_OVERLAP_WGRAD), VSR_OVERLAP_WGRAD=0/1 overrides
        env = os.environ.get("VSR_OVERLAP_WGRAD")
        self.overlap_wgrad = self._OVERLAP_WGRAD if env is None else env != "0"
        self._side = None
        self._side_used = False
        self._side_keep: list = []  # operands of side-stream launches captured into a graph (see _on_wgrad_stream)
        self._packers: dict = {}

    # -- gradient plumbing used by the subclasses' backward passes ----------
    def _grad_buffer(self, p: torch.Tensor) -> torch.Tensor:
        """fp32 tensor the wgrad kernel writes p's gradient into (a slice of a
        communication bucket when data-parallel)."""
        if self._grad_sink is not None:
            return self._grad_sink.view(p)
        return torch.empty_like(p, dtype=torch.float32)

    def _grad_done(self, grads: dict, p: torch.Tensor, g: torch.Tensor) -> None:
        """Record p's finished gradient; with a sink this may launch its bucket's
        all-reduce right away (overlapping the rest of the backward pass)."""
        if self._grad_sink is not None:
            self._grad_sink.ready(p)
        else:
            grads[id(p)] = g

    # -- weight gradients on a side stream ----------------------------------
    # A weight gradient is a leaf of the backward graph: nothing in the step
    # reads it before the optimizer.  Launched on a second stream (after the
    # producer of its output gradient on the caller's stream), it overlaps the
    # data-gradient chain: an MFMA-bound wgrad beside an HBM-bound BN / PReLU
    # pass, or beside a conv whose grid leaves CUs idle (DRF's per-frame
    # 4 x 128 x 128 launches).  Same kernels, same per-stream order:
    # results stay bitwise reproducible.
    def _on_wgrad_stream(self, fn, *reads):
        """Run fn (a weight-gradient launch) on the side stream after all work
        queued so far on the current stream; `reads` are the tensors it reads
        (kept alive for the allocator until the side stream is done)."""
        if not self.overlap_wgrad:
            return fn()
        main = torch.cuda.current_stream()
        if self._side is None or self._side.device != main.device:
            self._side = torch.cuda.Stream(main.device)
        self._side.wait_stream(main)
        with torch.cuda.stream(self._side):
            out = fn()
        for t in reads:
            t.record_stream(self._side)
        if torch.cuda.is_current_stream_capturing():
            # record_stream does not defer a free inside graph capture: a
            # tensor dropped now could go to a later captured allocation on
            # the main stream while the side stream still reads it.  Hold
            # every operand until _join_wgrad orders the main stream after
            # the side stream.
            self._side_keep.extend(reads)
        self._side_used = True
        return out

    def _pack_weights(self, specs) -> dict:
        """Pack every (weight, mode, perm_r) of specs in one launch (persistent
        buffers, see functional.WeightPacker) -> {(id(weight), mode, perm_r): packed}."""
        cd = self.compute_dtype
        key = (cd, tuple((id(w), m, r) for w, m, r in specs))
        pk = self._packers.get(key)
        if pk is None:
            pk = self._packers[key] = F.WeightPacker(specs, cd)
        return pk.run()

    def _join_wgrad(self) -> None:
        """Make the current stream wait for every side-stream weight gradient
        (before a gradient is consumed, or before a buffer a weight gradient
        reads is overwritten in place)."""
        if self._side_used:
            torch.cuda.current_stream().wait_stream(self._side)
            self._side_used = False
        self._side_keep.clear()

    def set_precision(self, precision: str, loss_scale: float | None = None) -> "BaseNet":
        """'bf16' or 'fp16' (16-bit activations and data gradients, fp32 master
        weights, fp32 accumulation and fp32 weight gradients) or 'fp32'.  fp16
        backward passes run loss-scaled (see _loss_scale); loss_scale fixes
        the factor instead."""
        self.compute_dtype = _COMPUTE_DTYPES[precision]
        self.loss_scale = loss_scale
        self._scale = None
        self._good_steps = 0
        self._found_inf = None
        return self

    def _loss_scale(self, grads) -> float:
        """Factor the output gradient is multiplied by before an fp16 backward
        (and every parameter gradient divided by after it), as
        torch.cuda.amp.GradScaler does.  The reference's losses are means over
        the output (losses.py:5-34, nn.L1Loss/MSELoss), so the output gradient
        is O(1/N) for N output elements: below fp16's normal range (6.1e-5) at
        N > 16k, and the data gradients of early layers sit further down in
        fp16's subnormals, where fewer significant bits remain.  The dynamic
        scale starts at 2^floor(log2 N) (output gradients in [1, 2)); step_ok()
        halves it after an overflow and doubles it after
        scale_growth_interval finite steps.  bf16 / fp32: 1."""
        if self.compute_dtype != torch.float16:
            return 1.0
        if self.loss_scale is not None:
            return float(self.loss_scale)
        if self._scale is None:
            gs = grads if isinstance(grads, (tuple, list)) else (grads,)
            n = sum(g.numel() for g in gs if g is not None)
            self._scale = float(2 ** max(0, max(n, 1).bit_length() - 1))
        return self._scale

    def step_ok(self) -> bool:
        """GradScaler.step/update for the fp16 path: False when the last
        backward produced an inf or NaN gradient (the caller then skips
        optimizer.step(), so Adam's state never sees it), and the dynamic scale
        backs off by half; after scale_growth_interval finite steps it grows by
        2.  One host read of a device flag per fp16 step; True without one
        (bf16 / fp32, or no backward since the last call)."""
        f = self._found_inf
        if f is None:
            return True
        self._found_inf = None
        found = bool(f.item())
        if self.loss_scale is None and self._scale is not None:
            if found:
                # no floor (GradScaler): the check below keeps running at any scale
                self._scale = self._scale * 0.5
                self._good_steps = 0
            else:
                self._good_steps += 1
                if self._good_steps >= self.scale_growth_interval:
                    self._scale *= 2.0
                    self._good_steps = 0
        return not found

    def __repr__(self):
        n = sum(p.numel() for p in self.parameters() if p.requires_grad)
        return super().__repr__() + f"\nTrainable parameters: {n / 1e6} M\nMemory usage: {(n * 4) / (1 << 20)} MB"

    # -- subclasses implement these two ------------------------------------
    def _run(self, inputs, tape: dict | None):
        """Forward with HIP kernels; when tape is a dict, save what backward needs."""
        raise NotImplementedError

    def _backward(self, tape: dict, grads) -> dict:
        """Reverse pass: returns {id(parameter): gradient} (missing = no grad)."""
        raise NotImplementedError

    # ----------------------------------------------------------------------
    def forward(self, inputs):
        params = [p for p in self.parameters()]
        if torch.is_grad_enabled() and any(p.requires_grad for p in params):
            out = _TapeFunction.apply(self, inputs, *params)
            return list(out) if isinstance(out, tuple) and self._returns_list() else out
        with torch.no_grad():
            return self._run(inputs, None)

    def _returns_list(self) -> bool:
        return False


def unscale_check(tensors, inv_scale: float) -> torch.Tensor:
    """t *= inv_scale for every fp32 tensor; returns a device flag (float32 [1])
    that is nonzero when any element was inf or NaN (torch's GradScaler
    kernel, _amp_foreach_non_finite_check_and_unscale_)."""
    dev = tensors[0].device
    found = torch.zeros(1, dtype=torch.float32, device=dev)
    inv = torch.full((1,), inv_scale, dtype=torch.float32, device=dev)
    torch._amp_foreach_non_finite_check_and_unscale_(tensors, found, inv)
    return found


class _TapeFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, net, inputs, *params):
        tape: dict = {}
        out = net._run(inputs, tape)
        ctx.net = net
        ctx.tape = tape
        ctx.params = params
        if isinstance(out, list):
            return tuple(out)
        return out

    @staticmethod
    def backward(ctx, *grads):
        net = ctx.net
        scale = net._loss_scale(grads)
        if scale != 1.0:
            grads = tuple(g * scale if g is not None else None for g in grads)
        net._grad_unscale = 1.0 / scale
        g = net._backward(ctx.tape, grads if len(grads) > 1 else grads[0])
        net._join_wgrad()
        ctx.tape = None
        if net.compute_dtype == torch.float16 and net._grad_sink is None:
            # unscale every parameter gradient and flag any inf / NaN (one fused
            # pass; the data-parallel path does this on its buckets in
            # GradSync.finish).  fp16 always checks, at scale 1 too: an
            # overflow is not a property of the scale alone
            net._found_inf = unscale_check([t for t in g.values()], 1.0 / scale)
        return (None, None, *[g.get(id(p)) for p in ctx.params])
