"""Base class of the fused generators.

Mirrors src/model/nets/base_net.py:5-13 (BaseNet.__repr__ reports trainable
parameters and fp32 size) and adds the bridge between torch autograd and the
hand-written backward passes: a net's forward runs HIP kernels directly and
records a tape; one autograd.Function replays the tape in reverse, writing
every parameter gradient with the deterministic wgrad kernels.
"""
from __future__ import annotations

import torch
import torch.nn as nn

_COMPUTE_DTYPES = {"bf16": torch.bfloat16, "bfloat16": torch.bfloat16, "fp32": torch.float32,
                   "float32": torch.float32}


class BaseNet(nn.Module):
    """Base of every vsr_amd generator (reference: base_net.py:5-13)."""

    def __init__(self):
        super().__init__()
        self.compute_dtype = torch.bfloat16
        self._grad_sink = None  # vsr_amd.ddp.GradSync when data-parallel

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

    def set_precision(self, precision: str) -> "BaseNet":
        """'bf16' (bf16 activations, fp32 master weights/accumulation) or 'fp32'."""
        self.compute_dtype = _COMPUTE_DTYPES[precision]
        return self

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
        g = ctx.net._backward(ctx.tape, grads if len(grads) > 1 else grads[0])
        ctx.tape = None
        return (None, None, *[g.get(id(p)) for p in ctx.params])
