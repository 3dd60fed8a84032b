"""Data-parallel gradient synchronisation over RCCL (torch.distributed 'nccl').

The reference is single-device (main.py:38); the build shards minibatches
across the GPUs of one node (one process per GPU).  GradSync owns flat fp32
communication buckets: every parameter's .grad is a view into one, the
hand-written backward passes write gradients straight into those views, and a
bucket's all-reduce is launched (async, on RCCL's stream) the moment its last
gradient is written — so communication overlaps the rest of backward instead
of running after it.  Buckets follow the backward order (reverse registration)
and are ~4 MiB: the models have 6-10 MB of fp32 gradients, i.e. 2-3 buckets,
each a single ring all-reduce over xGMI.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


class GradSync:
    def __init__(self, net, world: int, bucket_bytes: int = 4 << 20):
        self.world = world
        self.net = net
        params = [p for p in net.parameters() if p.requires_grad]
        order = list(reversed(params))
        self.buckets: list[list[torch.Tensor]] = [[]]
        size = 0
        for p in order:
            if size >= bucket_bytes:
                self.buckets.append([])
                size = 0
            self.buckets[-1].append(p)
            size += p.numel() * 4
        dev = params[0].device
        self.flat: list[torch.Tensor] = []
        self._view: dict[int, torch.Tensor] = {}
        self._bucket_of: dict[int, int] = {}
        for b, ps in enumerate(self.buckets):
            buf = torch.zeros(sum(p.numel() for p in ps), dtype=torch.float32, device=dev)
            self.flat.append(buf)
            off = 0
            for p in ps:
                v = buf[off:off + p.numel()].view_as(p)
                self._view[id(p)] = v
                self._bucket_of[id(p)] = b
                off += p.numel()
        self._params = params
        self._reset()
        net._grad_sink = self
        self._avg = hasattr(dist.ReduceOp, "AVG")
        self._attach()

    def _reset(self):
        self._remaining = [len(ps) for ps in self.buckets]
        self._handles: list = [None] * len(self.buckets)

    def _attach(self):
        for p in self._params:
            p.grad = self._view[id(p)]

    def view(self, p: torch.Tensor) -> torch.Tensor:
        return self._view[id(p)]

    def _launch(self, b: int):
        op = dist.ReduceOp.AVG if self._avg else dist.ReduceOp.SUM
        self._handles[b] = dist.all_reduce(self.flat[b], op=op, async_op=True)

    def ready(self, p: torch.Tensor) -> None:
        b = self._bucket_of[id(p)]
        self._remaining[b] -= 1
        if self._remaining[b] == 0:
            join = getattr(self.net, "_join_wgrad", None)
            if join is not None:
                join()  # the bucket's weight gradients may still run on the side stream
            self._launch(b)

    def finish(self) -> None:
        """Wait for every bucket (launching any not yet complete), average, and
        re-attach .grad views (zero_grad(set_to_none=True) may have dropped them)."""
        join = getattr(self.net, "_join_wgrad", None)
        if join is not None:
            join()
        for b, h in enumerate(self._handles):
            if h is None:
                self._launch(b)
        unscale = getattr(self.net, "_grad_unscale", 1.0)  # fp16 loss scale (BaseNet._loss_scale)
        for b, h in enumerate(self._handles):
            self._handles[b].wait()
        f = unscale if self._avg else unscale / self.world
        if getattr(self.net, "compute_dtype", None) == torch.float16:
            # fp16: unscale and flag inf / NaN in one pass over the buckets; an
            # overflow on any rank reaches every rank through the all-reduce,
            # so every rank skips the same step (BaseNet.step_ok)
            from .nets.base_net import unscale_check
            self.net._found_inf = unscale_check(self.flat, f)
        elif f != 1.0:
            for buf in self.flat:
                buf.mul_(f)
        self._reset()
        self._attach()

    def broadcast_params(self, src: int = 0) -> None:
        """Start from identical weights on every rank."""
        for p in self._params:
            dist.broadcast(p.data, src)
        for b in self.net.buffers():
            dist.broadcast(b.data, src)


class SyncBNAllReduce:
    """SyncBatchNorm hook for the fused BatchNorm3d of DUFNet (duf_net.py:116,
    198,201,209,212 in the reference; train-mode batch statistics couple the
    samples of a batch, so data-parallel ranks must share them).

    ``hook(sums)`` sums the per-channel (sum, sumsq) -- or, in backward,
    (sum_dy, sum_dy_xhat) -- over every rank in place (one small all-reduce
    per BN layer, at most 2 x 256 floats).  The global voxel count of a layer
    is its depth times the sum over ranks of N*H*W of the step's input
    (ranks may hold batches of different sizes: uncropped slices, a last
    partial batch): ``global_count(local, device)`` all-reduces that once per
    forward into a float64 DEVICE scalar, stream-ordered, and never reads it
    on the host: the BN kernels take the count from device memory
    (vsrk_bn_finalize_dcount) and the backward divides its all-reduced sums
    by the count on the device (duf_net._ScaledWork).  So a DUF training step
    has no host synchronisation on the count at any step, whatever the
    ranks' batch shapes."""

    def __init__(self, group=None):
        self.group = group
        self.world = dist.get_world_size(group)

    def __call__(self, t: torch.Tensor) -> None:
        dist.all_reduce(t, group=self.group)

    def start(self, t: torch.Tensor):
        """Asynchronous form: returns the work handle; ``handle.wait()`` makes the
        current stream wait for the sum (no host block on RCCL), so independent
        kernels queued in between (a weight gradient) hide the collective."""
        return dist.all_reduce(t, group=self.group, async_op=True)

    def global_count(self, local: int, device) -> torch.Tensor:
        """Sum of `local` over the ranks as a float64 scalar on `device`
        (exact up to 2^53).  RCCL: an async all-reduce whose wait() only
        orders the current stream -- no host read.  gloo (CPU tensors) blocks
        the host, as every gloo collective does."""
        if dist.get_backend(self.group) == "nccl":
            t = torch.full((1,), float(local), dtype=torch.float64, device=device)
            dist.all_reduce(t, group=self.group, async_op=True).wait()
            return t
        t = torch.full((1,), float(local), dtype=torch.float64)
        dist.all_reduce(t, group=self.group)
        return t.to(device)


def enable_sync_bn(net, group=None) -> bool:
    """Share BatchNorm batch statistics across the data-parallel ranks (a no-op
    for nets without BatchNorm).  Returns whether the net has the hook."""
    if not hasattr(net, "bn_allreduce"):
        return False
    net.bn_allreduce = SyncBNAllReduce(group) if dist.is_initialized() and dist.get_world_size(group) > 1 else None
    return True
