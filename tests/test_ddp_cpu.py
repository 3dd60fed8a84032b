"""GradSync (bucketed, backward-overlapped gradient all-reduce) on the gloo
backend with world_size 2: every rank ends with the average gradient, buckets
launch as soon as their last gradient is ready, and .grad views survive
zero_grad(set_to_none=True)."""
import os
import socket

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from vsr_amd.ddp import GradSync


class _Net(torch.nn.Module):
    def __init__(self):
        super().__init__()
        self.a = torch.nn.Linear(64, 64)
        self.b = torch.nn.Linear(64, 300)
        self.c = torch.nn.Linear(300, 8)
        self._grad_sink = None


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(0)
    net = _Net()
    sync = GradSync(net, world, bucket_bytes=64 * 64 * 4)
    assert len(sync.buckets) >= 2
    for step in range(2):
        for p in net.parameters():
            p.grad = None  # what zero_grad(set_to_none=True) does
        # "backward": write rank-dependent grads in reverse order, mark ready
        for i, p in enumerate(reversed(list(net.parameters()))):
            sync.view(p).fill_(float(rank + 1 + i + step))
            sync.ready(p)
        sync.finish()
        for i, p in enumerate(reversed(list(net.parameters()))):
            exp = (1 + 2) / 2 + i + step
            assert p.grad is sync.view(p)
            assert torch.allclose(p.grad, torch.full_like(p.grad, exp)), (rank, i)
    q.put(rank)
    dist.destroy_process_group()


def test_gradsync_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    assert sorted([q.get(timeout=5) for _ in range(2)]) == [0, 1]
