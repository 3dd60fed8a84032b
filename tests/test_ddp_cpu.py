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


def test_syncbn_global_count_has_no_host_read(monkeypatch):
    """On RCCL the SyncBN global voxel count is an async all-reduce into a
    device scalar that the BN kernels read (vsrk_bn_finalize_dcount): no
    .item() and no blocking collective in any DUF step, the first included
    (it used to block the host every training forward)."""
    from vsr_amd import ddp

    calls = []

    class _Work:
        def wait(self):
            calls.append("wait")

    def fake_all_reduce(t, group=None, async_op=False, op=None):
        calls.append(("all_reduce", async_op))
        t.mul_(2)  # two ranks holding the same count
        return _Work() if async_op else None

    monkeypatch.setattr(dist, "get_world_size", lambda group=None: 2)
    monkeypatch.setattr(dist, "get_backend", lambda group=None: "nccl")
    monkeypatch.setattr(dist, "all_reduce", fake_all_reduce)

    def no_item(self):
        raise AssertionError("host read of the SyncBN count")

    hook = ddp.SyncBNAllReduce()
    monkeypatch.setattr(torch.Tensor, "item", no_item)
    for step in range(2):
        calls.clear()
        c = hook.global_count(4 * 128 * 128, "cpu")
        assert calls == [("all_reduce", True), "wait"], calls
        assert c.dtype == torch.float64 and c.shape == (1,)
    monkeypatch.undo()
    assert c.item() == 2 * 4 * 128 * 128


def _count_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from vsr_amd.ddp import SyncBNAllReduce
    c = SyncBNAllReduce().global_count(3 if rank == 0 else 1, "cpu")
    q.put((rank, float(c[0])))
    dist.destroy_process_group()


def test_syncbn_global_count_uneven_gloo():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_count_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=60) for _ in range(2))
    for p in procs:
        p.join(30)
        assert p.exitcode == 0
    assert got == {0: 4.0, 1: 4.0}


def test_scaled_work_divides_once_in_double():
    """the SyncBN backward sums are divided by the global count,
    formed in double, exactly once however often wait() is called."""
    from vsr_amd.nets.duf_net import _ScaledWork

    class _Done:
        def wait(self):
            pass

    red = torch.tensor([[3.0, 6.0], [9.0, 12.0]])
    w = _ScaledWork(_Done(), red, torch.tensor(3.0, dtype=torch.float64), 1.0 / 3.0)
    w.wait()
    w.wait()
    assert torch.equal(red, torch.tensor([[3.0, 6.0], [9.0, 12.0]]) / torch.tensor(1.0))
