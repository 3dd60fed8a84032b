"""vsr_amd.data.Dataloader: the reference's Dataloader (dataloader.py:6-53)
plus DistributedSampler sharding.  On the gloo backend with world_size 2 the
ranks get disjoint, equally sized shards that together cover the dataset,
and set_epoch draws a new permutation."""
import os
import socket
import subprocess
import sys
from pathlib import Path

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from vsr_amd.data import Dataloader, SyntheticCine

ROOT = Path(__file__).resolve().parent.parent


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
    ds = SyntheticCine("sisr", volumes=2, frames=5, size=(8, 8), upscale_factor=2)  # 10 samples
    dl = Dataloader(ds, batch_size=2, shuffle=True, seed=3)
    epochs = []
    for e in (1, 2):
        dl.set_epoch(e)
        epochs.append([int(i) for b in dl for i in b["index"]])
    q.put((rank, epochs))
    dist.destroy_process_group()


def test_distributed_shards_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    got = dict(q.get(timeout=5) for _ in range(2))
    for e in range(2):
        a, b = got[0][e], got[1][e]
        assert len(a) == len(b) == 5
        assert set(a).isdisjoint(b) and sorted(a + b) == list(range(10))
    assert got[0][0] != got[0][1]  # set_epoch reshuffles


def test_single_process_is_the_reference_loader():
    ds = SyntheticCine("sisr", volumes=1, frames=6, size=(8, 8), upscale_factor=2)
    dl = Dataloader(ds, batch_size=4)
    assert dl.sampler.__class__.__name__ == "SequentialSampler"
    assert [b["lr_img"].shape[0] for b in dl] == [4, 2]
    assert dl.worker_init_fn is Dataloader._default_worker_init_fn


def test_bench_rejects_gpus_world_mismatch():
    """bench.py exits non-zero (before any GPU call) when --gpus disagrees with torchrun's WORLD_SIZE."""
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "1", "--steps", "1"], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 2 and "disagrees" in r.stderr


def test_shard_sampler_unpadded():
    """validation / test shards: contiguous, disjoint, no repeated samples."""
    from vsr_amd.data.dataloader import ShardSampler
    ds = list(range(10))
    parts = [list(ShardSampler(ds, num_replicas=3, rank=r)) for r in range(3)]
    assert sum(parts, []) == ds
    assert [len(p) for p in parts] == [3, 3, 4]
    assert all(len(ShardSampler(ds, 3, r)) == len(parts[r]) for r in range(3))
