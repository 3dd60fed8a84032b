#!/usr/bin/env python
"""Throughput benchmark of the cardiac cine-MRI SR train step on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--model edsr|duf|drf]
    torchrun --nproc-per-node N bench.py --gpus N ...      (driver, N > 1)

A step is one full train step (generator forward, L1 loss, backward, Adam)
over one synthetic batch of the BASELINE cfg-2 shape: per GPU a 4 x 16 x
128 x 128 cine volume at 4x SR (bf16).  Each rank holds its own volume
(weak scaling: data-parallel, gradients all-reduced over RCCL).

metric  = LR voxels/s (one LR input voxel of a target frame; B*T*H*W =
          1,048,576 per GPU per step), whole job.
roofline: the dominant kernel's algorithmic FLOP per launch / its mean
          launch time (HIP events on the launch stream, inside the timed
          region) against the 2.5 PFLOP/s dense bf16 MFMA peak.
cpu_baseline: the CPU fp32 restatement of the same generator (oracle/,
          the reference's algorithm) timed on this host for a bounded sample
          (rank 0, N = 1 only).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

import torch
import torch.distributed as dist

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

from vsr_amd import _native, nets  # noqa: E402
from vsr_amd import functional as F  # noqa: E402
from vsr_amd.data import cyclic_windows, synth_cine  # noqa: E402
from vsr_amd.ddp import GradSync  # noqa: E402
from vsr_amd.losses import L1Loss  # noqa: E402

METRIC = "voxels/sec fwd+bwd, 4× SR on 16×128×128 cine volumes, 1/2/4/8 MI355X"
PEAK_BF16 = 2.5e15
PEAK_F32 = 157.3e12
B, T, H, W, R = 4, 16, 128, 128, 4

MODELS = {
    "edsr": dict(cls="EDSRNet", task="sisr",
                 kwargs=dict(in_channels=1, out_channels=1, num_resblocks=16, num_features=64, upscale_factor=R)),
    "duf": dict(cls="DUFNet", task="misr",
                kwargs=dict(in_channels=1, out_channels=1, num_frames=7, size_filter=5, upscale_factor=R,
                            backbone="_DenseLayer16")),
    "drf": dict(cls="DRFNet", task="vsr",
                kwargs=dict(in_channels=1, out_channels=1, num_features=64, num_groups=4, upscale_factor=R)),
}


def make_batch(task, lr, hr):
    """cfg-2 volume (B,T,h,w) -> the net's input/target (Dataset dict contract)."""
    if task == "sisr":
        return lr.reshape(B * T, 1, H, W), hr.reshape(B * T, 1, H * R, W * R)
    if task == "misr":
        return cyclic_windows(lr, 7), hr.reshape(B * T, 1, H * R, W * R)
    return [lr[:, t:t + 1] for t in range(T)], [hr[:, t:t + 1] for t in range(T)]


def dominant(model):
    """(kernel selector, algorithmic FLOP per launch, description)."""
    if model == "edsr":
        n = B * T
        flop = 2 * 64 * 64 * 9 * n * H * W

        def match(kind, x, y):
            return kind == ("conv_fwd", (1, 3, 3)) and x.shape[-1] == 64 and y.shape[-1] == 64 and y.shape[2] == H

        return match, flop, f"conv3x3 64->64 bf16 implicit-GEMM (fwd+dgrad launches), {n}x{H}x{W} per launch"
    if model == "duf":
        n = B * T

        def match(kind, x, y):
            return kind == ("conv_fwd", (3, 3, 3)) and x.shape[-1] == 64 and y.shape[-1] == 32

        flop = 2 * 32 * 64 * 27 * n * 7 * H * W
        return match, flop, f"conv3d 3x3x3 64->32 bf16 implicit-GEMM, {n}x7x{H}x{W} per launch"
    n = B

    def match(kind, x, y):
        # LR (128^2, 64 ch) -> HR sub-pixel store: the up projection's forward
        # and the down projection's data gradient (same shape)
        return kind == ("conv_fwd", (1, 3, 3)) and x.shape[-1] == 64 and x.shape[2] == H and y.shape[2] == R * H

    # the reference's algorithmic FLOP: ConvTranspose2d(64, 64, 8, stride 4),
    # 64*(8/4)^2 MACs per HR output value (the 3x3 sub-pixel form executes 2.25x that)
    flop = 2 * 64 * 64 * 4 * n * (R * H) * (R * W)
    return match, flop, f"DRF 4x up projection (ConvTranspose2d 64->64 8x8/4 as sub-pixel 3x3 conv), {n}x{H}x{W} LR per launch"


def _traffic(model, precision):
    """HBM bytes per launch of the dominant kernel, from the committed
    rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over this bench
    (tools/pmc_traffic.py, gfx950 FETCH_SIZE correction applied), or None."""
    p = ROOT / "profiles" / f"traffic_{model}_{precision}.json"
    if not p.exists():
        return None
    return json.loads(p.read_text())["traffic_bytes"]


def cpu_baseline(model, budget_s=20.0):
    """Reference algorithm (oracle CPU restatement) on this host, bounded sample."""
    from oracle import cpu_nets

    threads = min(16, os.cpu_count() or 1)
    torch.set_num_threads(threads)
    spec = MODELS[model]
    cls = {"EDSRNet": cpu_nets.EDSRRef, "DUFNet": cpu_nets.DUFRef, "DRFNet": cpu_nets.DRFRef}[spec["cls"]]
    torch.manual_seed(0)
    net = cls(**spec["kwargs"])
    opt = torch.optim.Adam(net.parameters(), lr=1e-4)
    lr, hr = synth_cine(1, T, H, W, R, seed=99)
    if spec["task"] == "sisr":
        nb = 2
        x, y = lr[0, :nb].reshape(nb, 1, H, W), hr[0, :nb].reshape(nb, 1, H * R, W * R)
        vox, sample = nb * H * W, f"{nb} slices of 128x128 (x4), fp32"
    elif spec["task"] == "misr":
        nb = 1
        x = [w[:nb] for w in cyclic_windows(lr, 7)]
        y = hr[0, :nb].reshape(nb, 1, H * R, W * R)
        vox, sample = nb * H * W, f"{nb} 7-frame window of 128x128 (x4), fp32"
    else:
        x, y = [lr[:, t:t + 1] for t in range(2)], [hr[:, t:t + 1] for t in range(2)]
        vox, sample = 2 * H * W, "1 sequence x 2 frames of 128x128 (x4), fp32"
    l1 = torch.nn.L1Loss()

    def step():
        out = net(x)
        if isinstance(out, list):
            loss = torch.stack([l1(o, t) for o, t in zip(out, y)]).mean()
        else:
            loss = l1(out, y)
        opt.zero_grad()
        loss.backward()
        opt.step()

    step()  # warm-up
    times = []
    t_all = time.perf_counter()
    while (time.perf_counter() - t_all < budget_s and len(times) < 5) or len(times) < 1:
        t0 = time.perf_counter()
        step()
        times.append(time.perf_counter() - t0)
    times.sort()
    med = times[len(times) // 2]
    return {"value": vox / med, "unit": "voxels/s", "cores": threads, "kind": "port",
            "sample": f"{sample}; median of {len(times)} steps after 1 warm-up ({med:.2f} s/step)"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--model", default=os.environ.get("VSR_BENCH_MODEL", "edsr"), choices=list(MODELS))
    ap.add_argument("--precision", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # VSR_BENCH_BACKEND=gloo rehearses the N>1 path (GradSync, max-over-ranks
    # timing) with every rank on the GPUs one box has; the measured path is
    # RCCL ("nccl"), one process per GPU.
    backend = os.environ.get("VSR_BENCH_BACKEND", "nccl")
    if backend != "nccl":
        local = local % max(1, torch.cuda.device_count())
    if world > 1:
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    _native.load()

    spec = MODELS[args.model]
    torch.manual_seed(0)  # identical initial weights on every rank
    net = getattr(nets, spec["cls"])(**spec["kwargs"]).to(dev).set_precision(args.precision).train()
    opt = torch.optim.Adam(net.parameters(), lr=1e-4)
    sync = GradSync(net, world) if world > 1 else None
    lr, hr = synth_cine(B, T, H, W, R, seed=1234 + rank, device=dev)
    x, y = make_batch(spec["task"], lr, hr)
    l1 = L1Loss()

    def step():
        out = net(x)
        if isinstance(out, list):
            loss = torch.stack([l1(o, t) for o, t in zip(out, y)]).mean()
        else:
            loss = l1(out, y)
        opt.zero_grad(set_to_none=True)
        loss.backward()
        if sync is not None:
            sync.finish()
        opt.step()
        return loss

    for _ in range(args.warmup):
        step()
    match, flop_launch, kdesc = dominant(args.model)
    F.timer = F.KernelTimer(match)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kernel_ms = F.timer.mean_ms()
    F.timer = None
    if world > 1:
        t = torch.tensor([elapsed], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()
    vox_step = B * T * H * W
    value = world * vox_step * args.steps / elapsed
    peak = PEAK_BF16 if args.precision == "bf16" else PEAK_F32
    achieved = flop_launch / (kernel_ms * 1e-3) if kernel_ms == kernel_ms else None  # NaN: no launch matched
    if rank == 0:
        res = {
            "metric": METRIC, "value": value, "unit": "voxels/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": args.precision, "data": "synthetic",
            "config": {"workload": f"cfg2: ACDC 4x SR, {B}x{T}x{H}x{W} LR cine volume per GPU, "
                                   f"{spec['cls']} ({spec['task'].upper()}), L1 + Adam",
                       "model": spec["cls"], "global_batch": world * B * T, "seq_len": T,
                       "parallelism": f"dp{world}"},
            "roofline": {"bound": "mfma", "achieved": achieved / 1e12 if achieved else None, "peak": peak / 1e12,
                         "unit": "TFLOP/s", "frac": achieved / peak if achieved else None, "traffic": _traffic(args.model, args.precision), "kernel": kdesc,
                         "kernel_ms": kernel_ms if achieved else None, "flop_per_launch": flop_launch},
            "final_loss": float(loss.item()),
        }
        if world == 1 and not args.no_cpu_baseline:
            res["cpu_baseline"] = cpu_baseline(args.model)
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
