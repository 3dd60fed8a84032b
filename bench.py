#!/usr/bin/env python
"""Throughput benchmark of the cardiac cine-MRI SR train step on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--models edsr,duf] [--config cfg2|cfg3|cfg4|cfg5]
    torchrun --nproc-per-node N bench.py --gpus N ...      (driver, N > 1)

With --gpus N > 1 and no torchrun environment, bench.py starts the N ranks
itself (one process per GPU, before any GPU call); under torchrun --gpus must
equal WORLD_SIZE.

A step is one full train step (generator forward, L1 loss, backward, Adam)
over one synthetic batch of the BASELINE cfg-2 shape: per GPU a 4 x 16 x
128 x 128 cine volume at 4x SR.  Each rank holds its own volume (weak
scaling: data-parallel, gradients all-reduced over RCCL, BatchNorm statistics
synchronised for DUF).

Models (each timed on its own, all reported in the one JSON line):
  edsr  EDSRNet on the volume's 64 slices (2-D residual blocks + PixelShuffle)
  duf   DUFNet on the volume's 64 seven-frame cyclic windows (Conv3d 3x3x3 /
        BatchNorm3d dense blocks + dynamic upsampling filter)
The top-level value/roofline are the first model's; "models" holds each one.

metric  = LR voxels/s (one LR input voxel of a target frame; B*T*H*W =
          1,048,576 per GPU per step), whole job.
roofline: the model's dominant conv, forward + data gradient + weight
          gradient together: algorithmic FLOP (2*cin*cout*taps per output
          voxel, three times) over the summed launch time of those kernels
          (HIP events on the launch stream, inside the timed region), against
          the dense MFMA peak of the compute dtype.  EDSR: the 33 body convs
          3x3 64->64; DUF: the six Conv3d 3x3x3 F->32 (F = 64..224).
--config picks the BASELINE.json workload: cfg2 (default: ACDC, 4 x 16 x
128 x 128 per GPU, bf16, EDSR + DUF), cfg3 (DSB15, DRF on 4 x 30-frame
stacks), cfg4 (ACDC full volumes: DUF on 2 uncropped 30-frame cine
volumes of 64 x 64 LR / 256 x 256 HR per GPU), cfg5 (ACDC + DSB15 mixed,
fp16, batch 8 per GPU, EDSR + DUF).
comm (N > 1): the data-parallel traffic of one step -- gradient bytes and
          buckets, and the time of the step's bucket all-reduces and SyncBN
          all-reduces each run alone after the timed region (HIP events), to
          set beside ms_per_step: what the overlap with backward must hide.
measured_peak: this device's dense bf16 MFMA rate and HBM copy rate from
          two microbenchmarks (vsrk_peak_mfma / vsrk_peak_copy), with each
          roofline's fraction of the measured MFMA rate beside the vendor one.
cpu_baseline: the CPU fp32 restatement of the same generator (oracle/,
          the reference's algorithm) timed on this host for a bounded sample
          (rank 0, N = 1 only), threads = the CPU share of this process.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
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
from vsr_amd.ddp import GradSync, enable_sync_bn  # noqa: E402
from vsr_amd.losses import L1Loss  # noqa: E402

METRIC = "voxels/sec fwd+bwd, 4× SR on 16×128×128 cine volumes, 1/2/4/8 MI355X"
PEAK = {"bf16": 2.5e15, "fp16": 2.5e15, "fp32": 157.3e12}
HBM_PEAK = 8.0e12  # MI355X HBM3E spec (MI355X_MICROARCH.md; ~6.3e12 achievable)
B, T, H, W, R = 4, 16, 128, 128, 4
DATASET = "acdc"  # synthetic-data normalisation: "acdc", "dsb15" or "mixed" (half the volumes each)
# BASELINE.json configs measurable on one node (--config): the batch / frames /
# dataset / precision / models of each; cfg 2 is the default bench line.
CONFIGS = {
    "cfg2": dict(B=4, T=16, dataset="acdc", precision="bf16", models="edsr,duf",
                 desc="ACDC 4x SR, 3D 16x128x128 volumes bf16, batch 4 per GPU"),
    # cfg3: DRF's recurrent step (eager; a HIP-graph replay measured slower,
    # DESIGN.md section 7)
    "cfg3": dict(B=4, T=30, dataset="dsb15", precision="bf16", models="drf",
                 desc="DSB15 cine 4x SR, T=30 2D+t stacks (DRF), batch 4 per GPU"),
    "cfg4": dict(B=2, T=30, H=64, W=64, dataset="acdc", precision="bf16", models="duf",
                 desc="ACDC 4x SR, full 3D cine volumes (2 x 30 frames of 64x64 LR, 256x256 HR, no crop) per GPU"),
    "cfg5": dict(B=8, T=16, dataset="mixed", precision="fp16", models="edsr,duf",
                 desc="mixed ACDC+DSB15 4x SR, fp16 MFMA path, batch 8 per GPU"),
}

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


def _vox(v) -> int:
    return v.n * v.d * v.h * v.w


def dominant(model, precision="bf16"):
    """(matcher, description).  matcher(kind, xv, yv) -> algorithmic FLOP of the
    launch (counted as the forward conv's 2*cin*cout*taps per forward output
    voxel) when it is one of the roofline kernels, else 0.  xv/yv are the
    launch's logical views (for the weight gradient: input and output grad)."""
    if model == "edsr":
        def match(kind, xv, yv):
            if kind[1] != (1, 3, 3) or xv.c != 64 or yv.c != 64 or xv.h != H or yv.h != H:
                return 0
            if xv.shuffle > 1 or yv.shuffle > 1:
                return 0
            return 2 * 64 * 64 * 9 * _vox(yv)  # fwd: y is the output; dgrad: same size; wgrad: yv = dy

        return match, (f"EDSR body conv3x3 64->64 {precision} implicit-GEMM, fwd + dgrad + wgrad per layer, "
                       f"{B * T}x{H}x{W} per launch (33 layers)")
    if model == "duf":
        def match(kind, xv, yv):
            if kind[1] != (3, 3, 3):
                return 0
            if kind[0] == "conv_wgrad" and yv.c == 32:  # x: unit input (F ch), dy: unit output grad
                return 2 * 27 * xv.c * 32 * _vox(yv)
            if kind[0] == "conv_fwd" and yv.c == 32:  # forward: y = unit output
                return 2 * 27 * xv.c * 32 * _vox(yv)
            if kind[0] == "conv_fwd" and xv.c == 32:  # data gradient: x = dy (forward output)
                return 2 * 27 * yv.c * 32 * _vox(xv)
            return 0

        return match, (f"DUF Conv3d 3x3x3 F->32 (F = 64..224) {precision} implicit-GEMM, fwd + dgrad + wgrad, "
                       f"{B * T} windows x 7 x {H}x{W}")

    def match(kind, xv, yv):
        # LR (128^2, 64 ch) -> HR sub-pixel store: the up projection's forward and
        # the down projection's data gradient; reference FLOP of ConvTranspose2d
        # 64->64 8x8/4: 64*(8/4)^2 MACs per HR output value (the 3x3 sub-pixel
        # form executes 2.25x that)
        if kind == ("conv_fwd", (1, 3, 3)) and xv.c == 64 and xv.h == H and yv.shuffle == R:
            return 2 * 64 * 64 * 4 * xv.n * (R * H) * (R * W)
        return 0

    return match, "DRF 4x up projection (ConvTranspose2d 64->64 8x8/4 as sub-pixel 3x3 conv)"


def _traffic(model, precision):
    """HBM bytes per launch of the model's forward roofline kernel, from the
    committed rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over this bench
    (tools/pmc_traffic.py, gfx950 FETCH_SIZE correction applied), or None."""
    p = ROOT / "profiles" / f"traffic_{model}_{precision}.json"
    if not p.exists():
        return None, None
    d = json.loads(p.read_text())
    return d["traffic_bytes"], d.get("kernel")


def cpu_threads() -> int:
    """Threads for the CPU baseline: this process's CPU share (OMP_NUM_THREADS
    where the box sets it to the share, else the CPUs this process may run on)."""
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit() and int(env) > 0:
        return int(env)
    try:
        return len(os.sched_getaffinity(0))
    except AttributeError:
        return os.cpu_count() or 1


def cpu_baseline(model, budget_s=20.0):
    """Reference algorithm (oracle CPU restatement) on this host, bounded sample."""
    from oracle import cpu_nets

    threads = cpu_threads()
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


def comm_report(net, sync, dev, iters=20):
    """The step's collectives, each timed alone (after the timed region): the
    gradient bucket all-reduces of GradSync and the SyncBN all-reduces (one per
    BatchNorm per direction, 2 x C floats)."""
    def timed(fn):
        fn()
        torch.cuda.synchronize()
        dist.barrier()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(iters):
            fn()
        e.record()
        torch.cuda.synchronize()
        return s.elapsed_time(e) / iters

    def buckets():
        for b in range(len(sync.flat)):
            sync._launch(b)
        for h in sync._handles:
            h.wait()
        sync._reset()

    out = {"grad_bytes": int(sum(f.numel() * 4 for f in sync.flat)), "buckets": len(sync.flat),
           "grad_allreduce_ms": timed(buckets)}
    bns = [m for m in net.modules() if isinstance(m, torch.nn.BatchNorm3d)]
    if bns and getattr(net, "bn_allreduce", None) is not None:
        ts = [torch.zeros(2 * m.num_features, device=dev) for m in bns]
        out["syncbn_allreduces_per_step"] = 2 * len(bns)
        out["syncbn_allreduce_ms_per_step"] = 2 * timed(lambda: [dist.all_reduce(t) for t in ts])
    return out


def metric_report(net, x, y, dev, iters=10):
    """The reference's per-step metric computation (base_trainer.py:135:
    _compute_metrics = denormalize (utils.py:1-20) then PSNR / SSIM,
    metrics.py:20-36, 86-113) on the step's outputs, through the trainer
    mirror's _metric (one fused HIP kernel each), timed on its own after the
    timed train steps -- SURVEY 8(d): metrics excluded from the voxels/s
    figure and reported separately."""
    from vsr_amd import metrics as M
    from vsr_amd.runner.trainers import _metric
    with torch.no_grad():
        out = net(x)
    outs = out if isinstance(out, list) else [out]
    tgts = y if isinstance(y, list) else [y]
    res = {}
    for name, fn in (("psnr", M.PSNR()), ("ssim", M.SSIM())):
        def run():
            return torch.stack([_metric(fn, o, t, DATASET if DATASET != "mixed" else "acdc")
                                for o, t in zip(outs, tgts)]).mean()
        run()
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record()
        for _ in range(iters):
            v = run()
        ev1.record()
        torch.cuda.synchronize()
        res[name] = {"ms_per_step": ev0.elapsed_time(ev1) / iters, "value": float(v.item())}
    res["ms_per_step"] = res["psnr"]["ms_per_step"] + res["ssim"]["ms_per_step"]
    res["note"] = "denormalize + PSNR + SSIM of the step's outputs, per train step, outside the timed region"
    return res


def write_units(path, model, precision, rows):
    """Per-launch table of the roofline kernel (one step, launch order): the
    per-unit north-star table (DUF: 6 dense units x fwd / dgrad / wgrad)."""
    if not rows:
        return
    tot_us = sum(r["us"] for r in rows)
    tot_f = sum(r["gflop"] for r in rows)
    with open(path, "a") as f:
        f.write(f"# {model} {precision}: {len(rows)} launches per step, {tot_us / 1e3:.3f} ms, "
                f"{tot_f / 1e3:.3f} TFLOP, frac {tot_f * 1e9 / (tot_us * 1e-6) / PEAK[precision]:.3f} of "
                f"{PEAK[precision] / 1e15:.1f} PF; bound = max(FLOP / MFMA peak, bytes / {HBM_PEAK / 1e12:.0f} TB/s)\n")
        f.write(f"{'pos':>3} {'dir':<6} {'shape (taps cin x D -> cout x D @ n x h x w)':<44} {'us':>8} {'GFLOP':>8} "
                f"{'MB':>8} {'frac':>6} {'TB/s':>6} {'bound':>6}\n")
        for r in rows:
            f.write(f"{r['pos']:>3} {r['dir']:<6} {r['shape']:<44} {r['us']:>8.1f} {r['gflop']:>8.1f} {r['mb']:>8.1f} "
                    f"{r['frac']:>6.3f} {r['hbm_frac'] * HBM_PEAK / 1e12:>6.2f} {r['bound_frac']:>6.3f}\n")


def run_model(name, args, world, rank, dev):
    spec = MODELS[name]
    torch.manual_seed(0)  # identical initial weights on every rank
    net = getattr(nets, spec["cls"])(**spec["kwargs"]).to(dev).set_precision(args.precision).train()
    opt = torch.optim.Adam(net.parameters(), lr=1e-4)
    sync = None
    if world > 1:
        sync = GradSync(net, world)
        enable_sync_bn(net)  # DUF's BatchNorm3d: global-batch statistics (SyncBN)
    if DATASET == "mixed":  # ConcatDataset of the two: per-sample normalisation constants
        la, ha = synth_cine(B - B // 2, T, H, W, R, "acdc", seed=1234 + rank, device=dev)
        lb, hb = synth_cine(B // 2, T, H, W, R, "dsb15", seed=4321 + rank, device=dev)
        lr, hr = torch.cat([la, lb]), torch.cat([ha, hb])
    else:
        lr, hr = synth_cine(B, T, H, W, R, DATASET, seed=1234 + rank, device=dev)
    x, y = make_batch(spec["task"], lr, hr)
    l1 = L1Loss()

    def phase(p):
        if F.timer is not None:
            F.timer.phase = p

    def step():
        phase("fwd")
        out = net(x)
        if isinstance(out, list):
            loss = torch.stack([l1(o, t) for o, t in zip(out, y)]).mean()
        else:
            loss = l1(out, y)
        opt.zero_grad(set_to_none=True)
        phase("bwd")
        loss.backward()
        if sync is not None:
            sync.finish()
        if net.step_ok():  # fp16: skip a step whose gradients overflowed
            opt.step()
        return loss

    match, kdesc = dominant(name, args.precision)
    for _ in range(args.warmup):
        step()
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
    flop, kernel_s, launches = F.timer.totals()
    tsteps = getattr(F.timer, "steps", args.steps)  # steps the kernel timer saw
    by_dir = {}  # fwd / dgrad / wgrad launches of the roofline kernel on their own
    for lab in F.timer.labels():
        f_, t_, n_ = F.timer.totals(lab)
        tb_, _, b_ = F.timer.bound_seconds(PEAK[args.precision], HBM_PEAK, lab)
        by_dir[lab] = {"ms_per_step": t_ / tsteps * 1e3, "launches_per_step": n_ / tsteps,
                       "tflop_per_step": f_ / tsteps / 1e12,
                       "frac": (f_ / t_ / PEAK[args.precision]) if t_ > 0 else None,
                       "gb_per_step": b_ / tsteps / 1e9, "bound_frac": (tb_ / t_) if t_ > 0 else None}
    # each launch priced at max(FLOP / MFMA peak, algorithmic bytes / HBM peak):
    # the honest roofline of a conv near the ridge (EDSR's 64 -> 64 body convs)
    tb, tmf, bytes_ = F.timer.bound_seconds(PEAK[args.precision], HBM_PEAK)
    if args.units and rank == 0:
        write_units(args.units, name, args.precision, F.timer.per_launch(tsteps, PEAK[args.precision], HBM_PEAK))
    F.timer = None
    if world > 1:
        t = torch.tensor([elapsed], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()
    comm = comm_report(net, sync, dev) if world > 1 else None
    metrics = metric_report(net, x, y, dev)
    vox_step = B * T * H * W
    peak = PEAK[args.precision]
    achieved = flop / kernel_s if kernel_s > 0 else None
    traffic, tkern = _traffic(name, args.precision)
    res = {
        "value": world * vox_step * args.steps / elapsed, "unit": "voxels/s",
        "ms_per_step": elapsed / args.steps * 1e3,
        "config": {"workload": f"{args.config}: {CONFIGS[args.config]['desc']}; {B}x{T}x{H}x{W} LR voxels per GPU, "
                               f"{spec['cls']} ({spec['task'].upper()}), L1 + Adam",
                   "model": spec["cls"], "global_batch": world * B * T, "seq_len": T,
                   "parallelism": f"dp{world}" + ("+syncbn" if world > 1 and name == "duf" else "")},
        "roofline": {"bound": "mfma", "achieved": achieved / 1e12 if achieved else None, "peak": peak / 1e12,
                     "unit": "TFLOP/s", "frac": achieved / peak if achieved else None, "traffic": traffic,
                     "mfma_frac": achieved / peak if achieved else None,
                     "traffic_kernel": tkern, "kernel": kdesc,
                     "kernel_ms_per_step": kernel_s / tsteps * 1e3, "launches_per_step": launches / tsteps,
                     "flop_per_step": flop / tsteps, "by_direction": by_dir,
                     "bytes_per_step": bytes_ / tsteps, "hbm_peak_tbs": HBM_PEAK / 1e12,
                     "bound_ms_per_step": tb / tsteps * 1e3,
                     "bound_frac": (tb / kernel_s) if kernel_s > 0 else None,
                     "bound_mix": {"mfma_ms_per_step": tmf / tsteps * 1e3,
                                   "hbm_ms_per_step": (tb - tmf) / tsteps * 1e3},
                     "bound_note": "bound_frac = sum over launches of max(FLOP/MFMA peak, algorithmic bytes/HBM "
                                   "peak) / measured time; frac prices FLOP alone"},
        "final_loss": float(loss.item()),
    }
    rf = res["roofline"]
    if kernel_s > 0 and tb - tmf > tmf:
        # the launches are HBM-bound by their algorithmic bytes (EDSR's 64 -> 64
        # body convs: 268-402 MB per launch, 34-50 us at 8 TB/s against 31 us
        # of MFMA work): the roofline is the HBM one
        rf.update(bound="hbm", achieved=bytes_ / kernel_s / 1e9, peak=HBM_PEAK / 1e9, unit="GB/s",
                  frac=bytes_ / kernel_s / HBM_PEAK)
    if comm is not None:
        res["comm"] = comm
    if getattr(net, "_seq_run_k", None):  # DRF: frames per sequence-buffer chunk and per weight-gradient run
        ks = net._seq_run_k
        res["wgrad_runs"] = {"chunk_frames": net._seq_run_frames,
                             "run_frames": {str(k): sorted(n for n, v in ks.items() if v == k) for k in sorted(set(ks.values()))}}
    res["metrics"] = metrics
    del net, opt, sync
    torch.cuda.empty_cache()
    return res


def worker(args, world, rank, local):
    backend = os.environ.get("VSR_BENCH_BACKEND", "nccl")
    # VSR_BENCH_BACKEND=gloo rehearses the N>1 path with every rank on the GPUs
    # one box has; the measured path is RCCL ("nccl"), one process per GPU.
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

    names = [m for m in args.models.split(",") if m]
    results = {m: run_model(m, args, world, rank, dev) for m in names}
    if rank == 0:
        first = results[names[0]]
        out = {
            "metric": METRIC, "value": first["value"], "unit": "voxels/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": first["ms_per_step"], "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": args.precision, "data": "synthetic",
            "config": first["config"], "roofline": first["roofline"], "final_loss": first["final_loss"],
            "models": results,
        }
        if not args.no_peaks:
            # the measured ceilings beside the vendor peak the fractions use
            pk = F.measured_peaks(dev)
            out["measured_peak"] = pk
            for m in names:
                rf = results[m]["roofline"]
                if rf["achieved"]:
                    rf["frac_of_measured_peak"] = (rf["achieved"] / pk["mfma_bf16_tflops"] if rf["unit"] == "TFLOP/s"
                                                   else rf["achieved"] / (pk["hbm_copy_tbs"] * 1e3))
        if "duf" in results:
            # BASELINE.json north_star: ">= 50 % of CDNA4 bf16 MFMA roofline on the
            # 3x3x3 conv fwd+bwd at batch 4x16x128x128" -- the DUF line's roofline
            rf = results["duf"]["roofline"]
            out["north_star"] = {"model": "duf", "kernel": rf["kernel"], "achieved": rf["achieved"],
                                 "peak": rf["peak"], "unit": rf["unit"], "frac": rf["frac"], "target_frac": 0.5,
                                 "frac_of_measured_peak": rf.get("frac_of_measured_peak"),
                                 "launches_per_step": rf["launches_per_step"],
                                 "tflop_per_step": rf["flop_per_step"] / 1e12, "by_direction": rf["by_direction"]}
        if world == 1 and not args.no_cpu_baseline:
            for m in names:
                results[m]["cpu_baseline"] = cpu_baseline(m)
            out["cpu_baseline"] = results[names[0]]["cpu_baseline"]
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


def apply_config(args):
    """Set the module-level workload of --config (also in spawned ranks, which
    re-import this module with the cfg-2 defaults)."""
    global B, T, H, W, DATASET
    cfg = CONFIGS[args.config]
    B, T, DATASET = cfg["B"], cfg["T"], cfg["dataset"]
    H, W = cfg.get("H", 128), cfg.get("W", 128)


def _spawned(local, args, world, port):
    apply_config(args)
    os.environ.update(RANK=str(local), LOCAL_RANK=str(local), WORLD_SIZE=str(world),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    worker(args, world, local, local)


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="cfg2", choices=sorted(CONFIGS),
                    help="BASELINE.json config (batch, frames, dataset, precision, default models)")
    ap.add_argument("--models", default=os.environ.get("VSR_BENCH_MODELS"),
                    help="comma-separated subset of " + ",".join(MODELS))
    ap.add_argument("--model", default=None, help="a single model (same as --models NAME)")
    ap.add_argument("--precision", default=None, choices=["bf16", "fp16", "fp32"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-peaks", action="store_true", help="skip the measured MFMA / HBM peak microbenchmarks")
    ap.add_argument("--units", default=None, help="append the roofline kernel's per-launch table (one step) to FILE")
    args = ap.parse_args()
    cfg = CONFIGS[args.config]
    args.models = args.model or args.models or cfg["models"]
    args.precision = args.precision or cfg["precision"]
    apply_config(args)
    for m in args.models.split(","):
        if m not in MODELS:
            ap.error(f"unknown model {m!r}")

    env_world = os.environ.get("WORLD_SIZE")
    if env_world is not None:
        world = int(env_world)
        if world != args.gpus:
            print(f"bench.py: --gpus {args.gpus} disagrees with WORLD_SIZE={world}", file=sys.stderr)
            sys.exit(2)
        worker(args, world, int(os.environ.get("RANK", "0")), int(os.environ.get("LOCAL_RANK", "0")))
    elif args.gpus > 1:
        # start the ranks here, before this process touches the GPU
        import torch.multiprocessing as mp
        mp.spawn(_spawned, args=(args, args.gpus, _free_port()), nprocs=args.gpus, join=True)
    else:
        worker(args, 1, 0, 0)


if __name__ == "__main__":
    main()
