"""Standalone timing of the conv kernels at the cfg-2 shapes (for rocprofv3
--pmc passes and A/B work).  Prints one line per case: mean ms and TFLOP/s."""
import argparse
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from vsr_amd import _native  # noqa: E402
from vsr_amd import functional as F  # noqa: E402

CASES = {
    # name: (N, D, H, W, Cin, Cout, k, pad)
    "edsr3x3": (64, 1, 128, 128, 64, 64, (1, 3, 3), (0, 1, 1)),
    "duf3x3x3": (4, 16, 128, 128, 64, 32, (3, 3, 3), (1, 1, 1)),
    # the bench's DUF unit convs: 64 windows x 7 frames
    "duf64": (64, 7, 128, 128, 64, 32, (3, 3, 3), (1, 1, 1)),
    "duf224v": (64, 7, 128, 128, 224, 32, (3, 3, 3), (0, 1, 1)),
    # the bench's three depth-valid DUF units (T = 7: 7 -> 5, 5 -> 3, 3 -> 1 depths)
    "duf_u3": (64, 7, 128, 128, 160, 32, (3, 3, 3), (0, 1, 1)),
    "duf_u4": (64, 5, 128, 128, 192, 32, (3, 3, 3), (0, 1, 1)),
    "duf_u5": (64, 3, 128, 128, 224, 32, (3, 3, 3), (0, 1, 1)),
    "duf1x1x1": (64, 7, 128, 128, 128, 128, (1, 1, 1), (0, 0, 0)),
    "duf1x1x1_224": (64, 3, 128, 128, 224, 224, (1, 1, 1), (0, 0, 0)),
    "duf1x1x1_160": (64, 7, 128, 128, 160, 160, (1, 1, 1), (0, 0, 0)),
    "duf1x1x1_192": (64, 5, 128, 128, 192, 192, (1, 1, 1), (0, 0, 0)),
    "duf1x1x1_64": (64, 7, 128, 128, 64, 64, (1, 1, 1), (0, 0, 0)),
    # DUF's filter / residual head 1x1 convs at depth 1 (duf_net.py:40-49)
    "duf_fn1": (64, 1, 128, 128, 256, 512, (1, 1, 1), (0, 0, 0)),
    "duf_fn2": (64, 1, 128, 128, 512, 400, (1, 1, 1), (0, 0, 0)),
    "duf_rn1": (64, 1, 128, 128, 256, 256, (1, 1, 1), (0, 0, 0)),
    # EDSR tail conv F -> 1 at HR (thin-channel kernels: fwd = thin-out, dgrad = thin-in)
    "tail": (64, 1, 512, 512, 64, 1, (1, 3, 3), (0, 1, 1)),
    "head": (64, 1, 128, 128, 1, 64, (1, 3, 3), (0, 1, 1)),
}


def _padded(t, dt):
    """thin (c < 8) tensors live in 8-channel storage, as in the nets."""
    if t.shape[-1] >= 8:
        return t.to("cuda", dt)
    st = torch.zeros((*t.shape[:-1], 8), dtype=dt, device="cuda")
    st[..., :t.shape[-1]] = t.to("cuda", dt)
    return st[..., :t.shape[-1]]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--case", default="edsr3x3")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--what", default="fwd,res,wgrad")
    ap.add_argument("--yf32", action="store_true", help="fp32 forward output (DUF's filter head)")
    ap.add_argument("--paths", default="", help="e.g. k3=0,fast=1 (vsrk_conv_set_path)")
    ap.add_argument("--stamps", action="store_true",
                    help="after each case, print the s_memtime stamps of a ROLL_STAMP diagnostic build")
    args = ap.parse_args()
    _native.load()
    for kv in filter(None, args.paths.split(",")):
        p, m = kv.split("=")
        F.set_conv_path(p, int(m))
    dev = "cuda"
    n, d, h, w, ci, co, k, pad = CASES[args.case]
    dt = torch.bfloat16
    g = torch.Generator(device="cpu").manual_seed(0)
    x = _padded(torch.randn((n, d, h, w, ci), generator=g), dt)
    wt = (torch.randn((co, ci, *k), generator=g) * 0.05).to(dev)
    b = torch.randn(co, generator=g).to(dev)
    do = d + 2 * pad[0] - k[0] + 1
    y = torch.empty((n, do, h, w, co), dtype=dt if co >= 8 and not args.yf32 else torch.float32, device=dev)
    res = torch.randn((n, do, h, w, co), generator=g).to(dev, y.dtype)
    gy = _padded(torch.randn((n, do, h, w, co), generator=g), dt)
    dx = torch.empty((n, d, h, w, ci), dtype=dt if ci >= 8 else torch.float32, device=dev)
    wp1 = F.pack_weight(wt, 1, dt)
    dpad = tuple(kk - 1 - p for kk, p in zip(k, pad))
    # HBM bytes of one pass over the wide side + the narrow side (thin kernels are HBM-bound)
    esz = {torch.bfloat16: 2, torch.float32: 4}
    nbytes = {"fwd": x.numel() // x.shape[-1] * (ci * 2) + y.numel() * esz[y.dtype],
              "dgrad": gy.numel() // gy.shape[-1] * (co * 2) + dx.numel() * esz[dx.dtype],
              "fwdpro": x.numel() // x.shape[-1] * (ci * 2) + y.numel() * esz[y.dtype],
              "wgradpro": x.numel() // x.shape[-1] * (ci * 2) + gy.numel() // gy.shape[-1] * (co * 2),
              "wgrad": x.numel() // x.shape[-1] * (ci * 2) + gy.numel() // gy.shape[-1] * (co * 2)}
    nbytes["dgradred"] = nbytes["dgrad"] + dx.numel() * esz[dx.dtype]
    dw = torch.empty((co, ci, *k), device=dev)
    db = torch.empty(co, device=dev)
    wp = F.pack_weight(wt, 0, dt)
    psc = torch.rand(ci, generator=g).to(dev) + 0.5
    psh = torch.randn(ci, generator=g).to(dev)
    flop = 2.0 * n * do * h * w * co * ci * k[0] * k[1] * k[2]
    cases = {
        "fwd": lambda: F.conv(x, wp, y, k, pad, bias=b),
        "fwdpro": lambda: F.conv(x, wp, y, k, pad, bias=b, prologue=F.PRO_AFFINE_RELU, pro_scale=psc, pro_shift=psh),
        "res": lambda: F.conv(x, wp, y, k, pad, bias=b, out_scale=0.1, residual=res),
        "relu": lambda: F.conv(x, wp, y, k, pad, bias=b, act=F.ACT_RELU),
        "mask": lambda: F.conv(gy, wp1, dx, k, dpad, out_scale=0.1, mask=x),
        "resacc": lambda: F.conv(gy, wp1, dx, k, dpad, residual=x, accumulate=True),
        "wgrad": lambda: F.conv_wgrad(x, gy, k, pad, dw, db),
        "wgradpro": lambda: F.conv_wgrad(x, gy, k, pad, dw, db, prologue=F.PRO_AFFINE_RELU, pro_scale=psc,
                                         pro_shift=psh),
        "dgrad": lambda: F.conv(gy, wp1, dx, k, dpad),
        # the fused form DUF runs (bn2's backward reduce in the data gradient's store pass)
        "dgradred": lambda: F.conv_reduce(gy, wp1, dx, bnx=bnx, st=st, k=k, pad=dpad),
    }
    bnx = torch.randn((n, d, h, w, ci), generator=g).to(dev, dt) if ci >= 8 else None
    st = torch.stack([torch.rand(ci, generator=g) + 0.5, torch.randn(ci, generator=g) * 0.1,
                      torch.randn(ci, generator=g) * 0.1, torch.rand(ci, generator=g) + 0.5]).to(dev)
    for name in args.what.split(","):
        fn = cases[name]
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(args.iters):
            fn()
        e.record()
        torch.cuda.synchronize()
        ms = s.elapsed_time(e) / args.iters
        print(f"{args.case:10s} {name:6s} {ms * 1e3:9.1f} us  {flop / ms / 1e9:8.1f} TFLOP/s  "
              f"({flop / ms / 1e9 / 2500 * 100:.1f}% of 2.5 PF)  "
              f"{nbytes.get(name, 0) / ms / 1e9:7.2f} TB/s (min HBM bytes)", flush=True)
        if args.stamps:
            if name.startswith("wgrad"):
                stamp_report(fn, "vsrk_wroll_stamps", ["wait", "barrier", "compute"])
            else:
                stamp_report(fn)


def stamp_report(fn, sym="vsrk_roll_stamps", names=("wait", "barrier", "flush", "compute")):
    """Per-step cycle split of waves 0 and 4 (one SIMD) of workgroups 0-15
    from a conv_roll.hip ROLL_STAMP build: stage wait, barrier, flush
    (epilogue), compute."""
    import ctypes
    import numpy as np
    lib = _native.load()
    fn()
    torch.cuda.synchronize()
    buf = (ctypes.c_uint * (16 * 2 * 128))()
    if getattr(lib, sym)(buf) != 0:
        raise RuntimeError(f"{sym} failed")
    st = np.frombuffer(buf, dtype=np.uint32).reshape(32, 128).astype(np.int64)
    ne = len(names)
    tot = np.zeros(ne)
    cnt = 0
    for w in range(32):
        s = st[w]
        if not s.any():
            continue
        d = np.diff(s) % (1 << 32)
        # d[i] = stamp[i+1] - stamp[i]: event (i+1) % 4 ends the phase
        per = np.zeros(ne)
        for i, v in enumerate(d):
            per[(i + 1) % ne] += v
        tot += per
        cnt += 1
        if w in (0, 1):
            print(f"  wg{w // 2} wave{4 * (w % 2)}: " + " ".join(
                f"{names[(i + 1) % ne][0]}{int(v)}" for i, v in enumerate(d[:40])))
    if cnt:
        steps = 127 / ne
        print("  mean cycles per step: " + "  ".join(f"{n} {tot[i] / cnt / steps:8.0f}" for i, n in enumerate(names)))


if __name__ == "__main__":
    main()
