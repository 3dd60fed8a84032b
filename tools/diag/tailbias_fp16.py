"""Diagnostic: EDSR golden tail.conv.bias gradient and the
L1 residual sign flips against fp64, with the one-channel stencil tail on / off,
per precision; per-voxel output error statistics of both paths."""
import sys
from pathlib import Path
sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
sys.path.insert(0, str(Path(__file__).resolve().parents[2] / "tests"))
import torch
from vsr_amd import functional as F
import test_nets_gpu as T

for name in ("edsr_x4_canon", "edsr_x2_small") if len(sys.argv) < 2 else sys.argv[1:]:
    try:
        fx = T.load_golden(name)
    except Exception as e:  # noqa: BLE001
        print(name, "missing", e)
        continue
    o64, h64 = T._flat(fx["output64"]).double(), T._flat(fx["hr"]).double()
    r64 = o64 - h64
    for mode in (1, 0):
        F.set_conv_path("stencil", mode)
        for prec in ("fp16", "bf16"):
            net = T._build(fx, prec)
            lr, hr = T._to(fx["lr"]), T._to(fx["hr"])
            out = net(lr)
            loss = T._l1(out, hr)
            loss.backward()
            torch.cuda.synchronize()
            got = T._flat(out).detach().cpu().double()
            d = got - o64
            flips = ((got - h64).sign() != r64.sign())
            p = dict(net.named_parameters())["tail.conv.bias"]
            rel = T._rel(p.grad.detach().cpu().double(), fx, "tail.conv.bias")
            env = fx[f"{prec}_env"]["tail.conv.bias"]
            print(f"{name} stencil={mode} {prec}: out dtype {out.dtype} max|d| {d.abs().max().item():.3e} "
                  f"mean|d| {d.abs().mean().item():.3e} mean d {d.mean().item():+.3e} rms {d.pow(2).mean().sqrt().item():.3e} | "
                  f"flips {int(flips.sum())} (|r64| of flipped: max {r64.abs()[flips].max().item() if flips.any() else 0:.2e}) "
                  f"| tail.bias rel {rel:.4f} env {env:.4f} | N {o64.numel()}", flush=True)
    F.set_conv_path("stencil", -1)
