"""Direct single-channel conv vs fp64 and vs the MFMA thin path (diagnostic)."""
import sys
from pathlib import Path

import torch
import torch.nn.functional as Fn

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
from vsr_amd import functional as F  # noqa: E402


def run(dt, shape, cout, mode):
    n, h, w = shape
    g = torch.Generator().manual_seed(0)
    x = torch.randn((n, 1, h, w), generator=g)
    wt = torch.randn((cout, 1, 3, 3), generator=g) * 0.3 if mode == 0 else torch.randn((1, cout, 3, 3), generator=g) * 0.3
    b = torch.randn(cout, generator=g) if mode == 0 else None
    xs = torch.zeros((n, 1, h, w, 8), dtype=dt, device="cuda")
    xs[:, 0, :, :, 0] = x[:, 0].to("cuda", dt)
    xv = xs[..., :1]
    wp = F.pack_weight(wt.cuda(), mode, dt)
    xq = xs[:, 0, :, :, 0].double().cpu().unsqueeze(1)
    if mode == 0:
        ref = Fn.conv2d(xq, wt.to(dt).double(), b.double(), padding=1)
    else:
        ref = Fn.conv_transpose2d(xq, wt.to(dt).double(), padding=1)
    outs = {}
    for path in (1, 0):
        F.set_conv_path("thin", path)
        y = torch.empty((n, 1, h, w, cout), dtype=dt, device="cuda")
        F.conv(xv, wp, y, (1, 3, 3), (0, 1, 1), bias=b.cuda() if b is not None else None)
        torch.cuda.synchronize()
        outs[path] = y[:, 0].permute(0, 3, 1, 2).double().cpu()
    F.set_conv_path("thin", -1)
    for path, o in outs.items():
        d = (o - ref).abs()
        print(dt, shape, cout, "mode", mode, "thin" if path else "generic", "max", d.max().item(), "mean", d.mean().item(),
              flush=True)


for dt in (torch.float16, torch.bfloat16):
    run(dt, (2, 64, 96), 64, 0)
    run(dt, (2, 64, 96), 64, 1)
