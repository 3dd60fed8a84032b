"""Diagnostic: EDSR golden fp16 tail.conv.bias gradient with the stencil paths on / off."""
import sys
from pathlib import Path
sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
sys.path.insert(0, str(Path(__file__).resolve().parents[2] / "tests"))
import torch
from vsr_amd import functional as F
import test_nets_gpu as T

fx = T.load_golden("edsr_x4_canon")
for mode in (1, 0):
    F.set_conv_path("stencil", mode)
    for prec in ("fp16", "bf16", "fp32"):
        net = T._build(fx, prec)
        lr, hr = T._to(fx["lr"]), T._to(fx["hr"])
        out = net(lr)
        loss = T._l1(out, hr)
        loss.backward()
        torch.cuda.synchronize()
        got, exp = T._flat(out).detach().cpu().double(), T._flat(fx["output64"]).double()
        d = (got - exp).abs()
        p = dict(net.named_parameters())["tail.conv.bias"]
        rel = T._rel(p.grad.detach().cpu().double(), fx, "tail.conv.bias")
        near = ((out.detach().double() - hr.double()).abs() < 2e-3).sum().item()
        print(f"stencil={mode} {prec}: out max {d.max().item():.3e} mean {d.mean().item():.3e} "
              f"tail.bias rel {rel:.4f} env {fx['fp16_env']['tail.conv.bias']:.4f} |o-hr|<2e-3: {near} of {out.numel()}",
              flush=True)
