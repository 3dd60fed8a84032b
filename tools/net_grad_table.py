"""Per-parameter gradient error table of a net fixture vs its fp64 yardstick.

    python tools/net_grad_table.py duf_x4_canon [fp32|bf16]
"""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from tests.conftest import load_golden  # noqa: E402
from tests.test_nets_gpu import _build, _flat, _l1, _to  # noqa: E402

name = sys.argv[1]
prec = sys.argv[2] if len(sys.argv) > 2 else "fp32"
fx = load_golden(name)
net = _build(fx, prec)
lr, hr = _to(fx["lr"]), _to(fx["hr"])
out = net(lr)
_l1(out, hr).backward()
torch.cuda.synchronize()
d = (_flat(out).detach().cpu().double() - _flat(fx["output64"]).double()).abs()
print(f"output max|d| {d.max().item():.3e}  ref32 {fx['out_err32']:.3e}")
for k, p in net.named_parameters():
    g = p.grad.detach().cpu().double()
    r32 = fx["ref32_err"][k]
    if k in fx["grad_full64"]:
        ref = fx["grad_full64"][k].double()
        rel = (g - ref).norm().item() / max(ref.norm().item(), 1e-300)
        how = "full"
    else:
        rel = abs(g.norm().item() - fx["grad_norm64"][k]) / fx["grad_norm64"][k]
        how = "norm"
    flag = "" if r32 is None or rel <= max(1e-4, 3 * r32) else "  <<<"
    print(f"{k:40s} {how} rel={rel:.3e} ref32={'-' if r32 is None else f'{r32:.2e}'}{flag}")
