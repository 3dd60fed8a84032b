"""Per-parameter gradient rel-L2 vs the fp64 fixture for bf16 and fp16 (diagnostic)."""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
from tests.conftest import load_golden  # noqa: E402
from tests.test_nets_gpu import _build, _flat, _l1, _rel, _to  # noqa: E402

for name in sys.argv[1:]:
    fx = load_golden(name)
    res = {}
    for prec in ("bf16", "fp16"):
        net = _build(fx, prec)
        lr, hr = _to(fx["lr"]), _to(fx["hr"])
        out = net(lr)
        _l1(out, hr).backward()
        d = (_flat(out).detach().cpu().double() - _flat(fx["output64"]).double()).abs()
        res[prec] = ({k: (_rel(p.grad.detach().cpu().double(), fx, k) if fx["ref32_err"][k] is not None else None)
                      for k, p in net.named_parameters()}, d.max().item(), d.mean().item())
    print(f"== {name}: out max/mean bf16 {res['bf16'][1]:.2e}/{res['bf16'][2]:.2e}  fp16 {res['fp16'][1]:.2e}/{res['fp16'][2]:.2e}")
    rows = []
    for k in res["bf16"][0]:
        b, f = res["bf16"][0][k], res["fp16"][0][k]
        if b is None:
            continue
        rows.append((f / max(b, 1e-12), k, b, f, fx["bf16_env"][k]))
    rows.sort(reverse=True)
    for r in rows[:8]:
        print(f"  {r[1]:45s} bf16 {r[2]:.3e}  fp16 {r[3]:.3e}  ratio {r[0]:.3f}  bf16_env {r[4]:.3e}")
    print("  median ratio", sorted(x[0] for x in rows)[len(rows) // 2])
