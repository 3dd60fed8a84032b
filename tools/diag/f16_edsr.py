"""EDSR: fp16 / bf16 gradients vs the fp32 HIP path, and fp32 HIP vs fp64 fixture (diagnostic)."""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
from tests.conftest import load_golden  # noqa: E402
from tests.test_nets_gpu import _build, _l1, _rel, _to  # noqa: E402

name = sys.argv[1]
fx = load_golden(name)
res = {}
for prec in ("fp32", "bf16", "fp16"):
    net = _build(fx, prec)
    out = net(_to(fx["lr"]))
    _l1(out, _to(fx["hr"])).backward()
    res[prec] = {k: p.grad.detach().double().cpu().clone() for k, p in net.named_parameters()}
rows = []
for k in res["fp32"]:
    if fx["ref32_err"][k] is None:
        continue
    r = res["fp32"][k]
    e16 = ((res["fp16"][k] - r).norm() / r.norm()).item()
    eb = ((res["bf16"][k] - r).norm() / r.norm()).item()
    rows.append((e16, k, eb, _rel(res["fp16"][k], fx, k), _rel(r, fx, k), fx["fp16_env"][k]))
rows.sort(reverse=True)
for e16, k, eb, e16_64, e32_64, env in rows[:10]:
    print(f"{k:36s} fp16-vs-fp32 {e16:.2e} bf16-vs-fp32 {eb:.2e} | fp16-vs-fp64 {e16_64:.2e} fp32-vs-fp64 {e32_64:.2e} env16 {env:.2e}")
