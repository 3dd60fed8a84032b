"""fp16 gradient error vs loss scale for one fixture (diagnostic)."""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
from tests.conftest import load_golden  # noqa: E402
from tests.test_nets_gpu import _build, _l1, _rel, _to  # noqa: E402

name = sys.argv[1]
keys = sys.argv[2].split(",")
fx = load_golden(name)
for sc in [1.0, 2.0 ** 6, 2.0 ** 10, 2.0 ** 14, 2.0 ** 18, None]:
    net = _build(fx, "fp16")
    net.loss_scale = sc
    out = net(_to(fx["lr"]))
    _l1(out, _to(fx["hr"])).backward()
    g = dict(net.named_parameters())
    errs = [_rel(g[k].grad.detach().cpu().double(), fx, k) for k in keys]
    fin = all(p.grad.isfinite().all().item() for p in net.parameters())
    print(f"scale {sc}: finite {fin} " + " ".join(f"{k}={e:.3e}" for k, e in zip(keys, errs)), flush=True)
