"""DRF fp16 vs bf16 in_block gradient error with / without the thin kernels (diagnostic)."""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
from tests.conftest import load_golden  # noqa: E402
from tests.test_nets_gpu import _build, _l1, _rel, _to  # noqa: E402
from vsr_amd import functional as F  # noqa: E402

name = sys.argv[1]
keys = ["in_block.conv1.weight", "in_block.conv2.weight", "in_block.prelu1.weight", "out_block.conv3.weight",
        "f_block.in_block.conv.weight"]
fx = load_golden(name)
for prec in ("bf16", "fp16"):
    for paths in ({}, {"thin": 0}, {"pw": 0}, {"fast": 0}):
        for p, m in paths.items():
            F.set_conv_path(p, m)
        net = _build(fx, prec)
        out = net(_to(fx["lr"]))
        _l1(out, _to(fx["hr"])).backward()
        g = dict(net.named_parameters())
        errs = [_rel(g[k].grad.detach().cpu().double(), fx, k) for k in keys]
        print(prec, paths, " ".join(f"{k.split('.')[0]}.{k.split('.')[-2]}={e:.2e}" for k, e in zip(keys, errs)),
              flush=True)
        for p in paths:
            F.set_conv_path(p, -1)
