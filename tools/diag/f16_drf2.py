"""DRF: fp16 / bf16 gradients vs the fp32 HIP path for small configs (diagnostic)."""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
from vsr_amd import nets  # noqa: E402

dev = "cuda"
for T, G in [(1, 1), (2, 1), (1, 2), (3, 3)]:
    g = torch.Generator().manual_seed(3)
    lr = [torch.randn(2, 1, 8, 12, generator=g).to(dev) for _ in range(T)]
    hr = [torch.randn(2, 1, 32, 48, generator=g).to(dev) for _ in range(T)]
    res = {}
    for prec in ("fp32", "bf16", "fp16"):
        torch.manual_seed(7)
        net = nets.DRFNet(1, 1, 64, G, 4).to(dev).set_precision(prec).train()
        out = net(lr)
        torch.stack([torch.nn.functional.l1_loss(o, t) for o, t in zip(out, hr)]).mean().backward()
        res[prec] = {k: p.grad.detach().double().clone() for k, p in net.named_parameters()}
    ref = res["fp32"]
    print(f"T={T} G={G}")
    for k in ["in_block.conv1.weight", "in_block.conv2.weight", "in_block.prelu2.weight", "f_block.in_block.conv.weight",
              "out_block.conv3.weight"]:
        e = {p: ((res[p][k] - ref[k]).norm() / ref[k].norm()).item() for p in ("bf16", "fp16")}
        print(f"   {k:32s} bf16 {e['bf16']:.2e}  fp16 {e['fp16']:.2e}", flush=True)
