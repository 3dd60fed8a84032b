"""Count ReLU-mask disagreements between the HIP fp32 DUF forward and the
fp64 oracle at the filter/residual heads (diagnostic for gradient parity).

    python tools/duf_mask_flips.py
"""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from oracle import cpu_nets  # noqa: E402
from tests.conftest import load_golden  # noqa: E402
from tests.test_nets_gpu import _build  # noqa: E402

fx = load_golden("duf_x4_canon")
net = _build(fx, "fp32")
tape = {}
net._run([t.cuda() for t in fx["lr"]], tape)
torch.cuda.synchronize()

torch.manual_seed(fx["seed"])
ref = cpu_nets.DUFRef(**fx["kwargs"])
ref.load_state_dict({k: v.detach().cpu() for k, v in net.state_dict().items()})
ref = ref.double().train()
cap = {}
ref.filterNet.conv1.register_forward_hook(lambda m, i, o: cap.__setitem__("h1", o.detach()))
ref.residualNet.conv1.register_forward_hook(lambda m, i, o: cap.__setitem__("r1", o.detach()))
ref([t.double() for t in fx["lr"]])
for key in ("h1", "r1"):
    pre = cap[key][:, :, 0].permute(0, 2, 3, 1)  # (n,h,w,c) pre-activation, fp64
    ours = tape[key][:, 0].double().cpu()        # post-ReLU, fp32 kernel
    flips = ((pre > 0) != (ours > 0))
    nf = int(flips.sum())
    print(f"{key}: {pre.numel()} elements, {nf} mask flips; min |pre| = {pre.abs().min().item():.3e}")
    if nf:
        print("   |pre| at flips:", pre[flips][:10].tolist())
