"""k3 conv mapping experiments: sparse weights reveal how couts / cin / taps map."""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
from vsr_amd import _native  # noqa: E402
from vsr_amd import functional as F  # noqa: E402

_native.load()
torch.set_printoptions(linewidth=200, precision=2)
n, d, h, w = 1, 1, 16, 32
for ci, co in ((16, 32), (64, 64)):
    x = torch.zeros((n, d, h, w, ci))
    x[0, 0, 5, 7, :] = torch.arange(1, ci + 1).float()  # one voxel, channel c holds c+1
    for label, wfill in (("cout5 all-ones", "c5"), ("identity centre tap", "id")):
        wt = torch.zeros((co, ci, 1, 3, 3))
        if wfill == "c5":
            wt[5, :, 0, 1, 1] = 1.0
        else:
            for c in range(co):
                wt[c, c % ci, 0, 1, 1] = 1.0
        y = torch.zeros((n, d, h, w, co), dtype=torch.bfloat16, device="cuda")
        F.conv(x.to("cuda", torch.bfloat16), F.pack_weight(wt.cuda(), 0, torch.bfloat16), y, (1, 3, 3), (0, 1, 1))
        yy = y.float().cpu()[0, 0]
        nz = (yy != 0).nonzero().tolist()
        print(f"ci={ci} co={co} {label}: {len(nz)} nonzero; first: {nz[:6]}")
        print("  y[5,7,:16] =", yy[5, 7, :16].tolist())
        if wfill == "id":
            print("  expected    =", [(c % ci) + 1.0 for c in range(16)])
