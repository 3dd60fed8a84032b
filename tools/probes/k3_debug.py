"""Where does the k3 conv differ from the fp64 reference? (error map by channel / column / row)"""
import sys
from pathlib import Path

import torch
import torch.nn.functional as Fn

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
from vsr_amd import _native  # noqa: E402
from vsr_amd import functional as F  # noqa: E402

_native.load()
n, d, h, w, ci, co = 2, 1, 13, 37, 16, 32
g = torch.Generator().manual_seed(0)
x = torch.randn((n, d, h, w, ci), generator=g)
wt = torch.randn((co, ci, 1, 3, 3), generator=g) / 12
b = torch.zeros(co)
ref = Fn.conv3d(x.to(torch.bfloat16).double().permute(0, 4, 1, 2, 3), wt.to(torch.bfloat16).double(), b.double(),
                padding=(0, 1, 1)).permute(0, 2, 3, 4, 1)
for mode in (0, 1):
    F.set_conv_path("k3", mode)
    y = torch.zeros((n, d, h, w, co), dtype=torch.bfloat16, device="cuda")
    F.conv(x.to("cuda", torch.bfloat16), F.pack_weight(wt.cuda(), 0, torch.bfloat16), y, (1, 3, 3), (0, 1, 1),
           bias=b.cuda())
    err = (y.cpu().double() - ref).abs()
    print(f"k3={mode}: max err {err.max().item():.3f}")
    if err.max() > 0.1:
        print(" per channel:", [round(v, 2) for v in err.amax(dim=(0, 1, 2, 3)).tolist()])
        print(" per column:", [round(v, 2) for v in err.amax(dim=(0, 1, 2, 4)).tolist()])
        print(" per row:", [round(v, 2) for v in err.amax(dim=(0, 1, 3, 4)).tolist()])
        yy = y.cpu().double()
        # is the output a channel permutation of the reference?
        for c in range(4):
            dif = (yy[..., c:c + 1] - ref).abs().amax(dim=(0, 1, 2, 3))
            print(f"  y channel {c} best matches ref channel {int(dif.argmin())} (err {dif.min().item():.3f})")
        print("  y[0,0,5,5,:8]", [round(v, 2) for v in yy[0, 0, 5, 5, :8].tolist()])
        print("  r[0,0,5,5,:8]", [round(v, 2) for v in ref[0, 0, 5, 5, :8].tolist()])
