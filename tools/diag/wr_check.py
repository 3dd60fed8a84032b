"""Forced resident-weight (WR) 2-D roll form vs the streamed-weight kernel on
the prefetched residual / mask epilogues: where they differ, print both
outputs and the fp64 reference (a rounding flip of the fp32 sum, or a wrong
operand?)."""
import sys

import torch

sys.path.insert(0, ".")  # run from the repo root
sys.path.insert(0, "tests")
import test_roll_gpu as T  # noqa: E402
from vsr_amd import functional as F  # noqa: E402

for case in [(3, 1, 20, 40, 64, 64)]:
    for epi in ["res", "mask"]:
        outs = {}
        for wr in (0, 2):
            F.set_conv_path("roll_wr", wr)
            outs[wr], ref = T._run2d(case, torch.bfloat16, epi)
        F.set_conv_path("roll_wr", -1)
        d = (outs[2] - outs[0]).abs()
        idx = (d > 0).nonzero()
        print(case, epi, "ndiff", idx.shape[0], flush=True)
        for r in idx[:12].tolist():
            n, dd, h, w, c = r
            print("   ", r, "streamed", float(outs[0][n, dd, h, w, c]), "wr", float(outs[2][n, dd, h, w, c]),
                  "ref", float(ref[n, dd, h, w, c]))
