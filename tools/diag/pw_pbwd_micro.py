"""Timing of the pointwise data gradient's PReLU-backward forms (DRF's
dHc / dL producers, round 5): plain, accumulate, and the post-accumulate
PReLU backward on the tail channels, against the separate prelu_bwd pass."""
import sys

import torch

sys.path.insert(0, ".")  # run from the repo root
from vsr_amd import functional as F  # noqa: E402


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    dev, dt = "cuda", torch.bfloat16
    for (b, h, w, cout) in ((4, 512, 512, 256), (4, 128, 128, 256)):
        x = torch.randn((b, 1, h, w, 64), device=dev).to(dt)
        big = torch.randn((b, 1, h, w, cout), device=dev).to(dt)
        y = big.clone()
        mask = torch.randn((b, 1, h, w, cout), device=dev).to(dt)
        wp = F.pack_weight(torch.randn((64, cout, 1, 1, 1), device=dev) * 0.1, 1, dt)
        a = torch.tensor([0.2], device=dev)
        da = torch.zeros(1, device=dev)
        K, P = (1, 1, 1), (0, 0, 0)
        c_lo = cout - 64
        res = {
            "plain": timeit(lambda: F.conv(x, wp, y, K, P)),
            "acc": timeit(lambda: F.conv(x, wp, y, K, P, accumulate=True)),
            "pbwd": timeit(lambda: F.conv_prelu_bwd(x, wp, y, K, P, mask, a, da, True, c_lo=c_lo)),
            "pbwd_acc": timeit(lambda: F.conv_prelu_bwd(x, wp, y, K, P, mask, a, da, True, accumulate=True,
                                                        c_lo=c_lo)),
            "pbwd_all": timeit(lambda: F.conv_prelu_bwd(x, wp, y, K, P, mask, a, da, True, c_lo=0)),
            "prelu_bwd_tail": timeit(lambda: F.prelu_bwd(mask[..., c_lo:], y[..., c_lo:], a, y[..., c_lo:], da, True)),
        }
        print((b, h, w, cout), {k: round(v, 1) for k, v in res.items()}, flush=True)


if __name__ == "__main__":
    main()
