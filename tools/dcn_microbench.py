"""Timing of the DCNv2 op at EDVR's alignment shape (64 ch, 3x3, 8 deformable
groups) on 4 x 128 x 128 frames: forward and forward+backward, HIP events."""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from vsr_amd import dcn  # noqa: E402


def main():
    n, c, h, w, co, dg = 4, 64, 128, 128, 64, 8
    g = torch.Generator(device="cpu").manual_seed(0)
    x = torch.randn((n, c, h, w), generator=g).cuda().requires_grad_(True)
    off = (torch.randn((n, dg * 18, h, w), generator=g) * 2).cuda().requires_grad_(True)
    m = torch.rand((n, dg * 9, h, w), generator=g).cuda().requires_grad_(True)
    wt = (torch.randn((co, c, 3, 3), generator=g) * 0.05).cuda().requires_grad_(True)
    b = torch.zeros(co).cuda().requires_grad_(True)
    gy = torch.randn((n, co, h, w), generator=g).cuda()
    flop = 2.0 * n * h * w * co * c * 9

    def fwd():
        return dcn.modulated_deform_conv(x, off, m, wt, b, 1, 1, 1, 1, dg)

    def fwdbwd():
        fwd().backward(gy)

    for name, fn, f in (("fwd", fwd, flop), ("fwd+bwd", fwdbwd, 3 * flop)):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(10):
            fn()
        e.record()
        torch.cuda.synchronize()
        ms = s.elapsed_time(e) / 10
        print(f"dcnv2 {n}x{c}x{h}x{w} dg{dg} {name:8s} {ms * 1e3:9.1f} us  {f / ms / 1e9:7.1f} TFLOP/s (conv FLOP)",
              flush=True)


if __name__ == "__main__":
    main()
