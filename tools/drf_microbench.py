"""Standalone timing of DRF's per-frame convs at the cfg-3 frame shape
(B = 4, 128 x 128 LR, F = 64, x4: ConvTranspose2d / Conv2d(8, 4, 2) as 3x3
sub-pixel convs over shuffle-4 views, drf_net.py:70-102) and its high-res
1x1 projections (drf_net.py:81-92), for A/B work and rocprofv3 --pmc passes.
Prints one line per case: mean us, TFLOP/s at the executed (3x3 sub-pixel)
FLOP and at the reference's (k x k strided) FLOP, and algorithmic TB/s."""
import argparse
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from vsr_amd import _native  # noqa: E402
from vsr_amd import functional as F  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--what", default="up,down,up_dgrad,down_dgrad,up_wgrad,down_wgrad,hr1x1,hr1x1_dgrad,hr1x1_wgrad,"
                                      "prelu_hr,prelu_lr")
    ap.add_argument("--paths", default="")
    args = ap.parse_args()
    _native.load()
    for kv in filter(None, args.paths.split(",")):
        p, m = kv.split("=")
        F.set_conv_path(p, int(m))
    dev, dt = "cuda", torch.bfloat16
    b, h, w, f, s, k, p, G = 4, 128, 128, 64, 4, 8, 2, 4
    H, W = h * s, w * s
    g = torch.Generator(device="cpu").manual_seed(0)

    def rnd(*shape):
        return torch.randn(shape, generator=g).to(dev, dt)

    lr = rnd(b, 1, h, w, f)                 # deconv input / strided-conv output gradient
    Hc = rnd(b, 1, H, W, G * f)             # high-res concat buffer
    dHc = rnd(b, 1, H, W, G * f)
    wt_up = torch.randn((f, f, k, k), generator=g).to(dev) * 0.05   # ConvTranspose2d weight (ci, co, k, k)
    wt_dn = torch.randn((f, f, k, k), generator=g).to(dev) * 0.05   # Conv2d weight (co, ci, k, k)
    bias = torch.randn(f, generator=g).to(dev)
    wq_up, bq_up = F.subpixel_conv_weight(wt_up, bias, k, s, p, True)
    wq_dn, bq_dn = F.subpixel_conv_weight(wt_dn, bias, k, s, p, False)
    pu0, pu1 = F.pack_weight(wq_up, 0, dt), F.pack_weight(wq_up, 1, dt)
    pd0, pd1 = F.pack_weight(wq_dn, 0, dt), F.pack_weight(wq_dn, 1, dt)
    K3, P1, K1, P0 = (1, 3, 3), (0, 1, 1), (1, 1, 1), (0, 0, 0)
    out_lr = torch.empty((b, 1, h, w, f), dtype=dt, device=dev)
    dweq_up = torch.empty((s * s * f, f, 1, 3, 3), device=dev)
    dbeq_up = torch.empty(s * s * f, device=dev)
    dweq_dn = torch.empty((f, s * s * f, 1, 3, 3), device=dev)
    dbeq_dn = torch.empty(f, device=dev)
    ci1 = G * f
    w1 = (torch.randn((f, ci1, 1, 1, 1), generator=g) / ci1 ** 0.5).to(dev)
    pw0, pw1 = F.pack_weight(w1, 0, dt), F.pack_weight(w1, 1, dt)
    hr_out = torch.empty((b, 1, H, W, f), dtype=dt, device=dev)
    dw1 = torch.empty((f, ci1, 1, 1, 1), device=dev)
    db1 = torch.empty(f, device=dev)
    slope = torch.tensor([0.2], device=dev)
    da = torch.zeros(1, device=dev)
    sub_flop = 2.0 * b * h * w * (s * s * f) * f * 9
    ref_flop = 2.0 * b * H * W * f * f * (k // s) ** 2  # the reference's strided / transposed conv
    pw_flop = 2.0 * b * H * W * ci1 * f
    cases = {
        # deconv forward: LR 64 -> HR slice of Hc through the shuffle-4 output view, PReLU
        "up": (lambda: F.conv(lr, pu0, Hc[..., f:2 * f], K3, P1, bias=bq_up, bias_r=1, y_shuffle=s,
                              act=F.ACT_PRELU, act_param=slope, subpixel=F.subpixel_code(k, s, p, True, False)), sub_flop,
               2.0 * b * (h * w * f + H * W * f)),
        # strided conv forward: HR slice through the shuffle-4 input view -> LR 64
        "down": (lambda: F.conv(Hc[..., f:2 * f], pd0, out_lr, K3, P1, bias=bq_dn, x_shuffle=s, act=F.ACT_PRELU,
                                act_param=slope, subpixel=F.subpixel_code(k, s, p, False, False)), sub_flop, 2.0 * b * (h * w * f + H * W * f)),
        "up_dgrad": (lambda: F.conv(dHc[..., f:2 * f], pu1, out_lr, K3, P1, x_shuffle=s,
                                    subpixel=F.subpixel_code(k, s, p, True, True)), sub_flop,
                     2.0 * b * (h * w * f + H * W * f)),
        "down_dgrad": (lambda: F.conv(lr, pd1, dHc[..., :f], K3, P1, y_shuffle=s, accumulate=True,
                                      subpixel=F.subpixel_code(k, s, p, False, True)), sub_flop,
                       2.0 * b * (h * w * f + 2 * H * W * f)),
        "up_wgrad": (lambda: F.conv_wgrad(lr, dHc[..., f:2 * f], K3, P1, dweq_up, dbeq_up, dy_shuffle=s,
                                          subpixel=F.subpixel_code(k, s, p, True, False)), sub_flop,
                     2.0 * b * (h * w * f + H * W * f)),
        "down_wgrad": (lambda: F.conv_wgrad(Hc[..., f:2 * f], lr, K3, P1, dweq_dn, dbeq_dn, x_shuffle=s,
                                            subpixel=F.subpixel_code(k, s, p, False, False)), sub_flop,
                       2.0 * b * (h * w * f + H * W * f)),
        # high-res 1x1 projection (G f -> f) and its data / weight gradient
        "hr1x1": (lambda: F.conv(Hc, pw0, hr_out, K1, P0, bias=bias, act=F.ACT_PRELU, act_param=slope), pw_flop,
                  2.0 * b * H * W * (ci1 + f)),
        "hr1x1_dgrad": (lambda: F.conv(hr_out, pw1, dHc, K1, P0, accumulate=True), pw_flop,
                        2.0 * b * H * W * (2 * ci1 + f)),
        "hr1x1_wgrad": (lambda: F.conv_wgrad(Hc, hr_out, K1, P0, dw1, db1), pw_flop, 2.0 * b * H * W * (ci1 + f)),
        # PReLU backward of an up projection's output (a 64-channel slice of the
        # high-res concat and of its gradient -> a dense buffer) and a low-res one
        "prelu_hr": (lambda: F.prelu_bwd(Hc[..., f:2 * f], dHc[..., f:2 * f], slope, hr_out, da, True), 0.0,
                     2.0 * b * H * W * 3 * f),
        "prelu_lr": (lambda: F.prelu_bwd(lr, lr, slope, out_lr, da, True), 0.0, 2.0 * b * h * w * 3 * f),
    }
    for name in args.what.split(","):
        fn, flop, nbytes = cases[name]
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        st.record()
        for _ in range(args.iters):
            fn()
        en.record()
        torch.cuda.synchronize()
        ms = st.elapsed_time(en) / args.iters
        extra = f"  ref-FLOP {ref_flop / ms / 1e9:7.1f} TF/s" if "1x1" not in name and flop else ""
        print(f"drf {name:12s} {ms * 1e3:8.1f} us  {flop / ms / 1e9:7.1f} TFLOP/s{extra}  "
              f"{nbytes / ms / 1e9:5.2f} TB/s", flush=True)


if __name__ == "__main__":
    main()
