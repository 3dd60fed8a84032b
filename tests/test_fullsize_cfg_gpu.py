"""Net-level parity at the sizes of BASELINE configs 3 and 5, and an fp32
train step at the config-2 size (tests/test_fullsize_gpu.py holds the bf16
config-2 step).

Every case runs one train step of the HIP generator and of the oracle
restatement (oracle/cpu_nets: the reference's algorithm, bitwise-pinned to it
by oracle/make_golden.py) in fp32 on the same device, with the same weights
and inputs, and compares the output, the PSNR of the denormalised output
(within 0.01 dB) and every parameter gradient (relative L2).

  * cfg 3 -- DSB15 VSR, DRF (drf_net.py:38-49) at B = 4, T = 30 frames of
    128 x 128, bf16, with the weight gradients on the side stream (the bench
    setting).  The loss covers all four samples; the oracle runs them one
    sequence at a time (no sample coupling in DRF) and accumulates.
    Bounds: output max |d| <= 3e-2, mean <= 3e-3;
    gradients rel-L2 worst <= 5e-2, median <= 3e-2; the scalar PReLU slopes
    (sums of cancelling terms over 30 frames) |d| <= 5e-2 x the largest slope
    gradient.
  * cfg 5 -- mixed ACDC + DSB15 (half the volumes each, per-volume
    normalisation constants), fp16, batch 8 per GPU: EDSR on 128 slices, DUF
    on 128 seven-frame windows (loss on the first 16 samples, oracle on
    those).  fp16 keeps 3 more significand bits than bf16: output max
    <= 1e-2, mean <= 1e-3; gradients worst <= 3e-2, median <= 1e-2.
  * fp32 at cfg 2 -- EDSR on 64 slices, DUF on 64 windows (loss on the first
    8 samples): the fp32 MFMA path against fp32 torch, different summation
    order only: output max |d| <= 1e-4, gradients worst <= 2e-3
    (a few parameters whose gradient is a near-cancelling sum), median <= 1e-4.
"""
import pytest
import torch
import torch.nn.functional as Fn

from oracle import cpu_nets
from vsr_amd import nets
from vsr_amd.data import cyclic_windows, synth_cine
from vsr_amd.metrics import psnr_denorm

pytestmark = pytest.mark.gpu
DEV = "cuda"
R = 4


def _grads(net):
    return {k: p.grad.detach().float() for k, p in net.named_parameters() if p.grad is not None}


def _compare(mine, ref, out, rout, y, dataset, omax, omean, gworst, gmed, sworst=0.1):
    d = (out.detach().float() - rout.detach()).abs()
    assert d.max().item() <= omax and d.mean().item() <= omean, (d.max().item(), d.mean().item())
    p_m = psnr_denorm(out.detach().float(), y, dataset).item()
    p_r = psnr_denorm(rout.detach(), y, dataset).item()
    assert abs(p_m - p_r) <= 0.01, (p_m, p_r)
    g_m, g_r = _grads(mine), _grads(ref)
    gmax = max(v.norm().item() for v in g_r.values())
    # A scalar PReLU slope's gradient is one sum over every voxel of a frame
    # sequence, of terms of both signs: its 16-bit error scales with the sum
    # of |terms|, not with the (cancelling) sum.  The slopes are held to an
    # absolute bound on the scale of the largest slope gradient instead.
    smax = max([v.abs().item() for v in g_r.values() if v.numel() == 1] or [0.0])
    rels = {}
    for k, gr in g_r.items():
        if gr.numel() == 1:
            assert (g_m[k] - gr).abs().item() <= sworst * smax, (k, g_m[k].item(), gr.item(), smax)
            continue
        if gr.norm().item() <= 1e-6 * gmax:  # exact gradient ~0 (conv bias before a BatchNorm)
            assert g_m[k].norm().item() <= 2e-2 * gmax, k
            continue
        rels[k] = (g_m[k] - gr).norm().item() / gr.norm().item()
    worst = max(rels.items(), key=lambda kv: kv[1])
    med = sorted(rels.values())[len(rels) // 2]
    print("output max / mean", d.max().item(), d.mean().item(), "worst / median gradient", worst, med)
    assert worst[1] <= gworst and med <= gmed, (worst, med)
    return worst, med


def _pair(cls_m, cls_r, kwargs, precision):
    torch.manual_seed(0)
    mine = cls_m(**kwargs).to(DEV).set_precision(precision).train()
    torch.manual_seed(0)
    ref = cls_r(**kwargs).to(DEV).train()
    ref.load_state_dict(mine.state_dict())
    return mine, ref


def test_cfg3_drf_t30_bf16():
    B, T, H, W = 4, 30, 128, 128
    lr, hr = synth_cine(B, T, H, W, R, "dsb15", seed=77, device=DEV)
    kwargs = dict(in_channels=1, out_channels=1, num_features=64, num_groups=4, upscale_factor=R)
    mine, ref = _pair(nets.DRFNet, cpu_nets.DRFRef, kwargs, "bf16")
    mine.overlap_wgrad = True  # side-stream weight gradients, as the bench runs DRF
    x = [lr[:, t:t + 1] for t in range(T)]
    y = [hr[:, t:t + 1] for t in range(T)]
    outs = mine(x)
    torch.stack([Fn.l1_loss(o, t) for o, t in zip(outs, y)]).mean().backward()
    # the oracle one sequence at a time (DRF couples no samples): the loss over
    # all B samples is the mean of the per-sample losses, so each run's
    # backward carries 1 / B and the gradients accumulate
    routs = []
    with torch.backends.cudnn.flags(enabled=False):
        for i in range(B):
            ro = ref([v[i:i + 1] for v in x])
            (torch.stack([Fn.l1_loss(o, t[i:i + 1]) for o, t in zip(ro, y)]).mean() / B).backward()
            routs.append(torch.stack([o.detach() for o in ro]))
    torch.cuda.synchronize()
    out = torch.stack(outs)
    rout = torch.cat(routs, dim=1)
    stats = _compare(mine, ref, out, rout, torch.stack(y), "dsb15", 3e-2, 3e-3, 5e-2, 3e-2, sworst=5e-2)
    print("cfg3 drf worst / median gradient", stats)


def _mixed(B, T, H, W, seed):
    la, ha = synth_cine(B - B // 2, T, H, W, R, "acdc", seed=seed, device=DEV)
    lb, hb = synth_cine(B // 2, T, H, W, R, "dsb15", seed=seed + 1, device=DEV)
    return torch.cat([la, lb]), torch.cat([ha, hb])


@pytest.mark.parametrize("model", ["edsr", "duf"])
def test_cfg5_fp16_batch8(model):
    B, T, H, W = 8, 16, 128, 128
    lr, hr = _mixed(B, T, H, W, 5)
    n = 16  # samples in the loss (ACDC volume 0); the kernels run all B*T = 128
    if model == "edsr":
        kwargs = dict(in_channels=1, out_channels=1, num_resblocks=16, num_features=64, upscale_factor=R)
        mine, ref = _pair(nets.EDSRNet, cpu_nets.EDSRRef, kwargs, "fp16")
        x, y = lr.reshape(B * T, 1, H, W), hr.reshape(B * T, 1, H * R, W * R)
        xr = x[:n]
    else:
        kwargs = dict(in_channels=1, out_channels=1, num_frames=7, size_filter=5, upscale_factor=R,
                      backbone="_DenseLayer16")
        mine, ref = _pair(nets.DUFNet, cpu_nets.DUFRef, kwargs, "fp16")
        mine.eval(), ref.eval()  # BatchNorm couples the batch: compare with running statistics
        x, y = cyclic_windows(lr, 7), hr.reshape(B * T, 1, H * R, W * R)
        xr = [v[:n] for v in x]
    out = mine(x)
    Fn.l1_loss(out[:n], y[:n]).backward()
    assert mine.step_ok()  # no fp16 overflow at the automatic scale
    with torch.backends.cudnn.flags(enabled=False):
        rout = ref(xr)
        Fn.l1_loss(rout, y[:n]).backward()
    torch.cuda.synchronize()
    _compare(mine, ref, out[:n], rout, y[:n], "acdc", 1e-2, 1e-3, 3e-2, 1e-2)


@pytest.mark.parametrize("model", ["edsr", "duf"])
def test_cfg2_fp32_step(model):
    B, T, H, W = 4, 16, 128, 128
    lr, hr = synth_cine(B, T, H, W, R, seed=1234, device=DEV)
    n = 8
    if model == "edsr":
        kwargs = dict(in_channels=1, out_channels=1, num_resblocks=16, num_features=64, upscale_factor=R)
        mine, ref = _pair(nets.EDSRNet, cpu_nets.EDSRRef, kwargs, "fp32")
        x, y = lr.reshape(B * T, 1, H, W), hr.reshape(B * T, 1, H * R, W * R)
        xr = x[:n]
    else:
        kwargs = dict(in_channels=1, out_channels=1, num_frames=7, size_filter=5, upscale_factor=R,
                      backbone="_DenseLayer16")
        mine, ref = _pair(nets.DUFNet, cpu_nets.DUFRef, kwargs, "fp32")
        mine.eval(), ref.eval()
        x, y = cyclic_windows(lr, 7), hr.reshape(B * T, 1, H * R, W * R)
        xr = [v[:n] for v in x]
    out = mine(x)
    Fn.l1_loss(out[:n], y[:n]).backward()
    with torch.backends.cudnn.flags(enabled=False):
        torch.backends.cuda.matmul.allow_tf32 = False
        rout = ref(xr)
        Fn.l1_loss(rout, y[:n]).backward()
    torch.cuda.synchronize()
    _compare(mine, ref, out[:n], rout, y[:n], "acdc", 1e-4, 1e-5, 2e-3, 1e-4)
