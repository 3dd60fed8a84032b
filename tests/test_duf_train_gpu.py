"""Train-mode DUF (duf_net.py:51-99, dense units duf_net.py:195-214) through
the fused kernels, at the BASELINE sizes.

  * The bench's north-star timer sees every Conv3d 3x3x3 launch of a step,
    fused or not: 6 forward, 6 data-gradient (the fused BN-reduce form,
    F.conv_reduce) and 6 weight-gradient launches, the same 18 with
    VSRK_FUSE off.
  * cfg 2 (64 seven-frame windows of 128 x 128, bf16): one train step with
    the fused forms (BN statistics in conv1's store pass, bn1 / bn2 backward
    reduces in the data gradients' store pass) against the same step with
    the separate kernels.  Both are the same arithmetic up to fp32 summation
    order of the per-channel sums, which moves a few bf16 roundings
    downstream: output max |d| <= 2e-2 and mean <= 1e-3 (a tenth of the bf16
    storage bound against fp32), every parameter
    gradient within 1e-2 rel-L2 (the conv biases whose consumers are all
    BatchNorms have exact gradient 0: both runs hold rounding noise there,
    held to 2e-2 of the largest gradient), running statistics within 1e-5
    relative.
  * cfg 5 (fp16, batch 8: 128 windows) and cfg 4 (two uncropped 30-frame
    64 x 64 volumes: 60 windows, bf16) in train mode against the oracle
    restatement (oracle/cpu_nets, fp32, the same device) on the FULL batch --
    BatchNorm couples the samples, so no subset is taken.  Bounds as
    tests/test_fullsize_cfg_gpu.py for fp16 (output max <= 1e-2, mean <= 1e-3,
    gradients worst <= 3e-2, median <= 1e-2) and tests/test_fullsize_gpu.py
    for bf16 (output max <= 3e-2, mean <= 3e-3, worst <= 0.1, median <= 3e-2);
    PSNR within 0.01 dB; running statistics within 2e-2 (bf16) / 5e-3 (fp16).
"""
import pytest
import torch
import torch.nn.functional as Fn

from oracle import cpu_nets
from vsr_amd import functional as F
from vsr_amd import nets
from vsr_amd.data import cyclic_windows, synth_cine
from vsr_amd.metrics import psnr_denorm

pytestmark = pytest.mark.gpu
DEV = "cuda"
R = 4
KW = dict(in_channels=1, out_channels=1, num_frames=7, size_filter=5, upscale_factor=R, backbone="_DenseLayer16")


def _grads(net):
    return {k: p.grad.detach().float().clone() for k, p in net.named_parameters() if p.grad is not None}


def _running(net):
    return {k: v.detach().float().clone() for k, v in net.state_dict().items() if "running" in k}


def _step(net, x, y, timer=None):
    if timer is not None:
        F.timer = timer
    try:
        if timer is not None:
            timer.phase = "fwd"
        out = net(x)
        if timer is not None:
            timer.phase = "bwd"
        Fn.l1_loss(out, y).backward()
    finally:
        F.timer = None
    torch.cuda.synchronize()
    return out.detach()


def _with_fuse(on):
    class _Ctx:
        def __enter__(self):
            self.old = F.FUSE
            F.FUSE = on

        def __exit__(self, *a):
            F.FUSE = self.old
    return _Ctx()


def _match3(kind, xv, yv):
    return 1 if kind[1] == (3, 3, 3) else 0


@pytest.mark.parametrize("precision", ["bf16", "fp16"])
def test_north_star_timer_sees_every_3x3x3_launch(precision):
    lr, hr = synth_cine(2, 7, 24, 40, R, seed=3, device=DEV)
    x, y = cyclic_windows(lr, 7), hr.reshape(14, 1, 24 * R, 40 * R)
    counts = {}
    for fuse in (True, False):
        torch.manual_seed(0)
        net = nets.DUFNet(**KW).to(DEV).set_precision(precision).train()
        tm = F.KernelTimer(_match3)
        with _with_fuse(fuse):
            _step(net, x, y, tm)
        counts[fuse] = {lab: tm.totals(lab)[2] for lab in ("fwd", "dgrad", "wgrad")}
    assert counts[True] == counts[False] == {"fwd": 6, "dgrad": 6, "wgrad": 6}, counts


def test_cfg2_fused_vs_unfused_train_step():
    B, T, H, W = 4, 16, 128, 128
    lr, hr = synth_cine(B, T, H, W, R, seed=1234, device=DEV)
    x, y = cyclic_windows(lr, 7), hr.reshape(B * T, 1, H * R, W * R)
    res = {}
    for fuse in (True, False):
        torch.manual_seed(0)
        net = nets.DUFNet(**KW).to(DEV).set_precision("bf16").train()
        with _with_fuse(fuse):
            out = _step(net, x, y)
        res[fuse] = (out, _grads(net), _running(net))
        del net
        torch.cuda.empty_cache()
    (o1, g1, r1), (o0, g0, r0) = res[True], res[False]
    d = (o1 - o0).abs()
    assert d.max().item() <= 2e-2 and d.mean().item() <= 1e-3, (d.max().item(), d.mean().item())
    gmax = max(v.norm().item() for v in g0.values())
    worst = (None, 0.0)
    for k, g in g0.items():
        if k == "head.bias" or (k.startswith("denseLayer.conv") and k.endswith(("conv1.bias", "conv2.bias"))):
            # a conv bias whose every consumer is a BatchNorm: exact gradient 0,
            # both runs hold bf16 rounding noise there
            assert g1[k].norm().item() <= 2e-2 * gmax and g.norm().item() <= 2e-2 * gmax, k
            continue
        rel = (g1[k] - g).norm().item() / g.norm().item()
        worst = max(worst, (k, rel), key=lambda kv: kv[1])
    assert worst[1] <= 1e-2, worst
    for k, v in r0.items():
        assert (r1[k] - v).abs().max().item() <= 1e-5 * (1 + v.abs().max().item()), k


def _vs_oracle(precision, lr, hr, dataset, omax, omean, gworst, gmed, rtol):
    n = lr.shape[0] * lr.shape[1]
    h, w = lr.shape[2], lr.shape[3]
    x, y = cyclic_windows(lr, 7), hr.reshape(n, 1, h * R, w * R)
    torch.manual_seed(0)
    mine = nets.DUFNet(**KW).to(DEV).set_precision(precision).train()
    torch.manual_seed(0)
    ref = cpu_nets.DUFRef(**KW).to(DEV).train()
    ref.load_state_dict(mine.state_dict())
    out = mine(x)
    Fn.l1_loss(out, y).backward()
    if precision == "fp16":
        assert mine.step_ok()
    with torch.backends.cudnn.flags(enabled=False):
        torch.backends.cuda.matmul.allow_tf32 = False
        rout = ref(x)
        Fn.l1_loss(rout, y).backward()
    torch.cuda.synchronize()
    d = (out.detach().float() - rout.detach()).abs()
    assert d.max().item() <= omax and d.mean().item() <= omean, (d.max().item(), d.mean().item())
    p_m = psnr_denorm(out.detach().float(), y, dataset).item()
    p_r = psnr_denorm(rout.detach(), y, dataset).item()
    assert abs(p_m - p_r) <= 0.01, (p_m, p_r)
    g_m, g_r = _grads(mine), _grads(ref)
    gmax = max(v.norm().item() for v in g_r.values())
    rels = {}
    for k, gr in g_r.items():
        if gr.norm().item() <= 1e-6 * gmax:
            assert g_m[k].norm().item() <= 2e-2 * gmax, k
            continue
        rels[k] = (g_m[k] - gr).norm().item() / gr.norm().item()
    worst = max(rels.items(), key=lambda kv: kv[1])
    med = sorted(rels.values())[len(rels) // 2]
    print("output max / mean", d.max().item(), d.mean().item(), "worst / median gradient", worst, med)
    assert worst[1] <= gworst and med <= gmed, (worst, med)
    rm, rr = _running(mine), _running(ref)
    for k, v in rr.items():
        assert (rm[k] - v).abs().max().item() <= rtol * (1 + v.abs().max().item()), k


def test_cfg5_fp16_duf_train_full_batch():
    B, T, H, W = 8, 16, 128, 128
    la, ha = synth_cine(B - B // 2, T, H, W, R, "acdc", seed=5, device=DEV)
    lb, hb = synth_cine(B // 2, T, H, W, R, "dsb15", seed=6, device=DEV)
    lr, hr = torch.cat([la, lb]), torch.cat([ha, hb])
    _vs_oracle("fp16", lr, hr, "acdc", 1e-2, 1e-3, 3e-2, 1e-2, 5e-3)


def test_cfg4_duf_full_volumes_train():
    # bench.py cfg4: two uncropped 30-frame volumes of 64 x 64 LR (256 x 256 HR)
    lr, hr = synth_cine(2, 30, 64, 64, R, "acdc", seed=44, device=DEV)
    _vs_oracle("bf16", lr, hr, "acdc", 3e-2, 3e-3, 5e-2, 3e-2, 2e-2)
