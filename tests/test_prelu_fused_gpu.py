"""DRF's PReLU backwards fused into the data gradient that completes their
input gradient (drf_net.py:55-106): vsrk_conv_fwd_prelu_bwd
with an accumulate (the gradient is a sum; the PReLU backward sees the whole
sum) and with c_lo (the PReLU owns the tail channels of a concat gradient --
the 1x1 projections' data gradients write every earlier slice too).

Against the unfused pair (conv [accumulate], then prelu_bwd on the tail):
channels below c_lo bitwise equal (the same kernel epilogue minus the mask),
the tail within one bf16 rounding (the fused form skips the rounding of the
sum before the mask), the slope gradient against the one recomputed in double
from the fused output and against the unfused one within an output ulp per
term (see test_roll_gpu.test_roll_prelu_bwd_fused).  Net level: the DRF
backward at f = 64 (every fused site eligible) against the same net with
fusion off, and its prelu_bwd launches (2 per frame left: gout, gin)."""
import pytest
import torch
import torch.nn.functional as Fn

from vsr_amd import functional as F
from vsr_amd import nets

pytestmark = pytest.mark.gpu
DEV = "cuda"
DT = torch.bfloat16
PROJ = {4: (8, 4, 2)}


def _check(y, y_ref, y_fwd, c_lo, a, da, da_ref, base):
    assert torch.equal(y[..., :c_lo], y_ref[..., :c_lo])
    yt, rt, m = y[..., c_lo:].float(), y_ref[..., c_lo:].float(), y_fwd[..., c_lo:].double()
    assert (yt - rt).abs().max().item() <= 1e-2 * rt.abs().max().item()
    neg = m < 0
    cond = (rt.double() * m)[neg].abs().sum().item() / a ** 2
    own = base + (yt.double() * m)[neg].sum().item() / a ** 2
    assert abs(da.item() - own) <= 1e-4 * cond + 1e-3, (da.item(), own)
    assert abs(da.item() - da_ref.item()) <= 2 ** -7 * cond, (da.item(), da_ref.item(), cond)


@pytest.mark.parametrize("acc", [False, True])
@pytest.mark.parametrize("cout,c_lo", [(64, 0), (256, 0), (128, 64), (256, 192), (192, 128),
                                       # tails not on a 64-channel group boundary (num_features 48):
                                       # the generic per-chunk store pass, not the grouped forms
                                       (192, 144), (128, 40)])
@pytest.mark.parametrize("acc_da", [False, True])
def test_pw_prelu_bwd_tail(acc, cout, c_lo, acc_da):
    """the 1x1 data gradient 64 -> cout into a channel slice of a wider
    buffer (DRF's dL[..., f:] / dHc[..., :(i+1) f]), PReLU backward on its
    last cout - c_lo channels"""
    g = torch.Generator().manual_seed(cout + c_lo + acc)
    n, h, w, ci = 2, 17, 45, 64
    x = torch.randn((n, 1, h, w, ci), generator=g).to(DEV, DT)
    wt = torch.randn((ci, cout, 1, 1, 1), generator=g) / ci ** 0.5  # forward weight of a cout -> ci conv
    wp = F.pack_weight(wt.to(DEV), 1, DT)
    big_fwd = torch.randn((n, 1, h, w, cout + 64), generator=g).to(DEV, DT)
    y_fwd = big_fwd[..., 64:]
    old = torch.randn((n, 1, h, w, cout + 64), generator=g).to(DEV, DT)
    a = 0.2
    at = torch.tensor([a], device=DEV)
    da0 = torch.tensor([0.5], device=DEV)
    y_ref_b = old.clone()
    y_ref = y_ref_b[..., 64:]
    F.conv(x, wp, y_ref, (1, 1, 1), (0, 0, 0), accumulate=acc)
    da_ref = da0.clone()
    F.prelu_bwd(y_fwd[..., c_lo:], y_ref[..., c_lo:], at, y_ref[..., c_lo:], da_ref, acc_da)
    outs = []
    for _ in range(2):
        yb = old.clone()
        da = da0.clone()
        assert F.conv_prelu_bwd(x, wp, yb[..., 64:], (1, 1, 1), (0, 0, 0), y_fwd, at, da, acc_da, accumulate=acc,
                                c_lo=c_lo)
        outs.append((yb, da))
    yb, da = outs[0]
    assert torch.equal(outs[1][0], yb) and torch.equal(outs[1][1], da)
    assert torch.equal(yb[..., :64], old[..., :64])  # outside the view: untouched
    _check(yb[..., 64:], y_ref, y_fwd, c_lo, a, da, da_ref, da0.item() if acc_da else 0.0)


@pytest.mark.parametrize("form", ["up_dgrad", "down_dgrad"])
def test_roll_prelu_bwd_after_accumulate(form):
    """DRF's sub-pixel data gradients that complete a gradient sum: down
    projection 0's into dHc[..., :f] (y through a shuffle-4 view) and up
    projection 0's into dL[..., :f] (x through the view), the consumer's
    PReLU backward applied to old + conv"""
    g = torch.Generator().manual_seed(3 + (form == "up_dgrad"))
    f, n, h, w, r = 64, 2, 11, 29, 4
    k, s, p = PROJ[r]
    tr = form == "up_dgrad"
    wt = torch.randn((f, f, k, k), generator=g) / (f * k) ** 0.5
    weq, _ = F.subpixel_conv_weight(wt.to(DEV), None, k, s, p, transposed=tr)
    wp = F.pack_weight(weq, 1, DT)
    code = F.subpixel_code(k, s, p, tr, True)
    if tr:
        x = torch.randn((n, 1, h * s, w * s, f), generator=g).to(DEV, DT)
        kw, yshape = dict(x_shuffle=s, subpixel=code), (n, 1, h, w, f)
    else:
        x = torch.randn((n, 1, h, w, f), generator=g).to(DEV, DT)
        kw, yshape = dict(y_shuffle=s, subpixel=code), (n, 1, h * s, w * s, f)
    y_fwd = torch.randn(yshape, generator=g).to(DEV, DT)
    old = torch.randn(yshape, generator=g).to(DEV, DT)
    a = 0.2
    at = torch.tensor([a], device=DEV)
    y_ref = old.clone()
    F.conv(x, wp, y_ref, (1, 3, 3), (0, 1, 1), accumulate=True, **kw)
    da_ref = torch.zeros(1, device=DEV)
    F.prelu_bwd(y_fwd, y_ref, at, y_ref, da_ref, False)
    y = old.clone()
    da = torch.zeros(1, device=DEV)
    assert F.conv_prelu_bwd(x, wp, y, (1, 3, 3), (0, 1, 1), y_fwd, at, da, False, accumulate=True, **kw)
    _check(y, y_ref, y_fwd, 0, a, da, da_ref, 0.0)


def _drf_grads(monkeypatch, fuse):
    monkeypatch.setattr(F, "FUSE", fuse)
    calls = []
    real = F.prelu_bwd
    monkeypatch.setattr(F, "prelu_bwd", lambda *a_, **k_: (calls.append(1), real(*a_, **k_))[1])
    torch.manual_seed(0)
    net = nets.DRFNet(in_channels=1, out_channels=1, num_features=64, num_groups=3,
                      upscale_factor=4).to(DEV).set_precision("bf16").train()
    g = torch.Generator().manual_seed(1)
    T = 3
    x = [torch.randn((2, 1, 10, 14), generator=g).to(DEV) for _ in range(T)]
    y = [torch.randn((2, 1, 40, 56), generator=g).to(DEV) for _ in range(T)]
    torch.stack([Fn.l1_loss(o, t) for o, t in zip(net(x), y)]).mean().backward()
    torch.cuda.synchronize()
    return {k: p.grad.detach().clone() for k, p in net.named_parameters()}, len(calls), T


def test_drf_fused_prelu_backward_matches_unfused(monkeypatch):
    gf, nf, T = _drf_grads(monkeypatch, True)
    gu, nu, _ = _drf_grads(monkeypatch, False)
    assert nf == 2 * T, nf  # gout and gin per frame; the other 2G + 2 fused
    assert nu > nf
    for k, v in gu.items():
        assert torch.isfinite(gf[k]).all(), k
        if v.numel() == 1:  # slopes: one bf16 rounding per term apart
            assert (gf[k] - v).abs().item() <= 2e-2 * max(abs(v.item()), 1e-3), (k, gf[k].item(), v.item())
        else:
            err = (gf[k] - v).norm().item() / max(v.norm().item(), 1e-30)
            assert err <= 2e-2, (k, err)


def test_deferred_slope_slots_equal_direct():
    """vsrk_slope_final_sum over per-call slots (da = NULL: the partials stay
    in each call's slot) gives the slope gradient the direct calls accumulate,
    within fp32 rounding of the per-call float adds."""
    g = torch.Generator().manual_seed(21)
    a = torch.tensor([0.2], device=DEV)
    S = F.slope_slot_doubles()
    region = torch.zeros((3, S), dtype=torch.float64, device=DEV)
    da = torch.zeros(1, device=DEV)
    for k in range(3):
        y = torch.randn((2, 1, 9, 21, 64), generator=g).to(DEV, DT)
        dy = torch.randn(y.shape, generator=g).to(DEV, DT)
        F.prelu_bwd(y, dy, a, torch.empty_like(y), da, k > 0)
        F.prelu_bwd(y, dy, a, torch.empty_like(y), None, False, slot=region[k])
    dd = torch.zeros(1, device=DEV)
    F.slope_final_sum(region, a, dd, False, False)
    torch.cuda.synchronize()
    assert abs(dd.item() - da.item()) <= 1e-5 * (1 + abs(da.item())), (dd.item(), da.item())
