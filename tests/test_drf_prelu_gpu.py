"""PReLU slopes <= 0 in DRF (nn.PReLU's slope is
unconstrained, drf_net.py:55-58,66,83-100).  The nets keep PReLU OUTPUTS on the
tape; for a slope <= 0 the output no longer tells x < 0 apart (a < 0) or
loses x (a = 0), so the backward recomputes that PReLU's pre-activation from
the tape and runs nn.PReLU's own backward from it (vsrk_prelu_bwd_pre):
dx = g (x > 0 ? 1 : a), da = sum_{x<0} g x.  Checked against the oracle
(oracle/cpu_nets.DRFRef: stock nn modules, fp32, the same device) with the
net's PReLU slopes set to -0.3, 0, 1e-4 and 0.2 in turn, fp32 tolerance of
SURVEY 8(d) (outputs 1e-4, gradients rel-L2 1e-4 per parameter; slope
gradients, one scalar each, relative 1e-4 of the largest slope gradient)."""
import pytest
import torch
import torch.nn as nn
import torch.nn.functional as Fn

from oracle import cpu_nets
from vsr_amd import functional as F
from vsr_amd import nets

pytestmark = pytest.mark.gpu
DEV = "cuda"
SLOPES = (-0.3, 0.0, 1e-4, 0.2)


def _pair(precision, slopes=SLOPES, seed=0):
    kw = dict(in_channels=1, out_channels=1, num_features=16, num_groups=2, upscale_factor=4)
    torch.manual_seed(seed)
    mine = nets.DRFNet(**kw).to(DEV).set_precision(precision).train()
    ref = cpu_nets.DRFRef(**kw).to(DEV).train()
    prelus = [m for m in mine.modules() if isinstance(m, nn.PReLU)]
    with torch.no_grad():
        for i, m in enumerate(prelus):  # every slope value on several layers
            m.weight.fill_(slopes[i % len(slopes)])
    ref.load_state_dict(mine.state_dict())
    return mine, ref, len(prelus)


@pytest.mark.parametrize("shift", range(len(SLOPES)))
def test_drf_prelu_any_slope_matches_oracle(shift):
    # each PReLU layer sees each slope value across the four cases
    mine, ref, n = _pair("fp32", SLOPES[shift:] + SLOPES[:shift])
    assert n >= 8
    g = torch.Generator().manual_seed(5)
    T = 3
    x = [torch.randn((2, 1, 12, 16), generator=g).to(DEV) for _ in range(T)]
    y = [torch.randn((2, 1, 48, 64), generator=g).to(DEV) for _ in range(T)]
    outs = mine(x)
    torch.stack([Fn.l1_loss(o, t) for o, t in zip(outs, y)]).mean().backward()
    with torch.backends.cudnn.flags(enabled=False):
        routs = ref(x)
        torch.stack([Fn.l1_loss(o, t) for o, t in zip(routs, y)]).mean().backward()
    torch.cuda.synchronize()
    for o, r in zip(outs, routs):
        assert (o - r).abs().max().item() <= 1e-4, (o - r).abs().max().item()
    gm = {k: p.grad for k, p in mine.named_parameters()}
    gr = {k: p.grad for k, p in ref.named_parameters()}
    smax = max(v.abs().item() for k, v in gr.items() if v.numel() == 1)
    for k, v in gr.items():
        assert torch.isfinite(gm[k]).all(), k
        if v.numel() == 1:  # PReLU slope gradients
            assert (gm[k] - v).abs().item() <= 1e-4 * smax, (k, gm[k].item(), v.item())
        else:
            rel = (gm[k] - v).norm().item() / max(v.norm().item(), 1e-30)
            assert rel <= 1e-4, (k, rel)


def test_drf_prelu_nonpositive_bf16_finite_and_close():
    """bf16 with slopes <= 0: finite gradients within the bf16 bound of
    SURVEY 8(d) against the fp32 oracle (worst parameter rel-L2 <= 8e-2)."""
    mine, ref, _ = _pair("bf16")
    g = torch.Generator().manual_seed(6)
    x = [torch.randn((2, 1, 12, 16), generator=g).to(DEV) for _ in range(3)]
    y = [torch.randn((2, 1, 48, 64), generator=g).to(DEV) for _ in range(3)]
    torch.stack([Fn.l1_loss(o, t) for o, t in zip(mine(x), y)]).mean().backward()
    with torch.backends.cudnn.flags(enabled=False):
        torch.stack([Fn.l1_loss(o, t) for o, t in zip(ref(x), y)]).mean().backward()
    torch.cuda.synchronize()
    gr = {k: p.grad for k, p in ref.named_parameters()}
    smax = max(v.abs().item() for k, v in gr.items() if v.numel() == 1)
    for k, p in mine.named_parameters():
        assert torch.isfinite(p.grad).all(), k
        v = gr[k]
        if v.numel() == 1:
            assert (p.grad - v).abs().item() <= 8e-2 * smax, (k, p.grad.item(), v.item())
        else:
            assert (p.grad - v).norm().item() <= 8e-2 * max(v.norm().item(), 1e-30), k


def test_prelu_bwd_pre_matches_autograd():
    """The op alone: vsrk_prelu_bwd_pre against torch's PReLU autograd in fp32
    for every slope sign, with a second gradient contribution."""
    g = torch.Generator().manual_seed(7)
    x = torch.randn((2, 1, 9, 13, 24), generator=g).to(DEV)
    x[..., 0, 0, :5] = 0.0  # exact zeros: nn.PReLU takes the a-branch there
    dy = torch.randn(x.shape, generator=g).to(DEV)
    dy2 = torch.randn(x.shape, generator=g).to(DEV)
    for a0 in SLOPES:
        a = torch.tensor([a0], device=DEV)
        at = a.clone().requires_grad_()
        xt = x.clone().requires_grad_()
        (Fn.prelu(xt, at) * (dy + dy2)).sum().backward()
        dx = torch.empty_like(x)
        da = torch.zeros(1, device=DEV)
        F.prelu_bwd(x, dy, a, dx, da, False, dy2=dy2, pre=True)
        torch.cuda.synchronize()
        assert torch.allclose(dx, xt.grad, rtol=0, atol=1e-6), a0
        assert abs(da.item() - at.grad.item()) <= 1e-5 * (1 + abs(at.grad.item())), (a0, da.item(), at.grad.item())
