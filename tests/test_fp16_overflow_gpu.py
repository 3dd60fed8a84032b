"""fp16 loss-scale overflow handling (GradScaler semantics) of the HIP
generators: an fp16 backward whose scaled gradients overflow is detected
(inf / NaN in any parameter gradient), the optimizer step is skipped so the
weights and Adam's state stay untouched, and the dynamic scale backs off by
half; finite steps proceed and the scale grows again after
scale_growth_interval of them.  Data-parallel: the check runs on the
all-reduced buckets (GradSync.finish), so every rank skips the same step.

Reference: the reference trains in fp32 only (main.py:73, no autocast); this
is the build's fp16 path (BASELINE config 5), checked here against
torch.cuda.amp.GradScaler's rules, not against a reference fixture."""
import pytest
import torch

from vsr_amd import nets
from vsr_amd.losses import L1Loss

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _setup(seed=0):
    torch.manual_seed(seed)
    net = nets.EDSRNet(in_channels=1, out_channels=1, num_resblocks=2, num_features=16, upscale_factor=2,
                       res_scale=0.1).to(DEV).set_precision("fp16")
    opt = torch.optim.Adam(net.parameters(), lr=1e-3)
    g = torch.Generator().manual_seed(seed)
    x = torch.randn((2, 1, 16, 16), generator=g).to(DEV)
    y = torch.randn((2, 1, 32, 32), generator=g).to(DEV)
    return net, opt, x, y


def _step(net, opt, x, y):
    loss = L1Loss()(net(x), y)
    opt.zero_grad(set_to_none=True)
    loss.backward()
    ok = net.step_ok()
    if ok:
        opt.step()
    return ok


def test_overflow_skips_step_and_backs_off():
    net, opt, x, y = _setup()
    assert _step(net, opt, x, y)  # a finite step: initialises the scale, updates the weights
    s0 = net._scale
    assert s0 == 2.0 ** 11  # 2 x 32 x 32 = 2048 output values: output gradients in [1, 2)
    before = {k: v.clone() for k, v in net.state_dict().items()}
    state_before = {k: {n: t.clone() for n, t in st.items() if torch.is_tensor(t)} for k, st in opt.state.items()}
    net._scale = 2.0 ** 40  # scaled fp16 gradients overflow
    assert not _step(net, opt, x, y)
    assert net._scale == 2.0 ** 39
    for k, v in net.state_dict().items():
        assert torch.equal(v, before[k]), k
    for k, st in opt.state.items():
        for n, t in st.items():
            if torch.is_tensor(t):
                assert torch.equal(t, state_before[k][n]), n
    # back to a sane scale: the step runs and the weights move
    net._scale = s0
    assert _step(net, opt, x, y)
    assert any(not torch.equal(v, before[k]) for k, v in net.state_dict().items())
    assert all(torch.isfinite(p).all() for p in net.parameters())


def test_scale_growth():
    net, opt, x, y = _setup(1)
    net.scale_growth_interval = 3
    assert _step(net, opt, x, y)
    s0 = net._scale
    assert _step(net, opt, x, y) and _step(net, opt, x, y)
    assert net._scale == 2 * s0 and net._good_steps == 0


def test_fixed_scale_overflow_is_flagged():
    net, opt, x, y = _setup(2)
    net.loss_scale = 2.0 ** 40
    assert not _step(net, opt, x, y)
    assert net._scale is None  # a fixed scale is not adjusted


def test_bf16_has_no_check():
    net, opt, x, y = _setup(3)
    net.set_precision("bf16")
    assert _step(net, opt, x, y)
    assert net._found_inf is None


def test_check_stays_on_at_unit_scale():
    """The dynamic scale may back off to 1 and below (no floor, as GradScaler):
    a NaN step at scale 1 is still detected and skipped, and the scale keeps
    halving (the guard used to switch itself off at scale 1)."""
    net, opt, x, y = _setup(3)
    assert _step(net, opt, x, y)
    net._scale = 1.0
    before = {k: v.clone() for k, v in net.state_dict().items()}
    xn = x.clone()
    xn[0, 0, 3, 5] = float("nan")
    assert not _step(net, opt, xn, y)
    assert net._scale == 0.5
    for k, v in net.state_dict().items():
        assert torch.equal(v, before[k]), k
    assert _step(net, opt, x, y)  # finite again at scale 0.5
    net.loss_scale = 1.0  # a fixed unit scale checks as well
    assert not _step(net, opt, xn, y)
