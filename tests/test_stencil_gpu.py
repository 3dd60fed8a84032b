"""One-channel 3x3 stencils (conv_stencil.hip): the network head
nn.Conv2d(1, 64, 3, padding=1) (edsr_net.py:28, duf_net.py:35, drf_net.py:25)
and the data gradient of EDSR's tail nn.Conv2d(64, 1, 3, padding=1)
(edsr_net.py:32), 16-bit in and out; and the tail's forward (one output
channel, fp32 or 16-bit out).

Against fp64 convolutions of the same 16-bit operands (bf16 / fp16 storage
bound of the output, as every conv kernel test) and against the thin-input
implicit-GEMM kernel it replaces (path "stencil" off) within one output
rounding: both sum the 9 exact products in fp32, in different orders.
Inputs in the nets' 8-channel padded storage and plain views; tiles cut by
the image edge; several depths per sample.
"""
import pytest
import torch
import torch.nn.functional as Fn

from vsr_amd import functional as F

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(autouse=True)
def _paths():
    yield
    F.set_conv_path("stencil", -1)


def _ref(x_cl, w, b, relu):
    y = Fn.conv3d(x_cl.permute(0, 4, 1, 2, 3), w, b, padding=(0, 1, 1)).permute(0, 2, 3, 4, 1)
    return torch.relu(y) if relu else y


def _input(x, dt, padded):
    if not padded:
        return x.to(DEV, dt)
    st = torch.zeros((*x.shape[:-1], 8), dtype=dt, device=DEV)
    st[..., :1] = x.to(DEV, dt)
    return st[..., :1]


def _tol(dt, ref):
    return (1.5e-2 if dt == torch.bfloat16 else 2e-3) * max(ref.abs().max().item(), 1e-3)


CASES = [
    # (N, D, H, W, padded input storage, bias, relu)
    (2, 1, 20, 45, True, True, False),
    (1, 1, 13, 130, False, True, True),
    (2, 3, 9, 70, True, False, False),
    (1, 1, 8, 64, True, True, False),
    (3, 1, 17, 5, False, False, True),
]


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("case", CASES)
def test_stencil_head_forward(case, dt):
    n, d, h, w, padded, bias, relu = case
    g = torch.Generator().manual_seed(h * 100 + w)
    x = torch.randn((n, d, h, w, 1), generator=g)
    wt = torch.randn((64, 1, 1, 3, 3), generator=g) / 3
    b = torch.randn(64, generator=g) if bias else None
    ref = _ref(x.to(dt).double(), wt.to(dt).double(), b.double() if bias else None, relu)
    xin = _input(x, dt, padded)
    wp = F.pack_weight(wt.to(DEV), 0, dt)
    kw = dict(bias=b.to(DEV) if bias else None, act=F.ACT_RELU if relu else F.ACT_NONE)
    y = torch.empty((n, d, h, w, 64), dtype=dt, device=DEV)
    F.conv(xin, wp, y, (1, 3, 3), (0, 1, 1), **kw)
    assert (y.double().cpu() - ref).abs().max().item() <= _tol(dt, ref)
    F.set_conv_path("stencil", 0)
    y0 = torch.empty_like(y)
    F.conv(xin, wp, y0, (1, 3, 3), (0, 1, 1), **kw)
    assert (y.double() - y0.double()).abs().max().item() <= _tol(dt, ref)


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
def test_stencil_tail_data_gradient(dt):
    """dL/dx of the tail conv 64 -> 1 (mode-1 packed weight, the 1-channel
    gradient in 8-channel storage) -- the EDSR backward's first conv."""
    g = torch.Generator().manual_seed(7)
    n, h, w = 2, 40, 100
    gy = torch.randn((n, 1, h, w, 1), generator=g)
    wt = torch.randn((1, 64, 1, 3, 3), generator=g) / 24
    xr = torch.zeros((n, 1, h, w, 64), dtype=torch.float64, requires_grad=True)
    Fn.conv3d(xr.permute(0, 4, 1, 2, 3), wt.to(dt).double(), None, padding=(0, 1, 1)).permute(0, 2, 3, 4, 1) \
        .backward(gy.to(dt).double())
    ref = xr.grad
    dx = torch.empty((n, 1, h, w, 64), dtype=dt, device=DEV)
    F.conv(_input(gy, dt, True), F.pack_weight(wt.to(DEV), 1, dt), dx, (1, 3, 3), (0, 1, 1))
    assert (dx.double().cpu() - ref).abs().max().item() <= _tol(dt, ref)


def test_stencil_not_taken_with_epilogue_operands():
    """residual / mask / accumulate / a prologue keep the thin-input kernel
    (results still match fp64)."""
    g = torch.Generator().manual_seed(9)
    n, h, w = 1, 12, 40
    x = torch.randn((n, 1, h, w, 1), generator=g)
    wt = torch.randn((64, 1, 1, 3, 3), generator=g) / 3
    res = torch.randn((n, 1, h, w, 64), generator=g)
    bf = torch.bfloat16
    ref = _ref(x.to(bf).double(), wt.to(bf).double(), None, False) + res.to(bf).double()
    y = torch.empty((n, 1, h, w, 64), dtype=bf, device=DEV)
    F.conv(_input(x, bf, True), F.pack_weight(wt.to(DEV), 0, bf), y, (1, 3, 3), (0, 1, 1), residual=res.to(DEV, bf))
    assert (y.double().cpu() - ref).abs().max().item() <= 2 * _tol(bf, ref)


OUT_CASES = [
    # (N, D, H, W, Cin, y dtype, bias)
    (2, 1, 20, 45, 64, torch.float32, True),
    (1, 2, 9, 150, 64, torch.float32, True),
    (1, 1, 33, 128, 32, torch.bfloat16, False),
    (2, 1, 17, 19, 96, torch.float32, True),
    (1, 1, 5, 260, 256, torch.float32, True),
]


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("case", OUT_CASES)
def test_stencil_tail_forward(case, dt):
    """EDSR's tail nn.Conv2d(F, 1, 3, padding=1) (edsr_net.py:32): the
    one-output-channel rolling form against fp64 and the thin-output kernel."""
    n, d, h, w, ci, ydt, bias = case
    g = torch.Generator().manual_seed(ci + h)
    x = torch.randn((n, d, h, w, ci), generator=g)
    wt = torch.randn((1, ci, 1, 3, 3), generator=g) / (9 * ci) ** 0.5
    b = torch.randn(1, generator=g) if bias else None
    ref = _ref(x.to(dt).double(), wt.to(dt).double(), b.double() if bias else None, False)
    xd = x.to(DEV, dt)
    wp = F.pack_weight(wt.to(DEV), 0, dt)
    ydt = dt if ydt != torch.float32 else ydt
    y = torch.empty((n, d, h, w, 1), dtype=ydt, device=DEV)
    F.conv(xd, wp, y, (1, 3, 3), (0, 1, 1), bias=b.to(DEV) if bias else None)
    tol = 2e-5 * (1 + ref.abs().max().item()) if ydt == torch.float32 else _tol(dt, ref)
    assert (y.double().cpu() - ref).abs().max().item() <= tol + 1e-3 * ref.abs().max().item()
    F.set_conv_path("stencil", 0)
    y0 = torch.empty_like(y)
    F.conv(xd, wp, y0, (1, 3, 3), (0, 1, 1), bias=b.to(DEV) if bias else None)
    assert (y.double() - y0.double()).abs().max().item() <= tol + 1e-4 * ref.abs().max().item()
