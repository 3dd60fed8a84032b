"""The weight-gradient split reduce (conv_wgrad.hip): the row-order form
(wgrad_reduce_rows_kernel: few splits, many output channels -- DRF's sub-pixel
and 256-channel convs, DUF's wide 3x3x3 units) against an fp64 torch
reference, with torch pixel-shuffle channel order (perm_r), accumulate and the
dbias tails.  Inputs rounded to bf16 before the reference; max |d| <= 2e-3 *
max |ref| (fp32 sums of bf16 products over a few thousand voxels)."""
import pytest
import torch
import torch.nn.functional as Fn

from vsr_amd import functional as F

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _ref(x, gy, k, pad):
    xr = x.double().permute(0, 4, 1, 2, 3)
    w = torch.zeros((gy.shape[-1], x.shape[-1]) + k, dtype=torch.float64, requires_grad=True)
    b = torch.zeros(gy.shape[-1], dtype=torch.float64, requires_grad=True)
    Fn.conv3d(xr, w, b, padding=pad).backward(gy.double().permute(0, 4, 1, 2, 3))
    return w.grad, b.grad


@pytest.mark.parametrize("case", [
    # (N, D, H, W, Cin, Cout, k, pad)
    (2, 1, 24, 40, 64, 256, (1, 3, 3), (0, 1, 1)),   # 256 output channels, 12 tiles: row-order reduce
    (1, 1, 16, 64, 256, 64, (1, 3, 3), (0, 1, 1)),   # 4 input blocks x 64 outputs
    (1, 5, 16, 32, 192, 32, (3, 3, 3), (1, 1, 1)),   # DUF-like wide unit (rolling wgrad's slabs)
    (1, 1, 20, 36, 48, 320, (1, 3, 3), (0, 1, 1)),   # partial input block (48 of 64)
])
@pytest.mark.parametrize("acc", [False, True])
def test_wgrad_reduce_rows(case, acc):
    n, d, h, w, ci, co, k, pad = case
    g = torch.Generator().manual_seed(3)
    x = torch.randn((n, d, h, w, ci), generator=g).to(torch.bfloat16)
    do = d + 2 * pad[0] - (k[0] - 1)
    gy = torch.randn((n, do, h, w, co), generator=g).to(torch.bfloat16)
    wref, bref = _ref(x, gy, k, pad)
    dw0 = torch.randn((co, ci) + k, generator=g) if acc else torch.zeros((co, ci) + k)
    db0 = torch.randn(co, generator=g) if acc else torch.zeros(co)
    dw, db = dw0.to(DEV), db0.to(DEV)
    F.conv_wgrad(x.to(DEV), gy.to(DEV), k, pad, dw, db, accumulate=acc)
    torch.cuda.synchronize()
    ew = (dw.double().cpu() - dw0.double() - wref).abs().max().item()
    eb = (db.double().cpu() - db0.double() - bref).abs().max().item()
    assert ew <= 2e-3 * wref.abs().max().item(), ew
    assert eb <= 2e-3 * bref.abs().max().item(), eb


def test_wgrad_reduce_rows_perm():
    """an upsampler conv's weight gradient: dy through a pixel-shuffle view,
    dw / dbias in torch order (edsr_net.py Upsampler)"""
    g = torch.Generator().manual_seed(4)
    n, h, w, f, r = 2, 12, 20, 64, 2
    x = torch.randn((n, 1, h, w, f), generator=g).to(torch.bfloat16)
    gy_hr = torch.randn((n, 1, h * r, w * r, f), generator=g).to(torch.bfloat16)
    # torch: conv -> pixel_shuffle; the gradient of the conv output is pixel_unshuffle(gy)
    gy_conv = Fn.pixel_unshuffle(gy_hr[:, 0].permute(0, 3, 1, 2), r)            # (n, f r r, h, w)
    wref, bref = _ref(x, gy_conv.permute(0, 2, 3, 1).unsqueeze(1), (1, 3, 3), (0, 1, 1))
    dw = torch.zeros((f * r * r, f, 1, 3, 3), device=DEV)
    db = torch.zeros(f * r * r, device=DEV)
    F.conv_wgrad(x.to(DEV), gy_hr.to(DEV), (1, 3, 3), (0, 1, 1), dw, db, perm_r=r, dy_shuffle=r)
    torch.cuda.synchronize()
    assert (dw.double().cpu() - wref).abs().max().item() <= 2e-3 * wref.abs().max().item()
    assert (db.double().cpu() - bref).abs().max().item() <= 2e-3 * bref.abs().max().item()
