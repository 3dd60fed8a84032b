"""DRF building blocks on the HIP kernels against torch fp64 (CPU):
the strided projections nn.Conv2d / nn.ConvTranspose2d(k, s, p) of the
feedback block (drf_net.py:70-102) as 3x3 sub-pixel convolutions (forward,
data gradient, folded weight/bias gradient) for every upscale factor DRF
supports, the PReLU epilogue (drf_net.py:56) and the fused PReLU backward.

Tolerances as test_conv_kernels_gpu.py: fp32 max|d| <= 2e-5 (1 + max|ref|),
bf16 (inputs/weights rounded before the fp64 reference) 1.5e-2 max|ref|,
fp16 3e-3 max|ref|.
"""
import pytest
import torch
import torch.nn.functional as Fn

from vsr_amd import functional as F

pytestmark = pytest.mark.gpu
DEV = "cuda"
PROJ = {2: (6, 2, 2), 3: (7, 3, 2), 4: (8, 4, 2), 8: (12, 8, 2)}


def _tol(dtype, ref):
    s = ref.abs().max().item()
    if dtype == torch.float32:
        return 2e-5 * (1 + s)
    return (3e-3 if dtype == torch.float16 else 1.5e-2) * max(s, 1e-3)


def _wtol(dtype):
    return {torch.float32: 2e-5, torch.float16: 2e-3}.get(dtype, 1e-2)


def _q(t, dtype):
    return t.to(dtype).double()


def _cl(t):  # (N,C,H,W) -> (N,1,H,W,C)
    return t.permute(0, 2, 3, 1).unsqueeze(1).contiguous()


def _nchw(t):  # (N,1,H,W,C) -> (N,C,H,W)
    return t[:, 0].permute(0, 3, 1, 2)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("r", [2, 3, 4, 8])
@pytest.mark.parametrize("f", [16, 64])
@pytest.mark.parametrize("skip", [False, True])
def test_subpixel_deconv_and_conv(dtype, r, f, skip):
    """skip: the sub-pixel structure is passed (F.subpixel_code), so kernels
    that can skip each phase's zero taps do."""
    k, s, p = PROJ[r]
    sc = (lambda tr, fl: F.subpixel_code(k, s, p, tr, fl)) if skip else (lambda tr, fl: 0)
    g = torch.Generator().manual_seed(r * 10 + f)
    n, h, w = 2, 5, 7 if r < 8 else 3
    H, W = h * s, w * s
    x_lr = torch.randn((n, f, h, w), generator=g)
    x_hr = torch.randn((n, f, H, W), generator=g)
    wd = torch.randn((f, f, k, k), generator=g) / (f * k) ** 0.5   # ConvTranspose2d: (cin, cout, k, k)
    bd = torch.randn(f, generator=g)
    wc = torch.randn((f, f, k, k), generator=g) / (f * k) ** 0.5   # Conv2d: (cout, cin, k, k)
    bc = torch.randn(f, generator=g)
    gy_hr = torch.randn((n, f, H, W), generator=g)
    gy_lr = torch.randn((n, f, h, w), generator=g)
    # references (fp64 autograd)
    xl = _q(x_lr, dtype).requires_grad_(True)
    wdr = _q(wd, dtype).requires_grad_(True)
    bdr = bd.double().requires_grad_(True)
    yd = Fn.conv_transpose2d(xl, wdr, bdr, stride=s, padding=p)
    assert yd.shape[-2:] == (H, W)
    yd.backward(_q(gy_hr, dtype))
    xh = _q(x_hr, dtype).requires_grad_(True)
    wcr = _q(wc, dtype).requires_grad_(True)
    bcr = bc.double().requires_grad_(True)
    yc = Fn.conv2d(xh, wcr, bcr, stride=s, padding=p)
    assert yc.shape[-2:] == (h, w)
    yc.backward(_q(gy_lr, dtype))
    K3, P1 = (1, 3, 3), (0, 1, 1)
    # --- transposed conv: 3x3 conv f -> s*s*f written through a shuffle-s view
    weq, beq = F.subpixel_conv_weight(wd.to(DEV), bd.to(DEV), k, s, p, transposed=True)
    out = torch.empty((n, 1, H, W, f), dtype=dtype, device=DEV)
    F.conv(_cl(x_lr).to(DEV, dtype), F.pack_weight(weq, 0, dtype), out, K3, P1, bias=beq, y_shuffle=s, bias_r=1,
           subpixel=sc(True, False))
    ref = _cl(yd.detach())
    assert (out.double().cpu() - ref).abs().max().item() <= _tol(dtype, ref)
    g_hr = _cl(gy_hr).to(DEV, dtype)
    dx = torch.empty((n, 1, h, w, f), dtype=dtype, device=DEV)
    F.conv(g_hr, F.pack_weight(weq, 1, dtype), dx, K3, P1, x_shuffle=s, subpixel=sc(True, True))
    ref = _cl(xl.grad)
    assert (dx.double().cpu() - ref).abs().max().item() <= _tol(dtype, ref), "deconv dgrad"
    dweq = torch.empty_like(weq)
    dbeq = torch.empty_like(beq)
    F.conv_wgrad(_cl(x_lr).to(DEV, dtype), g_hr, K3, P1, dweq.view(*weq.shape[:2], 1, 3, 3), dbeq, dy_shuffle=s,
                 subpixel=sc(True, False))
    dw = torch.empty_like(wd, device=DEV)
    db = torch.empty_like(bd, device=DEV)
    F.subpixel_wgrad_fold(dweq, dbeq, dw, db, k, s, p, transposed=True)
    tw = _wtol(dtype) * (1 + wdr.grad.abs().max().item())
    assert (dw.double().cpu() - wdr.grad).abs().max().item() <= tw, "deconv wgrad"
    assert (db.double().cpu() - bdr.grad).abs().max().item() <= _wtol(dtype) * (
        1 + bdr.grad.abs().max().item()), "deconv bgrad"
    # --- strided conv: 3x3 conv on the shuffle-s view of the high-res input
    weq, beq = F.subpixel_conv_weight(wc.to(DEV), bc.to(DEV), k, s, p, transposed=False)
    xh_d = _cl(x_hr).to(DEV, dtype)
    out = torch.empty((n, 1, h, w, f), dtype=dtype, device=DEV)
    F.conv(xh_d, F.pack_weight(weq, 0, dtype), out, K3, P1, bias=beq, x_shuffle=s, subpixel=sc(False, False))
    ref = _cl(yc.detach())
    assert (out.double().cpu() - ref).abs().max().item() <= _tol(dtype, ref), "conv fwd"
    g_lr = _cl(gy_lr).to(DEV, dtype)
    dx = torch.empty((n, 1, H, W, f), dtype=dtype, device=DEV)
    F.conv(g_lr, F.pack_weight(weq, 1, dtype), dx, K3, P1, y_shuffle=s, bias_r=1, subpixel=sc(False, True))
    ref = _cl(xh.grad)
    assert (dx.double().cpu() - ref).abs().max().item() <= _tol(dtype, ref), "conv dgrad"
    dweq = torch.empty_like(weq)
    dbeq = torch.empty_like(beq)
    F.conv_wgrad(xh_d, g_lr, K3, P1, dweq.view(*weq.shape[:2], 1, 3, 3), dbeq, x_shuffle=s,
                 subpixel=sc(False, False))
    dw = torch.empty_like(wc, device=DEV)
    db = torch.empty_like(bc, device=DEV)
    F.subpixel_wgrad_fold(dweq, dbeq, dw, db, k, s, p, transposed=False)
    tw = _wtol(dtype) * (1 + wcr.grad.abs().max().item())
    assert (dw.double().cpu() - wcr.grad).abs().max().item() <= tw, "conv wgrad"
    assert (db.double().cpu() - bcr.grad).abs().max().item() <= _wtol(dtype) * (
        1 + bcr.grad.abs().max().item()), "conv bgrad"


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16])
def test_prelu_epilogue_and_backward(dtype):
    g = torch.Generator().manual_seed(21)
    n, h, w, ci, co = 2, 9, 35, 64, 64
    x = torch.randn((n, 1, h, w, ci), generator=g)
    wt = torch.randn((co, ci, 3, 3), generator=g) / 24
    b = torch.randn(co, generator=g)
    a = torch.tensor([0.2])
    pre = Fn.conv2d(_nchw(_q(x, dtype)), _q(wt, dtype), b.double(), padding=1)
    ref = _cl(Fn.prelu(pre, a.double()))
    y = torch.empty((n, 1, h, w, co), dtype=dtype, device=DEV)
    ad = a.to(DEV)
    F.conv(x.to(DEV, dtype), F.pack_weight(wt.to(DEV), 0, dtype), y, (1, 3, 3), (0, 1, 1), bias=b.to(DEV),
           act=F.ACT_PRELU, act_param=ad)
    assert (y.double().cpu() - ref).abs().max().item() <= _tol(dtype, ref)
    # backward of the PReLU given dL/dy (+ a second contribution), against autograd
    gy = torch.randn((n, 1, h, w, co), generator=g)
    gy2 = torch.randn((n, 1, h, w, co), generator=g)
    pre_r = pre.detach().clone().requires_grad_(True)
    ar = a.double().clone().requires_grad_(True)
    out = Fn.prelu(pre_r, ar)
    out.backward(_nchw(_q(gy, dtype) + _q(gy2, dtype)))
    dx = torch.empty_like(y)
    da = torch.zeros(1, device=DEV)
    F.prelu_bwd(y, gy.to(DEV, dtype), ad, dx, da, accumulate_da=False, dy2=gy2.to(DEV, dtype))
    refx = _cl(pre_r.grad)
    assert (dx.double().cpu() - refx).abs().max().item() <= _tol(dtype, refx) * 2
    rel = abs(da.item() - ar.grad.item()) / abs(ar.grad.item())
    assert rel <= {torch.float32: 1e-4, torch.float16: 5e-3}.get(dtype, 3e-2), rel
    da2 = torch.zeros(1, device=DEV)
    F.prelu_wgrad(y, dx, ad, da2, accumulate=False)
    assert abs(da2.item() - da.item()) <= 1e-5 * (1 + abs(da.item()))
    # data-gradient epilogue with a PReLU mask: dgrad(next conv) * (y > 0 ? 1 : a)
    gz = torch.randn((n, 1, h, w, co), generator=g)
    d_in = torch.empty_like(y)
    F.conv(gz.to(DEV, dtype), F.pack_weight(wt.to(DEV), 1, dtype), d_in, (1, 3, 3), (0, 1, 1), mask=y,
           mask_slope=ad)
    gin = Fn.conv_transpose2d(_nchw(_q(gz, dtype)), _q(wt, dtype), padding=1)
    refm = _cl(torch.where(_nchw(y.double().cpu()) > 0, gin, 0.2 * gin))
    assert (d_in.double().cpu() - refm).abs().max().item() <= _tol(dtype, refm) * 2


@pytest.mark.parametrize("slope", [0.0, -0.3])
def test_prelu_slope_gradient_nonpositive_slope_is_loud(slope):
    """The tape keeps PReLU outputs only; y < 0 marks x < 0 only while a > 0.
    With a <= 0 both slope-gradient paths (prelu_bwd and the fused rolling
    dgrad, vsrk_conv_fwd_prelu_bwd) write NaN instead of a silently wrong
    value."""
    g = torch.Generator().manual_seed(5)
    dt = torch.bfloat16
    n, h, w, f = 1, 8, 16, 64
    y = torch.randn((n, 1, h, w, f), generator=g).to(DEV, dt)
    gy = torch.randn((n, 1, h, w, f), generator=g).to(DEV, dt)
    ad = torch.tensor([slope], device=DEV)
    da = torch.zeros(1, device=DEV)
    F.prelu_bwd(y, gy, ad, torch.empty_like(y), da, accumulate_da=False)
    assert torch.isnan(da).all()
    wt = torch.randn((f, f, 3, 3), generator=g).to(DEV) / 24
    da2 = torch.zeros(1, device=DEV)
    ran = F.conv_prelu_bwd(gy, F.pack_weight(wt, 1, dt), torch.empty_like(y), (1, 3, 3), (0, 1, 1), y, ad, da2, False)
    if ran:
        assert torch.isnan(da2).all()
