"""Parity of the implicit-GEMM conv kernels (forward, data-gradient, weight
gradient) against torch fp64 on the CPU (the oracle for a floating-point
kernel), across the shapes the generators use and the fused prologue /
epilogue / sub-pixel addressing modes.

Tolerances: fp32 kernels: max |d| <= 2e-5 * (1 + max|ref|) (exact-fp32 MFMA,
different summation order).  bf16 / fp16 kernels: inputs and weights are
rounded to the 16-bit type before the fp64 reference, so only accumulation
order and the final 16-bit store differ: max |d| <= 1.5e-2 * max|ref| (bf16),
2e-3 * max|ref| (fp16).
"""
import pytest
import torch
import torch.nn.functional as Fn

from vsr_amd import functional as F

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _tol(dtype, ref):
    scale = ref.abs().max().item()
    if dtype == torch.float32:
        return 2e-5 * (1 + scale)
    if dtype == torch.float16:  # 11-bit significand: final store 2^-11 relative
        return 2e-3 * max(scale, 1e-3)
    return 1.5e-2 * max(scale, 1e-3)


def _q(t, dtype):
    """round to the compute dtype (what the kernel sees), back to fp64."""
    return t.to(dtype).double()


def _ref_conv(x_cl, w, b, pad):
    # x_cl (N,D,H,W,C) -> NCDHW fp64 conv3d -> (N,D,H,W,Co)
    x = x_cl.permute(0, 4, 1, 2, 3)
    y = Fn.conv3d(x, w, b, padding=pad)
    return y.permute(0, 2, 3, 4, 1)


CASES = [
    # (N, D, H, W, Cin, Cout, k, pad)
    (2, 1, 13, 37, 16, 32, (1, 3, 3), (0, 1, 1)),
    (1, 1, 9, 70, 64, 64, (1, 3, 3), (0, 1, 1)),
    (2, 5, 9, 35, 24, 40, (3, 3, 3), (1, 1, 1)),
    (1, 7, 6, 20, 48, 32, (3, 3, 3), (0, 1, 1)),
    (2, 3, 5, 33, 48, 130, (1, 1, 1), (0, 0, 0)),
    (2, 1, 11, 12, 1, 64, (1, 3, 3), (0, 1, 1)),
    (2, 1, 17, 19, 64, 1, (1, 3, 3), (0, 1, 1)),
    # DUF heads (duf_net.py:38-49) and tail (:118) at the golden fixture's LR size
    (2, 1, 12, 16, 256, 512, (1, 1, 1), (0, 0, 0)),
    (2, 1, 12, 16, 512, 400, (1, 1, 1), (0, 0, 0)),
    (2, 1, 12, 16, 256, 16, (1, 1, 1), (0, 0, 0)),
    (2, 1, 12, 16, 256, 256, (1, 3, 3), (0, 1, 1)),
]


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("case", CASES)
def test_conv_forward(case, dtype):
    n, d, h, w, ci, co, k, pad = case
    g = torch.Generator().manual_seed(0)
    x = torch.randn((n, d, h, w, ci), generator=g)
    wt = torch.randn((co, ci, *k), generator=g) / (ci * k[0] * k[1] * k[2]) ** 0.5
    b = torch.randn(co, generator=g)
    ref = _ref_conv(_q(x, dtype), _q(wt, dtype), b.double(), pad)
    do = d + 2 * pad[0] - k[0] + 1
    xd = x.to(DEV, dtype)
    y = torch.empty((n, do, h, w, co), dtype=dtype, device=DEV)
    F.conv(xd, F.pack_weight(wt.to(DEV), 0, dtype), y, k, pad, bias=b.to(DEV))
    err = (y.double().cpu() - ref).abs().max().item()
    assert err <= _tol(dtype, ref), err


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16])
def test_conv_fused_prologue_epilogue(dtype):
    """BN-affine+ReLU prologue, ReLU act, out_scale, mask, residual, accumulate,
    on channel-slice views of larger buffers (the DUF concat layout)."""
    g = torch.Generator().manual_seed(1)
    n, d, h, w, ci, co = 2, 3, 10, 40, 32, 32
    big = torch.randn((n, d, h, w, ci + 16), generator=g)
    x = big[..., 8:8 + ci]
    wt = torch.randn((co, ci, 3, 3, 3), generator=g) / 12
    b = torch.randn(co, generator=g)
    sc = torch.rand(ci, generator=g) + 0.5
    sh = torch.randn(ci, generator=g)
    mask = torch.randn((n, d, h, w, co), generator=g)
    res = torch.randn((n, d, h, w, co), generator=g)
    y0 = torch.randn((n, d, h, w, co), generator=g)
    xin = torch.relu(_q(x, dtype) * sc.double() + sh.double())
    xin = xin.to(dtype).double() if dtype != torch.float32 else xin
    ref = torch.relu(_ref_conv(xin, _q(wt, dtype), b.double(), (1, 1, 1)) * 0.5)
    ref = torch.where(_q(mask, dtype) > 0, ref, torch.zeros_like(ref)) + _q(res, dtype) + _q(y0, dtype)
    bigd = big.to(DEV, dtype)
    yd = y0.to(DEV, dtype)
    F.conv(bigd[..., 8:8 + ci], F.pack_weight(wt.to(DEV), 0, dtype), yd, (3, 3, 3), (1, 1, 1), bias=b.to(DEV),
           prologue=F.PRO_AFFINE_RELU, pro_scale=sc.to(DEV), pro_shift=sh.to(DEV), act=F.ACT_RELU, out_scale=0.5,
           mask=mask.to(DEV, dtype), residual=res.to(DEV, dtype), accumulate=True)
    err = (yd.double().cpu() - ref).abs().max().item()
    assert err <= _tol(dtype, ref) * 2, err


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("r", [2, 3])
def test_conv_pixel_shuffle_output(dtype, r):
    """conv written through a sub-pixel view == torch conv2d -> pixel_shuffle."""
    g = torch.Generator().manual_seed(2)
    n, h, w, ci, f = 2, 7, 33, 16, 16
    co = f * r * r
    x = torch.randn((n, 1, h, w, ci), generator=g)
    wt = torch.randn((co, ci, 3, 3), generator=g) / 12
    b = torch.randn(co, generator=g)
    ref = Fn.pixel_shuffle(Fn.conv2d(_q(x, dtype)[:, 0].permute(0, 3, 1, 2), _q(wt, dtype), b.double(), padding=1), r)
    ref = ref.permute(0, 2, 3, 1)  # (n, rh, rw, f)
    y = torch.empty((n, 1, h * r, w * r, f), dtype=dtype, device=DEV)
    F.conv(x.to(DEV, dtype), F.pack_weight(wt.to(DEV), 0, dtype, perm_r=r), y, (1, 3, 3), (0, 1, 1),
           bias=b.to(DEV), y_shuffle=r)
    err = (y[:, 0].double().cpu() - ref).abs().max().item()
    assert err <= _tol(dtype, ref), err


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("case", CASES)
def test_conv_backward(case, dtype):
    """data-gradient (mode-1 packed weight through the forward kernel) and the
    deterministic weight/bias gradient against torch autograd in fp64."""
    n, d, h, w, ci, co, k, pad = case
    g = torch.Generator().manual_seed(3)
    x = torch.randn((n, d, h, w, ci), generator=g)
    wt = torch.randn((co, ci, *k), generator=g) / (ci * k[0] * k[1] * k[2]) ** 0.5
    b = torch.randn(co, generator=g)
    do = d + 2 * pad[0] - k[0] + 1
    gy = torch.randn((n, do, h, w, co), generator=g)
    xr = _q(x, dtype).requires_grad_(True)
    wr = _q(wt, dtype).requires_grad_(True)
    br = b.double().requires_grad_(True)
    yr = _ref_conv(xr, wr, br, pad)
    yr.backward(_q(gy, dtype))
    # dgrad
    dpad = tuple(kk - 1 - p for kk, p in zip(k, pad))
    dx = torch.empty((n, d, h, w, ci), dtype=dtype, device=DEV)
    F.conv(gy.to(DEV, dtype), F.pack_weight(wt.to(DEV), 1, dtype), dx, k, dpad)
    err = (dx.double().cpu() - xr.grad).abs().max().item()
    assert err <= _tol(dtype, xr.grad), ("dgrad", err)
    # wgrad
    dw = torch.empty((co, ci, *k), dtype=torch.float32, device=DEV)
    db = torch.empty(co, dtype=torch.float32, device=DEV)
    F.conv_wgrad(x.to(DEV, dtype), gy.to(DEV, dtype), k, pad, dw, db)
    ew = (dw.double().cpu() - wr.grad).abs().max().item()
    eb = (db.double().cpu() - br.grad).abs().max().item()
    wt_ = {torch.float32: 2e-5, torch.float16: 2e-3}.get(dtype, 1e-2)
    tw = wt_ * (1 + wr.grad.abs().max().item())
    tb = wt_ * (1 + br.grad.abs().max().item())
    assert ew <= tw, ("wgrad", ew, tw)
    assert eb <= tb, ("bgrad", eb, tb)


def test_wgrad_deterministic():
    g = torch.Generator().manual_seed(4)
    x = torch.randn((2, 4, 16, 40, 32), generator=g).to(DEV, torch.bfloat16)
    gy = torch.randn((2, 4, 16, 40, 32), generator=g).to(DEV, torch.bfloat16)
    outs = []
    for _ in range(2):
        dw = torch.empty((32, 32, 3, 3, 3), device=DEV)
        F.conv_wgrad(x, gy, (3, 3, 3), (1, 1, 1), dw)
        outs.append(dw)
    assert torch.equal(outs[0], outs[1])


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_wgrad_prologue_and_shuffle(dtype):
    """weight gradient with BN-affine+ReLU prologue on x and a sub-pixel dy view."""
    g = torch.Generator().manual_seed(5)
    r, n, h, w, ci, f = 2, 2, 6, 20, 16, 16
    co = f * r * r
    x = torch.randn((n, 1, h, w, ci), generator=g)
    sc = torch.rand(ci, generator=g) + 0.5
    sh = torch.randn(ci, generator=g)
    wt = torch.randn((co, ci, 3, 3), generator=g) / 12
    gy = torch.randn((n, f, h * r, w * r), generator=g)  # grad of the shuffled output (NCHW)
    xin = torch.relu(_q(x, dtype) * sc.double() + sh.double())
    xin = xin.to(dtype).double() if dtype != torch.float32 else xin
    wr = _q(wt, dtype).requires_grad_(True)
    y = Fn.pixel_shuffle(Fn.conv2d(xin[:, 0].permute(0, 3, 1, 2), wr, padding=1), r)
    y.backward(_q(gy, dtype))
    dw = torch.empty((co, ci, 3, 3), device=DEV)
    gy_cl = gy.permute(0, 2, 3, 1).unsqueeze(1).contiguous().to(DEV, dtype)  # (n,1,rh,rw,f)
    F.conv_wgrad(x.to(DEV, dtype), gy_cl, (1, 3, 3), (0, 1, 1), dw.view(co, ci, 1, 3, 3),
                 prologue=F.PRO_AFFINE_RELU, pro_scale=sc.to(DEV), pro_shift=sh.to(DEV), perm_r=r, dy_shuffle=r)
    err = (dw.double().cpu() - wr.grad).abs().max().item()
    tol = (2e-5 if dtype == torch.float32 else 1e-2) * (1 + wr.grad.abs().max().item())
    assert err <= tol, err


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("combo", ["res", "mask", "mask+acc", "res+acc", "acc", "relu+mask+res+acc"])
@pytest.mark.parametrize("shape", [(2, 1, 16, 64, 64, 64, (1, 3, 3), (0, 1, 1)),
                                   (1, 4, 9, 40, 32, 32, (3, 3, 3), (1, 1, 1)),
                                   (2, 1, 10, 33, 64, 96, (1, 1, 1), (0, 0, 0))])
def test_conv_epilogue_combos(dtype, combo, shape):
    """Every epilogue form on its own and combined (the bf16 fast path
    specialises plain/residual/mask and routes the rest through a generic
    copy, whose absent views alias y and must not be applied)."""
    n, d, h, w, ci, co, k, pad = shape
    g = torch.Generator().manual_seed(11)
    x = torch.randn((n, d, h, w, ci), generator=g)
    wt = torch.randn((co, ci, *k), generator=g) / (ci * k[0] * k[1] * k[2]) ** 0.5
    b = torch.randn(co, generator=g)
    mask = torch.randn((n, d, h, w, co), generator=g)
    res = torch.randn((n, d, h, w, co), generator=g)
    y0 = torch.randn((n, d, h, w, co), generator=g)
    parts = set(combo.split("+"))
    ref = _ref_conv(_q(x, dtype), _q(wt, dtype), b.double(), pad) * 0.5
    if "relu" in parts:
        ref = torch.relu(ref)
    if "mask" in parts:
        ref = torch.where(_q(mask, dtype) > 0, ref, torch.zeros_like(ref))
    if "res" in parts:
        ref = ref + _q(res, dtype)
    if "acc" in parts:
        ref = ref + _q(y0, dtype)
    yd = y0.to(DEV, dtype)
    F.conv(x.to(DEV, dtype), F.pack_weight(wt.to(DEV), 0, dtype), yd, k, pad, bias=b.to(DEV), out_scale=0.5,
           act=F.ACT_RELU if "relu" in parts else F.ACT_NONE,
           mask=mask.to(DEV, dtype) if "mask" in parts else None,
           residual=res.to(DEV, dtype) if "res" in parts else None, accumulate="acc" in parts)
    err = (yd.double().cpu() - ref).abs().max().item()
    assert err <= _tol(dtype, ref) * 2, err


# Thin-channel kernels (conv_thin.hip): cin <= 4 (im2col k = (tap, c)) and
# cout <= 3 (m = (tap, co)), bf16 inputs, with every epilogue form; inputs in
# the nets' 8-channel padded storage as well as plain contiguous views.
THIN_FWD = [
    # (N, D, H, W, Cin, Cout, k, pad, padded_storage)
    (2, 1, 20, 45, 1, 64, (1, 3, 3), (0, 1, 1), True),
    (2, 1, 12, 33, 3, 48, (1, 3, 3), (0, 1, 1), False),
    (2, 4, 9, 40, 1, 32, (3, 3, 3), (1, 1, 1), True),
    (1, 1, 9, 35, 2, 256, (1, 3, 3), (0, 1, 1), False),
    (2, 3, 7, 19, 1, 40, (1, 1, 1), (0, 0, 0), True),
    (2, 1, 20, 70, 64, 1, (1, 3, 3), (0, 1, 1), False),
    (2, 1, 9, 33, 32, 3, (1, 3, 3), (0, 1, 1), False),
    (2, 2, 9, 33, 96, 2, (1, 1, 1), (0, 0, 0), False),
]


def _thin_input(x, padded):
    if not padded or x.shape[-1] >= 8:
        return x.to(DEV, torch.bfloat16)
    st = torch.zeros((*x.shape[:-1], 8), dtype=torch.bfloat16, device=DEV)
    st[..., :x.shape[-1]] = x.to(DEV, torch.bfloat16)
    return st[..., :x.shape[-1]]


@pytest.mark.parametrize("ydtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("case", THIN_FWD)
def test_thin_conv_forward(case, ydtype):
    n, d, h, w, ci, co, k, pad, padded = case
    g = torch.Generator().manual_seed(21)
    x = torch.randn((n, d, h, w, ci), generator=g)
    wt = torch.randn((co, ci, *k), generator=g) / (ci * k[0] * k[1] * k[2]) ** 0.5
    b = torch.randn(co, generator=g)
    do = d + 2 * pad[0] - k[0] + 1
    ref = _ref_conv(_q(x, torch.bfloat16), _q(wt, torch.bfloat16), b.double(), pad)
    y = torch.empty((n, do, h, w, co), dtype=ydtype, device=DEV)
    F.conv(_thin_input(x, padded), F.pack_weight(wt.to(DEV), 0, torch.bfloat16), y, k, pad, bias=b.to(DEV))
    err = (y.double().cpu() - ref).abs().max().item()
    assert err <= _tol(torch.bfloat16, ref), err


@pytest.mark.parametrize("case", [THIN_FWD[0], THIN_FWD[2], THIN_FWD[5], THIN_FWD[6]])
def test_thin_conv_fused(case):
    """prologue (BN-affine+ReLU), PReLU, out_scale, mask with slope, residual, accumulate."""
    n, d, h, w, ci, co, k, pad, padded = case
    g = torch.Generator().manual_seed(22)
    do = d + 2 * pad[0] - k[0] + 1
    x = torch.randn((n, d, h, w, ci), generator=g)
    wt = torch.randn((co, ci, *k), generator=g) / (ci * k[0] * k[1] * k[2]) ** 0.5
    b = torch.randn(co, generator=g)
    sc = torch.rand(ci, generator=g) + 0.5
    sh = torch.randn(ci, generator=g)
    slope = torch.tensor([0.25])
    mslope = torch.tensor([0.3])
    mask = torch.randn((n, do, h, w, co), generator=g)
    res = torch.randn((n, do, h, w, co), generator=g)
    y0 = torch.randn((n, do, h, w, co), generator=g)
    bf = torch.bfloat16
    xin = torch.relu(_q(x, bf) * sc.double() + sh.double()).to(bf).double()
    t = _ref_conv(xin, _q(wt, bf), b.double(), pad) * 0.5
    t = torch.where(t > 0, t, 0.25 * t)
    t = torch.where(_q(mask, bf) > 0, t, 0.3 * t)
    ref = t + _q(res, bf) + _q(y0, bf)
    yd = y0.to(DEV, bf)
    F.conv(_thin_input(x, padded), F.pack_weight(wt.to(DEV), 0, bf), yd, k, pad, bias=b.to(DEV),
           prologue=F.PRO_AFFINE_RELU, pro_scale=sc.to(DEV), pro_shift=sh.to(DEV), act=F.ACT_PRELU,
           act_param=slope.to(DEV), out_scale=0.5, mask=mask.to(DEV, bf), mask_slope=mslope.to(DEV),
           residual=res.to(DEV, bf), accumulate=True)
    err = (yd.double().cpu() - ref).abs().max().item()
    assert err <= _tol(bf, ref) * 2, err


@pytest.mark.parametrize("case", [(2, 1, 20, 70, 64, 1, (1, 3, 3), (0, 1, 1)),
                                  (2, 1, 9, 33, 32, 3, (1, 3, 3), (0, 1, 1)),
                                  (2, 2, 11, 40, 16, 2, (1, 1, 1), (0, 0, 0)),
                                  (1, 1, 13, 37, 128, 1, (1, 3, 3), (0, 1, 1))])
@pytest.mark.parametrize("prologue", [False, True])
def test_thin_wgrad(case, prologue):
    """weight/bias gradient of a cout <= 3 conv (the tail conv) against fp64 autograd."""
    n, d, h, w, ci, co, k, pad = case
    bf = torch.bfloat16
    g = torch.Generator().manual_seed(23)
    x = torch.randn((n, d, h, w, ci), generator=g)
    gy = torch.randn((n, d, h, w, co), generator=g)
    wt = torch.randn((co, ci, *k), generator=g) / 12
    sc = torch.rand(ci, generator=g) + 0.5
    sh = torch.randn(ci, generator=g)
    xin = _q(x, bf)
    if prologue:
        xin = torch.relu(xin * sc.double() + sh.double()).to(bf).double()
    wr = _q(wt, bf).requires_grad_(True)
    br = torch.zeros(co, dtype=torch.float64, requires_grad=True)
    _ref_conv(xin, wr, br, pad).backward(_q(gy, bf))
    dw = torch.empty((co, ci, *k), device=DEV)
    db = torch.empty(co, device=DEV)
    kw = dict(prologue=F.PRO_AFFINE_RELU, pro_scale=sc.to(DEV), pro_shift=sh.to(DEV)) if prologue else {}
    F.conv_wgrad(x.to(DEV, bf), _thin_input(gy, True), k, pad, dw, db, **kw)
    ew = (dw.double().cpu() - wr.grad).abs().max().item()
    eb = (db.double().cpu() - br.grad).abs().max().item()
    assert ew <= 1e-2 * (1 + wr.grad.abs().max().item()), ew
    assert eb <= 1e-2 * (1 + br.grad.abs().max().item()), eb


@pytest.mark.parametrize("case", THIN_FWD)
def test_thin_matches_generic(case):
    """thin-channel kernels == the generic implicit-GEMM kernels on the same bf16 operands
    (forward, data gradient) up to accumulation order."""
    n, d, h, w, ci, co, k, pad, padded = case
    g = torch.Generator().manual_seed(26)
    bf = torch.bfloat16
    x = _thin_input(torch.randn((n, d, h, w, ci), generator=g), padded)
    wt = (torch.randn((co, ci, *k), generator=g) / (ci * k[0] * k[1] * k[2]) ** 0.5).to(DEV)
    b = torch.randn(co, generator=g).to(DEV)
    do = d + 2 * pad[0] - k[0] + 1
    gy = _thin_input(torch.randn((n, do, h, w, co), generator=g), True)
    dpad = tuple(kk - 1 - p for kk, p in zip(k, pad))
    outs = []
    for mode in (1, 0):
        F.set_conv_path("thin", mode)
        try:
            y = torch.empty((n, do, h, w, co), dtype=torch.float32, device=DEV)
            F.conv(x, F.pack_weight(wt, 0, bf), y, k, pad, bias=b)
            dx = torch.empty((n, d, h, w, ci), dtype=torch.float32, device=DEV)
            F.conv(gy, F.pack_weight(wt, 1, bf), dx, k, dpad)
            outs.append((y, dx))
        finally:
            F.set_conv_path("thin", -1)
    for a_, b_ in zip(outs[0], outs[1]):
        assert (a_ - b_).abs().max().item() <= 1e-4 * (1 + b_.abs().max().item())


@pytest.mark.parametrize("case", THIN_FWD)
def test_thin_conv_fp16(case):
    """fp16 instantiation of the thin-channel kernels (forward and, for the
    cout <= 3 cases, the weight gradient) against fp64."""
    n, d, h, w, ci, co, k, pad, padded = case
    H = torch.float16
    g = torch.Generator().manual_seed(27)
    x = torch.randn((n, d, h, w, ci), generator=g)
    wt = torch.randn((co, ci, *k), generator=g) / (ci * k[0] * k[1] * k[2]) ** 0.5
    b = torch.randn(co, generator=g)
    do = d + 2 * pad[0] - k[0] + 1
    ref = _ref_conv(_q(x, H), _q(wt, H), b.double(), pad)
    if ci < 8 and padded:
        xs = torch.zeros((*x.shape[:-1], 8), dtype=H, device=DEV)
        xs[..., :ci] = x.to(DEV, H)
        xd = xs[..., :ci]
    else:
        xd = x.to(DEV, H)
    y = torch.empty((n, do, h, w, co), dtype=torch.float32, device=DEV)
    F.conv(xd, F.pack_weight(wt.to(DEV), 0, H), y, k, pad, bias=b.to(DEV))
    err = (y.double().cpu() - ref).abs().max().item()
    assert err <= _tol(H, ref), err
    if co <= 3 and ci % 8 == 0 and k[0] == 1:
        gy = torch.randn((n, do, h, w, co), generator=g)
        gys = torch.zeros((n, do, h, w, 8), dtype=H, device=DEV)
        gys[..., :co] = gy.to(DEV, H)
        wr = _q(wt, H).requires_grad_(True)
        br = torch.zeros(co, dtype=torch.float64, requires_grad=True)
        _ref_conv(_q(x, H), wr, br, pad).backward(_q(gy, H))
        dw = torch.empty((co, ci, *k), device=DEV)
        db = torch.empty(co, device=DEV)
        F.conv_wgrad(x.to(DEV, H), gys[..., :co], k, pad, dw, db)
        ew = (dw.double().cpu() - wr.grad).abs().max().item()
        assert ew <= 2e-3 * (1 + wr.grad.abs().max().item()), ew
