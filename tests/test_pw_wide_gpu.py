"""Parity of the wide pointwise GEMM kernel (conv_pw_wide.hip) against torch
fp64: DUF's filter-head convs (duf_net.py:40-46) and their data gradients --
512 -> 400 to fp32 logits with bias, 256 -> 512 with ReLU prologue and ReLU,
400 -> 512 and 512 -> 256 data gradients with the ReLU mask and the
accumulate -- on voxel counts that are not a multiple of the 256-voxel tile,
channel-slice views, fp16, and against the kernels it replaces (pw_wide off).
16-bit operands are rounded before the fp64 reference: max|d| <= 1.5e-2
max|ref| (bf16), 2e-3 (fp16), fp32 outputs 1e-2."""
import pytest
import torch

from vsr_amd import functional as F

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _q(t, dt):
    return t.to(dt).double()


@pytest.fixture(autouse=True)
def _wide_default():
    yield
    F.set_conv_path("pw_wide", -1)


CASES = {
    # name: (cin, cout, y fp32, prologue relu, act relu, mask, accumulate, weight mode)
    "fn2_fwd": (512, 400, True, False, False, False, False, 0),
    "fn1_fwd": (256, 512, False, True, True, False, False, 0),
    "fn2_dgrad": (400, 512, False, False, False, True, False, 1),
    "fn1_dgrad": (512, 256, False, False, False, True, True, 1),
    "rn1_fwd": (256, 256, False, True, True, False, False, 0),
}


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("case", sorted(CASES))
@pytest.mark.parametrize("shape", [(2, 1, 17, 45), (1, 3, 16, 32)])
def test_pw_wide(case, shape, dtype):
    ci, co, yf, pro, act, msk, acc, mode = CASES[case]
    g = torch.Generator().manual_seed(ci + co + shape[2])
    n, d, h, w = shape
    xb = torch.randn((n, d, h, w, ci + 16), generator=g)
    x = xb[..., 8:8 + ci]  # a channel slice: voxel stride != channels
    # weight of the conv as run: y = x W^T (mode 1 packs the transposed forward weight)
    wf = torch.randn((ci, co) if mode else (co, ci), generator=g) / ci ** 0.5
    wr = wf.t() if mode else wf  # (co, ci)
    b = torch.randn(co, generator=g) if not mode else None
    m = torch.randn((n, d, h, w, co), generator=g) if msk else None
    y0 = torch.randn((n, d, h, w, co), generator=g)
    xin = _q(x, dtype)
    if pro:
        xin = torch.relu(xin)
    ref = torch.einsum("ndhwc,oc->ndhwo", xin, _q(wr, dtype))
    if b is not None:
        ref = ref + b.double()
    if act:
        ref = torch.relu(ref)
    if msk:
        ref = torch.where(_q(m, dtype) > 0, ref, torch.zeros_like(ref))
    ydt = torch.float32 if yf else dtype
    if acc:
        ref = ref + y0.to(ydt).double()
    wshape = (ci, co, 1, 1, 1) if mode else (co, ci, 1, 1, 1)
    wp = F.pack_weight(wf.reshape(wshape).to(DEV), mode, dtype)
    outs = []
    for wide in (1, 0):
        F.set_conv_path("pw_wide", wide)
        yb = torch.full((n, d, h, w, co + 8), 3.0, dtype=ydt, device=DEV)
        y = yb[..., :co]
        if acc:
            y.copy_(y0.to(DEV, ydt))
        F.conv(xb.to(DEV, dtype)[..., 8:8 + ci], wp, y, (1, 1, 1), (0, 0, 0),
               bias=b.to(DEV) if b is not None else None, prologue=F.PRO_RELU if pro else F.PRO_NONE,
               act=F.ACT_RELU if act else F.ACT_NONE, mask=m.to(DEV, dtype) if msk else None, accumulate=acc)
        assert (yb[..., co:] == 3.0).all()  # past the view: untouched
        outs.append(y.double().cpu())
    tol = 1e-2 if yf else (2e-3 if dtype == torch.float16 else 1.5e-2)
    scale = ref.abs().max().item()
    for out in outs:
        err = (out - ref).abs().max().item()
        assert err <= tol * scale, (err, scale)
