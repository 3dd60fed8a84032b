"""Parity of the rolling-depth Conv3d 3x3x3 weight gradient
(conv_wgrad_roll.hip: dW / dbias of DUF's dense-unit convs, duf_net.py:203,214)
against torch fp64 autograd on the CPU.

The kernel walks the input depth slices of a tile once, keeps the output
gradient slices of the three kd taps in a five-slot ring and all 27 taps of a
32 x 32 channel block in registers, so the cases cover what that walk can get
wrong: depth padding 1, 0 and 2, fewer slices than taps, partial row / column
tiles, 32-channel blocks of wider inputs (the concat layout: a channel slice
of a wider buffer), the BN-affine+ReLU prologue applied in LDS, the bias, and
tiles that cover part of the depth range (the depth-run knob) or several
tiles per workgroup (the grid cap).

The per-workgroup fp32 sums depend on the tiling, so the settings are each
held to the fp64 bound, and every setting is reproducible bitwise (the slab
reduce sums in a fixed order).  Inputs are rounded to the 16-bit type (and
the prologue output too) before the fp64 reference; the kernel accumulates
in fp32: max |d| <= 2e-3 * max|ref| for dW and dbias.
"""
import pytest
import torch
import torch.nn.functional as Fn

from vsr_amd import functional as F

pytestmark = pytest.mark.gpu
DEV = "cuda"

CASES = [
    # (N, D, H, W, Cin, Cout, depth pad, channel offset in a wider buffer)
    (2, 5, 9, 35, 32, 32, 1, 0),      # partial row / column tiles
    (1, 7, 16, 32, 64, 32, 1, 32),    # DUF pad-1 unit shape, sliced input
    (1, 7, 12, 40, 96, 32, 0, 0),     # depth-valid unit: 7 -> 5
    (2, 3, 17, 33, 32, 64, 0, 0),     # 3 -> 1 output depth, two output blocks
    (1, 5, 10, 34, 32, 96, 2, 0),     # pad 2: 5 -> 7
    (1, 3, 16, 32, 224, 32, 0, 0),    # the last depth-valid unit (F = 224)
    (1, 2, 6, 9, 32, 32, 1, 0),       # fewer slices than kd taps
]


def _inputs(case, dtype, seed=0):
    n, d, h, w, ci, co, pdp, off = case
    g = torch.Generator().manual_seed(seed)
    big = torch.randn((n, d, h, w, off + ci + 32), generator=g)
    do = d + 2 * pdp - 2
    gy = torch.randn((n, do, h, w, co), generator=g)
    sc = torch.rand(ci, generator=g) + 0.5
    sh = torch.randn(ci, generator=g) * 0.5
    return big, gy, sc, sh


def _reference(case, dtype, prologue, big, gy, sc, sh):
    n, d, h, w, ci, co, pdp, off = case
    xin = big[..., off:off + ci].to(dtype).double()
    if prologue:
        xin = torch.relu(xin * sc.double() + sh.double()).to(dtype).double()
    wr = torch.zeros((co, ci, 3, 3, 3), dtype=torch.float64, requires_grad=True)
    br = torch.zeros(co, dtype=torch.float64, requires_grad=True)
    y = Fn.conv3d(xin.permute(0, 4, 1, 2, 3), wr, br, padding=(pdp, 1, 1))
    y.backward(gy.to(dtype).double().permute(0, 4, 1, 2, 3))
    return wr.grad, br.grad


def _run(case, dtype, prologue, big, gy, sc, sh, depth=0, cap=0, roll=1, bias=True):
    """roll=1 forces the rolling kernel (the default skips <= 3 output depths)"""
    n, d, h, w, ci, co, pdp, off = case
    kw = dict(prologue=F.PRO_AFFINE_RELU, pro_scale=sc.to(DEV), pro_shift=sh.to(DEV)) if prologue else {}
    dw = torch.empty((co, ci, 3, 3, 3), dtype=torch.float32, device=DEV)
    db = torch.empty(co, dtype=torch.float32, device=DEV) if bias else None
    F.set_roll_depth(depth)
    F.set_grid_cap(cap)
    F.set_conv_path("wgrad_roll", roll)
    try:
        F.conv_wgrad(big.to(DEV, dtype)[..., off:off + ci], gy.to(DEV, dtype), (3, 3, 3), (pdp, 1, 1), dw, db, **kw)
    finally:
        F.set_roll_depth(0)
        F.set_grid_cap(0)
        F.set_conv_path("wgrad_roll", -1)
    torch.cuda.synchronize()
    return dw.double().cpu(), (db.double().cpu() if bias else None)


def _check(dw, db, wref, bref):
    ew = (dw - wref).abs().max().item()
    tw = 2e-3 * max(wref.abs().max().item(), 1e-3)
    assert ew <= tw, (ew, tw)
    if db is not None:
        eb = (db - bref).abs().max().item()
        tb = 2e-3 * max(bref.abs().max().item(), 1e-3)
        assert eb <= tb, (eb, tb)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("prologue", [False, True])
@pytest.mark.parametrize("case", CASES)
def test_wgrad_roll(case, prologue, dtype):
    big, gy, sc, sh = _inputs(case, dtype)
    wref, bref = _reference(case, dtype, prologue, big, gy, sc, sh)
    dw, db = _run(case, dtype, prologue, big, gy, sc, sh)
    _check(dw, db, wref, bref)
    dw2, db2 = _run(case, dtype, prologue, big, gy, sc, sh)
    assert torch.equal(dw, dw2) and torch.equal(db, db2), "not reproducible"


@pytest.mark.parametrize("case", CASES)
def test_wgrad_roll_tiling(case):
    """depth runs of 1, 2, 3 output depths, a capped grid (many tiles per
    workgroup: the ring crosses tiles) and no bias: each within the fp64
    bound and reproducible"""
    dtype = torch.bfloat16
    big, gy, sc, sh = _inputs(case, dtype, seed=3)
    wref, bref = _reference(case, dtype, True, big, gy, sc, sh)
    for depth, cap in ((1, 0), (2, 0), (3, 0), (0, 1), (0, 3), (2, 5), (1, 1)):
        dw, db = _run(case, dtype, True, big, gy, sc, sh, depth, cap)
        _check(dw, db, wref, bref)
        dw2, db2 = _run(case, dtype, True, big, gy, sc, sh, depth, cap)
        assert torch.equal(dw, dw2) and torch.equal(db, db2), (depth, cap)
    dw, _ = _run(case, dtype, True, big, gy, sc, sh, bias=False)
    _check(dw, None, wref, None)


def test_wgrad_roll_switch():
    """the rolling kernel and the per-kd pipelined kernel agree to fp32
    summation order at a DUF unit shape (the switch really changes path)"""
    case = (2, 7, 16, 64, 64, 32, 1, 0)
    dtype = torch.bfloat16
    big, gy, sc, sh = _inputs(case, dtype, seed=5)
    wref, bref = _reference(case, dtype, True, big, gy, sc, sh)
    dw_r, db_r = _run(case, dtype, True, big, gy, sc, sh, roll=1)
    dw_p, db_p = _run(case, dtype, True, big, gy, sc, sh, roll=0)
    _check(dw_r, db_r, wref, bref)
    _check(dw_p, db_p, wref, bref)
    assert not torch.equal(dw_r, dw_p)
    assert (dw_r - dw_p).abs().max().item() <= 1e-4 * wref.abs().max().item()


def test_wgrad_roll_accumulate_scale():
    """accumulate adds into dW / dbias, dy_scale scales (the fp16 loss-scale
    and gradient-accumulation paths)"""
    case = (1, 5, 16, 32, 64, 32, 1, 0)
    dtype = torch.float16
    big, gy, sc, sh = _inputs(case, dtype, seed=9)
    wref, bref = _reference(case, dtype, True, big, gy, sc, sh)
    kw = dict(prologue=F.PRO_AFFINE_RELU, pro_scale=sc.to(DEV), pro_shift=sh.to(DEV))
    dw = torch.full((32, 64, 3, 3, 3), 1.0, device=DEV)
    db = torch.full((32,), -2.0, device=DEV)
    F.conv_wgrad(big.to(DEV, dtype)[..., :64], gy.to(DEV, dtype), (3, 3, 3), (1, 1, 1), dw, db, dy_scale=0.25,
                 accumulate=True, **kw)
    torch.cuda.synchronize()
    _check(((dw.double().cpu() - 1.0) * 4), ((db.double().cpu() + 2.0) * 4), wref, bref)
