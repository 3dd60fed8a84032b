"""Parity of the pointwise (1x1x1) bf16 conv kernels (conv_pw.hip) against
torch fp64: forward / data gradient with every prologue and epilogue form the
generators use, on channel- and depth-slice views of concat buffers (DUF's
dense-unit layout, duf_net.py:195-214), output-channel chunks (the 256->512
filter head, duf_net.py:40-44), and the weight gradient incl. cin/cout chunks,
split tails and grid caps (several tiles / voxel ranges per workgroup).

bf16 operands are rounded before the fp64 reference, so only accumulation
order and the final store differ: forward max|d| <= 1.5e-2 max|ref|, weight
gradient max|d| <= 1e-2 (1 + max|ref|)."""
import pytest
import torch
import torch.nn.functional as Fn

from vsr_amd import functional as F

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _fused_on(monkeypatch):
    """the fused entry points are tested whatever VSRK_FUSE says for the nets"""
    monkeypatch.setattr(F, "FUSE", True)


DEV = "cuda"
BF = torch.bfloat16


def _q(t, dt=BF):
    return t.to(dt).double()


def _ref1x1(x_cl, w, b):
    """x (N,D,H,W,Ci) fp64, w (Co,Ci) -> (N,D,H,W,Co)."""
    y = torch.einsum("ndhwc,oc->ndhwo", x_cl, w)
    return y + b if b is not None else y


@pytest.fixture(params=[0, 1, 3])
def grid_cap(request):
    F.set_grid_cap(request.param)
    yield request.param
    F.set_grid_cap(0)


@pytest.mark.parametrize("dhw", [(3, 7, 19), (2, 8, 32)])
@pytest.mark.parametrize("c", [64, 80, 96, 128, 160, 192, 224, 256])
def test_pw_forward_prologue_slices(c, dhw, grid_cap):
    """BN-affine+ReLU prologue on a channel slice of a concat buffer, output into
    a channel slice of another buffer, bias; tails of voxels (N*D*H*W not a
    multiple of the tile) and tiles aligned to samples (d*h*w % 128 == 0)."""
    g = torch.Generator().manual_seed(c)
    n, (d, h, w) = 2, dhw
    big = torch.randn((n, d, h, w, c + 40), generator=g)
    wt = torch.randn((c, c), generator=g) / c ** 0.5
    b = torch.randn(c, generator=g)
    sc = torch.rand(c, generator=g) + 0.5
    sh = torch.randn(c, generator=g)
    xin = torch.relu(_q(big[..., 8:8 + c]) * sc.double() + sh.double()).to(BF).double()
    ref = _ref1x1(xin, _q(wt), b.double())
    yb = torch.full((n, d, h, w, c + 24), 7.0, dtype=BF, device=DEV)
    bigd = big.to(DEV, BF)
    F.conv(bigd[..., 8:8 + c], F.pack_weight(wt.view(c, c, 1, 1, 1).to(DEV), 0, BF), yb[..., 16:16 + c],
           (1, 1, 1), (0, 0, 0), bias=b.to(DEV), prologue=F.PRO_AFFINE_RELU, pro_scale=sc.to(DEV),
           pro_shift=sh.to(DEV))
    y = yb[..., 16:16 + c].double().cpu()
    err = (y - ref).abs().max().item()
    assert err <= 1.5e-2 * ref.abs().max().item(), err
    # the rest of the output buffer is untouched
    assert (yb[..., :16] == 7.0).all() and (yb[..., 16 + c:] == 7.0).all()


def test_pw_forward_depth_slice_head_chunks(grid_cap):
    """256 -> 512 with ReLU prologue and ReLU act (filterNet.conv1) on a depth
    slice (n stride != d*h*w*c): two 256-channel output chunks."""
    g = torch.Generator().manual_seed(7)
    n, D, h, w, ci, co = 3, 5, 6, 21, 256, 512
    big = torch.randn((n, D, h, w, ci), generator=g)
    x = big[:, 2:3]
    wt = torch.randn((co, ci), generator=g) / ci ** 0.5
    b = torch.randn(co, generator=g)
    ref = torch.relu(_ref1x1(torch.relu(_q(x)), _q(wt), b.double()))
    y = torch.empty((n, 1, h, w, co), dtype=BF, device=DEV)
    F.conv(big.to(DEV, BF)[:, 2:3], F.pack_weight(wt.view(co, ci, 1, 1, 1).to(DEV), 0, BF), y, (1, 1, 1),
           (0, 0, 0), bias=b.to(DEV), prologue=F.PRO_RELU, act=F.ACT_RELU)
    err = (y.double().cpu() - ref).abs().max().item()
    assert err <= 1.5e-2 * ref.abs().max().item(), err


@pytest.mark.parametrize("combo", ["mask", "acc", "mask+acc"])
@pytest.mark.parametrize("c", [64, 128, 192, 256])
def test_pw_data_gradient_epilogues(c, combo, grid_cap):
    """dgrad form (mode-1 packed weight, no prologue) with the ReLU mask of the
    forward output and / or accumulation into an existing gradient."""
    g = torch.Generator().manual_seed(c + 1)
    n, d, h, w = 2, 2, 9, 13
    gy = torch.randn((n, d, h, w, c), generator=g)
    wt = torch.randn((c, c), generator=g) / c ** 0.5
    mask = torch.randn((n, d, h, w, c), generator=g)
    y0 = torch.randn((n, d, h, w, c), generator=g)
    parts = set(combo.split("+"))
    ref = torch.einsum("ndhwo,oc->ndhwc", _q(gy), _q(wt)) * 0.5
    if "mask" in parts:
        ref = torch.where(_q(mask) > 0, ref, torch.zeros_like(ref))
    if "acc" in parts:
        ref = ref + _q(y0)
    yd = y0.to(DEV, BF)
    F.conv(gy.to(DEV, BF), F.pack_weight(wt.view(c, c, 1, 1, 1).to(DEV), 1, BF), yd, (1, 1, 1), (0, 0, 0),
           out_scale=0.5, mask=mask.to(DEV, BF) if "mask" in parts else None, accumulate="acc" in parts)
    err = (yd.double().cpu() - ref).abs().max().item()
    assert err <= 2 * 1.5e-2 * ref.abs().max().item(), err


@pytest.mark.parametrize("ci,co", [(64, 64), (96, 96), (160, 160), (224, 224), (256, 256), (256, 512),
                                   (512, 400), (48, 130), (80, 72)])
@pytest.mark.parametrize("prologue", [False, True])
def test_pw_weight_gradient(ci, co, prologue, grid_cap):
    g = torch.Generator().manual_seed(ci * 3 + co)
    n, D, h, w = 2, 4, 5, 23
    big = torch.randn((n, D, h, w, ci + 16), generator=g)
    x = big[:, 1:4, :, :, 8:8 + ci]  # depth and channel slice
    gy = torch.randn((n, 3, h, w, co), generator=g)
    sc = torch.rand(ci, generator=g) + 0.5
    sh = torch.randn(ci, generator=g)
    xin = _q(x)
    if prologue:
        xin = torch.relu(xin * sc.double() + sh.double()).to(BF).double()
    ref_w = torch.einsum("ndhwo,ndhwc->oc", _q(gy), xin)
    ref_b = _q(gy).sum((0, 1, 2, 3))
    dw = torch.empty((co, ci, 1, 1, 1), device=DEV)
    db = torch.empty(co, device=DEV)
    kw = dict(prologue=F.PRO_AFFINE_RELU, pro_scale=sc.to(DEV), pro_shift=sh.to(DEV)) if prologue else {}
    F.conv_wgrad(big.to(DEV, BF)[:, 1:4, :, :, 8:8 + ci], gy.to(DEV, BF), (1, 1, 1), (0, 0, 0), dw, db, **kw)
    ew = (dw.view(co, ci).double().cpu() - ref_w).abs().max().item()
    eb = (db.double().cpu() - ref_b).abs().max().item()
    assert ew <= 1e-2 * (1 + ref_w.abs().max().item()), ew
    assert eb <= 1e-2 * (1 + ref_b.abs().max().item()), eb


def test_pw_weight_gradient_accumulate_scale_deterministic():
    g = torch.Generator().manual_seed(99)
    x = torch.randn((2, 7, 16, 40, 160), generator=g).to(DEV, BF)
    gy = torch.randn((2, 7, 16, 40, 160), generator=g).to(DEV, BF)
    outs = []
    for _ in range(2):
        dw = torch.ones((160, 160, 1, 1, 1), device=DEV)
        db = torch.ones(160, device=DEV)
        F.conv_wgrad(x, gy, (1, 1, 1), (0, 0, 0), dw, db, dy_scale=0.25, accumulate=True)
        outs.append((dw, db))
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    ref = torch.einsum("ndhwo,ndhwc->oc", gy.double(), x.double()).cpu() * 0.25 + 1
    assert (outs[0][0].view(160, 160).double().cpu() - ref).abs().max().item() <= 1e-2 * ref.abs().max().item()


@pytest.mark.parametrize("c", [64, 192])
def test_pw_matches_tile_kernels(c):
    """pointwise kernels == the tile kernels (path "pw" off) on the same bf16
    operands, forward with prologue, data gradient and weight gradient."""
    g = torch.Generator().manual_seed(5 + c)
    x = torch.randn((2, 3, 11, 33, c), generator=g).to(DEV, BF)
    gy = torch.randn((2, 3, 11, 33, c), generator=g).to(DEV, BF)
    wt = (torch.randn((c, c, 1, 1, 1), generator=g) / c ** 0.5).to(DEV)
    b = torch.randn(c, generator=g).to(DEV)
    sc = (torch.rand(c, generator=g) + 0.5).to(DEV)
    sh = torch.randn(c, generator=g).to(DEV)
    res = []
    for mode in (1, 0):
        F.set_conv_path("pw", mode)
        try:
            y = torch.empty_like(x)
            F.conv(x, F.pack_weight(wt, 0, BF), y, (1, 1, 1), (0, 0, 0), bias=b, prologue=F.PRO_AFFINE_RELU,
                   pro_scale=sc, pro_shift=sh)
            dx = torch.empty_like(x)
            F.conv(gy, F.pack_weight(wt, 1, BF), dx, (1, 1, 1), (0, 0, 0))
            dw = torch.empty((c, c, 1, 1, 1), device=DEV)
            db = torch.empty(c, device=DEV)
            F.conv_wgrad(x, gy, (1, 1, 1), (0, 0, 0), dw, db, prologue=F.PRO_AFFINE_RELU, pro_scale=sc,
                         pro_shift=sh)
            res.append((y.float(), dx.float(), dw, db))
        finally:
            F.set_conv_path("pw", -1)
    for a_, b_ in zip(res[0], res[1]):
        # bf16 outputs may differ by one rounding step; fp32 gradients by summation order
        assert (a_ - b_).abs().max().item() <= 1e-2 * (1 + b_.abs().max().item())


@pytest.mark.parametrize("c", [64, 160, 256])
def test_pw_fp16_forward_and_weight_gradient(c):
    """fp16 instantiation (v_mfma_f32_32x32x16_f16): forward with prologue into
    a channel slice, and the weight gradient; 11-bit rounding -> 2e-3 bounds."""
    H = torch.float16
    g = torch.Generator().manual_seed(3 * c)
    n, d, h, w = 2, 2, 8, 32
    big = torch.randn((n, d, h, w, c + 16), generator=g)
    wt = torch.randn((c, c), generator=g) / c ** 0.5
    b = torch.randn(c, generator=g)
    sc = torch.rand(c, generator=g) + 0.5
    sh = torch.randn(c, generator=g)
    xin = torch.relu(_q(big[..., 8:8 + c], H) * sc.double() + sh.double()).to(H).double()
    ref = _ref1x1(xin, _q(wt, H), b.double())
    y = torch.empty((n, d, h, w, c), dtype=H, device=DEV)
    bigd = big.to(DEV, H)
    F.conv(bigd[..., 8:8 + c], F.pack_weight(wt.view(c, c, 1, 1, 1).to(DEV), 0, H), y, (1, 1, 1), (0, 0, 0),
           bias=b.to(DEV), prologue=F.PRO_AFFINE_RELU, pro_scale=sc.to(DEV), pro_shift=sh.to(DEV))
    err = (y.double().cpu() - ref).abs().max().item()
    assert err <= 2e-3 * ref.abs().max().item(), err
    gy = torch.randn((n, d, h, w, c), generator=g)
    ref_w = torch.einsum("ndhwo,ndhwc->oc", _q(gy, H), xin)
    dw = torch.empty((c, c, 1, 1, 1), device=DEV)
    db = torch.empty(c, device=DEV)
    F.conv_wgrad(bigd[..., 8:8 + c], gy.to(DEV, H), (1, 1, 1), (0, 0, 0), dw, db, prologue=F.PRO_AFFINE_RELU,
                 pro_scale=sc.to(DEV), pro_shift=sh.to(DEV))
    ew = (dw.view(c, c).double().cpu() - ref_w).abs().max().item()
    assert ew <= 2e-3 * (1 + ref_w.abs().max().item()), ew


@pytest.mark.parametrize("ci,co", [(128, 64), (192, 64), (256, 64), (256, 16), (64, 128), (64, 192), (64, 256)])
@pytest.mark.parametrize("form", ["plain", "prologue+relu", "prelu", "mask+acc", "prelu-mask"])
def test_pw_non_square(ci, co, form, grid_cap):
    """Narrowing 1x1 convs (cout < cin: DRF's feedback projections
    Conv2d((i+1)F, F, 1) + PReLU at low and high resolution,
    drf_net.py:81-92; DUF's residual head 256 -> 16, duf_net.py:46-49) and
    widening ones (their data gradients F -> (i+1)F, accumulated) on the
    staged kernel with one output chunk: channel-slice input and output
    views, every epilogue form."""
    g = torch.Generator().manual_seed(ci + 7 * co)
    n, d, h, w = 2, 1, 13, 40
    big = torch.randn((n, d, h, w, ci + 32), generator=g)
    wt = torch.randn((co, ci), generator=g) / ci ** 0.5
    b = torch.randn(co, generator=g)
    sc = torch.rand(ci, generator=g) + 0.5
    sh = torch.randn(ci, generator=g)
    mask = torch.randn((n, d, h, w, co), generator=g)
    y0 = torch.randn((n, d, h, w, co + 64), generator=g)
    slope = torch.tensor([0.2])
    xin = _q(big[..., 16:16 + ci])
    kw = {}
    if form == "prologue+relu":
        xin = torch.relu(xin * sc.double() + sh.double()).to(BF).double()
        kw = dict(bias=b.to(DEV), prologue=F.PRO_AFFINE_RELU, pro_scale=sc.to(DEV), pro_shift=sh.to(DEV),
                  act=F.ACT_RELU)
    elif form == "plain":
        kw = dict(bias=b.to(DEV))
    elif form == "prelu":
        kw = dict(bias=b.to(DEV), act=F.ACT_PRELU, act_param=slope.to(DEV))
    ref = torch.einsum("ndhwc,oc->ndhwo", xin, _q(wt))
    if form == "plain":
        ref = ref + b.double()
    if form == "prelu":
        ref = ref + b.double()
        ref = torch.where(ref > 0, ref, 0.2 * ref)
    if form == "prologue+relu":
        ref = torch.relu(ref + b.double())
    if form == "mask+acc":
        ref = torch.where(_q(mask) > 0, ref, torch.zeros_like(ref)) + _q(y0[..., 32:32 + co])
        kw = dict(mask=mask.to(DEV, BF), accumulate=True)
    if form == "prelu-mask":
        ref = torch.where(_q(mask) > 0, ref, 0.2 * ref)
        kw = dict(mask=mask.to(DEV, BF), mask_slope=slope.to(DEV))
    yb = y0.to(DEV, BF)
    F.conv(big.to(DEV, BF)[..., 16:16 + ci], F.pack_weight(wt.view(co, ci, 1, 1, 1).to(DEV), 0, BF),
           yb[..., 32:32 + co], (1, 1, 1), (0, 0, 0), **kw)
    y = yb[..., 32:32 + co].double().cpu()
    err = (y - ref).abs().max().item()
    assert err <= 2 * 1.5e-2 * ref.abs().max().item(), err
    assert torch.equal(yb[..., :32].cpu(), y0[..., :32].to(BF)) and torch.equal(yb[..., 32 + co:].cpu(),
                                                                                 y0[..., 32 + co:].to(BF))


@pytest.mark.parametrize("c", [64, 96, 160, 224])
@pytest.mark.parametrize("mode", ["stats", "bn_backward"])
def test_pw_fused_reduce(c, mode, grid_cap):
    """vsrk_conv_fwd_reduce: DUF's conv1 with bn2's statistics fused into the
    store pass (duf_net.py:198-201), and its data gradient with bn1's
    BN+ReLU backward reduce fused (duf_net.py:198-200), on the dense-unit
    views (a depth window of a channel slice of the concat buffer).  The
    output equals the unfused conv bitwise; the sums match the separate
    reduction kernels within fp32 summation-order noise."""
    g = torch.Generator().manual_seed(c + (1 if mode == "stats" else 2))
    n, D, h, w = 2, 5, 9, 37
    big = torch.randn((n, D, h, w, c + 32), generator=g).to(DEV, BF)
    R = big[:, 1:4, :, :, :c]
    wt = (torch.randn((c, c, 1, 1, 1), generator=g) / c ** 0.5).to(DEV)
    b = torch.randn(c, generator=g).to(DEV)
    sc = (torch.rand(c, generator=g) + 0.5).to(DEV)
    sh = torch.randn(c, generator=g).to(DEV)
    if mode == "stats":
        x, wp = R, F.pack_weight(wt, 0, BF)
        kw = dict(bias=b, prologue=F.PRO_AFFINE_RELU, pro_scale=sc, pro_shift=sh)
    else:
        x, wp = torch.randn((n, 3, h, w, c), generator=g).to(DEV, BF), F.pack_weight(wt, 1, BF)
        kw = {}
        st = torch.stack([sc, sh, torch.randn(c, generator=g).to(DEV) * 0.1, (torch.rand(c, generator=g) + 0.5).to(DEV)])
    y_ref = torch.empty((n, 3, h, w, c), dtype=BF, device=DEV)
    F.conv(x, wp, y_ref, (1, 1, 1), (0, 0, 0), **kw)
    y = torch.empty_like(y_ref)
    if mode == "stats":
        red = F.conv_reduce(x, wp, y, **kw)
        ref = F.bn_stats(y_ref)
    else:
        red = F.conv_reduce(x, wp, y, bnx=R, st=st)
        ref = F.bn_relu_bwd_reduce(R, y_ref, st)
    assert red is not None
    assert torch.equal(y, y_ref)
    err = (red - ref).abs().max().item()
    assert err <= 1e-5 * (1 + ref.abs().max().item()), err
    # deterministic: the same launch twice gives the same sums bitwise
    y2 = torch.empty_like(y)
    red2 = F.conv_reduce(x, wp, y2, **kw) if mode == "stats" else F.conv_reduce(x, wp, y2, bnx=R, st=st)
    assert torch.equal(red, red2)


def test_pw_fused_reduce_unsupported_shape_launches_nothing():
    """256 channels (no staged square kernel) -> None, y untouched."""
    x = torch.randn((1, 1, 4, 8, 256)).to(DEV, BF)
    y = torch.full((1, 1, 4, 8, 256), 3.0, dtype=BF, device=DEV)
    wp = F.pack_weight(torch.randn((256, 256, 1, 1, 1), device=DEV), 1, BF)
    assert F.conv_reduce(x, wp, y, bnx=x, st=torch.ones((4, 256), device=DEV)) is None
    assert (y == 3.0).all()


@pytest.mark.parametrize("c", [64, 96, 128, 160, 192, 224])
@pytest.mark.parametrize("alias,hw", [(False, (9, 37)), (True, (9, 37)), (True, (8, 32))])
def test_pw_fused_reduce_bnb(c, alias, hw, grid_cap):
    """vsrk_conv_fwd_reduce_bnb: DUF's conv1 data gradient whose input is
    bn2's BN+ReLU backward apply, computed in the operand load
    (duf_net.py:198-201), with bn1's backward reduce in the store pass.  The
    applied gradient (x_out, the weight gradient's dY) equals
    bn_relu_bwd_apply bitwise, the conv output equals apply + conv bitwise
    (also written over the input gradient's own storage, as the net does),
    the sums match the separate reduction within fp32 summation noise, and
    a second launch repeats them bitwise."""
    g = torch.Generator().manual_seed(c + 7 * alias + hw[1])
    (n, D), (h, w) = (2, 5), hw  # 8 x 32: whole tiles per sample (the aligned kernel form)
    big = torch.randn((n, D, h, w, c + 32), generator=g).to(DEV, BF)
    R = big[:, 1:4, :, :, :c]                     # bn1's input (a concat-buffer view)
    t1 = torch.randn((n, 3, h, w, c + 16), generator=g).to(DEV, BF)[..., 8:8 + c]  # bn2's input, strided
    dz2 = torch.randn((n, 3, h, w, c), generator=g).to(DEV, BF)
    wt = (torch.randn((c, c, 1, 1, 1), generator=g) / c ** 0.5).to(DEV)
    wp = F.pack_weight(wt, 1, BF)

    def bn_consts():
        gm = (torch.rand(c, generator=g) + 0.5).to(DEV)
        ist = (torch.rand(c, generator=g) + 0.5).to(DEV)
        mu = (torch.randn(c, generator=g) * 0.1).to(DEV)
        sh = torch.randn(c, generator=g).to(DEV) * 0.5
        return gm, torch.stack([gm * ist, sh, mu, ist])  # scale = gamma * invstd, as bn_finalize

    gm2, st2 = bn_consts()
    _, st1 = bn_consts()
    red2 = torch.randn((2, c), generator=g).to(DEV) * 50
    count = 1234.0
    dt1_ref = torch.empty_like(dz2)
    F.bn_relu_bwd_apply(t1, dz2, st2, gm2, red2, count, dt1_ref, False)
    y_ref = torch.empty_like(dz2)
    F.conv(dt1_ref, wp, y_ref, (1, 1, 1), (0, 0, 0))
    ref = F.bn_relu_bwd_reduce(R, y_ref, st1)
    outs = []
    for _ in range(2):
        dz = dz2.clone()
        dt1 = torch.empty_like(dz2)
        y = dz if alias else torch.empty_like(dz2)
        red = F.conv_reduce_bnb(t1, dz, st2, gm2, red2, count, dt1, wp, y, bnx=R, st=st1)
        assert red is not None
        assert torch.equal(dt1, dt1_ref)
        assert torch.equal(y, y_ref)
        outs.append(red)
    err = (outs[0] - ref).abs().max().item()
    assert err <= 1e-5 * (1 + ref.abs().max().item()), err
    assert torch.equal(outs[0], outs[1])
