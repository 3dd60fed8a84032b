"""The persistent multi-tile conv loops -- the code path the bench times.

At full size every conv grid is one workgroup per CU and each workgroup walks
many tiles: the fast forward kernel's cross-tile DMA ring, the deferred
epilogue of the previous tile and the next-tile operand prefetch; the generic
and thin kernels' tile loops; the weight gradient's split of many tiles per
workgroup.  Small test shapes never get there (a few dozen tiles on 256
CUs), so here vsrk_conv_set_grid_cap forces the grid down to 1..7 workgroups
and the same shapes run 10-200 tiles per workgroup.

Checks: (1) forward / data-gradient outputs are bitwise identical for every
cap (each tile is computed independently of the grid) and match fp64 on the
CPU; (2) weight gradients match fp64 for every cap (the split changes, so the
fp32 sums re-associate) and are bitwise reproducible at a fixed cap.
Tolerances as tests/test_conv_kernels_gpu.py (bf16: inputs rounded to bf16
before the fp64 reference, max |d| <= 1.5e-2 max|ref|; fp32: 2e-5)."""
import pytest
import torch
import torch.nn.functional as Fn

from vsr_amd import functional as F

pytestmark = pytest.mark.gpu
DEV = "cuda"
CAPS = [0, 1, 3, 7]


@pytest.fixture(autouse=True)
def _reset_cap():
    yield
    F.set_grid_cap(0)


def _q(t, dtype):
    return t.to(dtype).double()


def _tol(dtype, ref):
    scale = ref.abs().max().item()
    return (2e-5 * (1 + scale)) if dtype == torch.float32 else 1.5e-2 * max(scale, 1e-3)


def _ref_conv(x_cl, w, b, pad):
    y = Fn.conv3d(x_cl.permute(0, 4, 1, 2, 3), w, b, padding=pad)
    return y.permute(0, 2, 3, 4, 1)


# (name, N, D, H, W, Cin, Cout, k, pad, epilogue) -- each >= 40 output tiles
FWD = [
    ("edsr_body_res", 3, 1, 40, 70, 64, 64, (1, 3, 3), (0, 1, 1), "res"),      # fast NT64: residual prefetch
    ("edsr_body_relu", 3, 1, 40, 70, 64, 64, (1, 3, 3), (0, 1, 1), "relu"),   # fast NT64: act, no prefetch
    ("dgrad_mask", 3, 1, 40, 70, 64, 64, (1, 3, 3), (0, 1, 1), "mask"),       # fast NT64: mask prefetch
    ("accumulate", 2, 1, 40, 70, 64, 64, (1, 3, 3), (0, 1, 1), "acc"),        # fast NT64: generic epilogue
    ("duf_3d_bn", 2, 5, 20, 40, 64, 32, (3, 3, 3), (1, 1, 1), "bn"),          # fast NT32: BN prologue, kd taps
    ("duf_3d_valid", 2, 5, 20, 40, 96, 32, (3, 3, 3), (0, 1, 1), "bn"),       # depth-valid
    ("pointwise_128", 2, 3, 20, 40, 128, 256, (1, 1, 1), (0, 0, 0), "bn"),    # fast k1 NT128
    ("pointwise_64", 2, 3, 20, 40, 64, 64, (1, 1, 1), (0, 0, 0), "relu"),     # fast k1 NT64
    ("head_thin", 3, 1, 40, 70, 1, 64, (1, 3, 3), (0, 1, 1), "none"),         # thin (cin = 1)
    ("tail_thin", 3, 1, 40, 70, 64, 1, (1, 3, 3), (0, 1, 1), "none"),         # thin (cout = 1)
]


def _fwd_case(case, dtype, cap, g_seed=0):
    name, n, d, h, w, ci, co, k, pad, epi = case
    g = torch.Generator().manual_seed(g_seed)
    cst = max(8, ci)  # 1-channel inputs live in 8-channel padded storage (as the nets hold them)
    xs = torch.randn((n, d, h, w, cst), generator=g)
    x = xs[..., :ci]
    wt = torch.randn((co, ci, *k), generator=g) / (ci * k[0] * k[1] * k[2]) ** 0.5
    b = torch.randn(co, generator=g)
    do = d + 2 * pad[0] - k[0] + 1
    other = torch.randn((n, do, h, w, co), generator=g)
    sc = torch.rand(ci, generator=g) + 0.5
    sh = torch.randn(ci, generator=g)
    # fp64 reference
    xin = _q(x, dtype)
    if epi == "bn":
        xin = torch.relu(xin * sc.double() + sh.double())
        xin = xin.to(dtype).double() if dtype != torch.float32 else xin
    ref = _ref_conv(xin, _q(wt, dtype), b.double(), pad)
    kw = {}
    if epi == "res":
        ref = ref * 0.1 + _q(other, dtype)
        kw = dict(out_scale=0.1, residual=other.to(DEV, dtype))
    elif epi == "relu":
        ref = torch.relu(ref)
        kw = dict(act=F.ACT_RELU)
    elif epi == "mask":
        ref = torch.where(_q(other, dtype) > 0, ref, torch.zeros_like(ref))
        kw = dict(mask=other.to(DEV, dtype))
    elif epi == "acc":
        ref = ref + _q(other, dtype)
    elif epi == "bn":
        kw = dict(prologue=F.PRO_AFFINE_RELU, pro_scale=sc.to(DEV), pro_shift=sh.to(DEV))
    ycs = co if co >= 8 or dtype == torch.float32 else 8
    ys = (other if epi == "acc" else torch.zeros((n, do, h, w, co)))
    yst = torch.zeros((n, do, h, w, ycs), dtype=dtype, device=DEV)
    yst[..., :co] = ys.to(DEV, dtype)
    y = yst[..., :co]
    F.set_grid_cap(cap)
    F.conv(xs.to(DEV, dtype)[..., :ci], F.pack_weight(wt.to(DEV), 0, dtype), y, k, pad, bias=b.to(DEV),
           accumulate=(epi == "acc"), **kw)
    torch.cuda.synchronize()
    return y.cpu(), ref


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("case", FWD, ids=[c[0] for c in FWD])
def test_multitile_forward(case, dtype):
    outs = []
    for cap in CAPS:
        y, ref = _fwd_case(case, dtype, cap)
        err = (y.double() - ref).abs().max().item()
        assert err <= _tol(dtype, ref), (case[0], cap, err)
        outs.append(y)
    for cap, y in zip(CAPS[1:], outs[1:]):
        assert torch.equal(y, outs[0]), (case[0], "grid cap changed the result", cap)


# sub-pixel views: conv -> PixelShuffle(2) store, and the data gradient reading
# the shuffled gradient (edsr_net.py:61-62)
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("which", ["y_shuffle", "x_shuffle"])
def test_multitile_subpixel(which, dtype):
    g = torch.Generator().manual_seed(5)
    n, h, w, f, r = 3, 30, 50, 64, 2
    if which == "y_shuffle":
        x = torch.randn((n, 1, h, w, f), generator=g)
        wt = torch.randn((f * r * r, f, 3, 3), generator=g) / 24
        b = torch.randn(f * r * r, generator=g)
        ref = Fn.pixel_shuffle(Fn.conv2d(_q(x, dtype)[:, 0].permute(0, 3, 1, 2), _q(wt, dtype), b.double(),
                                         padding=1), r).permute(0, 2, 3, 1)
    else:
        # dgrad of conv(f -> 4f) + PixelShuffle: x is the HR gradient read through a shuffle view
        x = torch.randn((n, 1, h * r, w * r, f), generator=g)
        wt = torch.randn((f * r * r, f, 3, 3), generator=g) / 24
        gy = Fn.pixel_unshuffle(_q(x, dtype)[:, 0].permute(0, 3, 1, 2), r)  # torch order c'*r*r + sub
        ref = Fn.conv_transpose2d(gy, _q(wt, dtype), padding=1).permute(0, 2, 3, 1)
    outs = []
    for cap in CAPS:
        F.set_grid_cap(cap)
        if which == "y_shuffle":
            y = torch.empty((n, 1, h * r, w * r, f), dtype=dtype, device=DEV)
            F.conv(x.to(DEV, dtype), F.pack_weight(wt.to(DEV), 0, dtype, perm_r=r), y, (1, 3, 3), (0, 1, 1),
                   bias=b.to(DEV), y_shuffle=r)
        else:
            y = torch.empty((n, 1, h, w, f), dtype=dtype, device=DEV)
            F.conv(x.to(DEV, dtype), F.pack_weight(wt.to(DEV), 1, dtype, perm_r=r), y, (1, 3, 3), (0, 1, 1),
                   x_shuffle=r)
        y = y[:, 0].cpu()
        err = (y.double() - ref).abs().max().item()
        assert err <= _tol(dtype, ref), (which, cap, err)
        outs.append(y)
    for y in outs[1:]:
        assert torch.equal(y, outs[0])


WG = [
    ("edsr_64", 3, 1, 40, 70, 64, 64, (1, 3, 3), (0, 1, 1), False),
    ("duf_3d_bn", 2, 5, 20, 40, 64, 32, (3, 3, 3), (1, 1, 1), True),
    ("duf_3d_valid", 2, 5, 20, 40, 96, 32, (3, 3, 3), (0, 1, 1), True),
    ("pointwise", 2, 3, 20, 40, 128, 256, (1, 1, 1), (0, 0, 0), True),
    ("head_thin", 3, 1, 40, 70, 1, 64, (1, 3, 3), (0, 1, 1), False),
]


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("case", WG, ids=[c[0] for c in WG])
def test_multitile_wgrad(case, dtype):
    name, n, d, h, w, ci, co, k, pad, bn = case
    g = torch.Generator().manual_seed(7)
    cst = max(8, ci)
    xs = torch.randn((n, d, h, w, cst), generator=g)
    x = xs[..., :ci]
    do = d + 2 * pad[0] - k[0] + 1
    gy = torch.randn((n, do, h, w, co), generator=g)
    sc = torch.rand(ci, generator=g) + 0.5
    sh = torch.randn(ci, generator=g)
    xin = _q(x, dtype)
    if bn:
        xin = torch.relu(xin * sc.double() + sh.double())
        xin = xin.to(dtype).double() if dtype != torch.float32 else xin
    wr = torch.zeros((co, ci, *k), dtype=torch.float64, requires_grad=True)
    br = torch.zeros(co, dtype=torch.float64, requires_grad=True)
    _ref_conv(xin, wr, br, pad).backward(_q(gy, dtype))
    kw = dict(prologue=F.PRO_AFFINE_RELU, pro_scale=sc.to(DEV), pro_shift=sh.to(DEV)) if bn else {}
    tw = (2e-5 if dtype == torch.float32 else 1e-2) * (1 + wr.grad.abs().max().item())
    tb = (2e-5 if dtype == torch.float32 else 1e-2) * (1 + br.grad.abs().max().item())
    for cap in CAPS:
        F.set_grid_cap(cap)
        res = []
        for _ in range(2):
            dw = torch.empty((co, ci, *k), dtype=torch.float32, device=DEV)
            db = torch.empty(co, dtype=torch.float32, device=DEV)
            F.conv_wgrad(xs.to(DEV, dtype)[..., :ci], gy.to(DEV, dtype), k, pad, dw, db, **kw)
            res.append((dw.cpu(), db.cpu()))
        assert torch.equal(res[0][0], res[1][0]) and torch.equal(res[0][1], res[1][1]), (name, cap, "not reproducible")
        ew = (res[0][0].double() - wr.grad).abs().max().item()
        eb = (res[0][1].double() - br.grad).abs().max().item()
        assert ew <= tw and eb <= tb, (name, cap, ew, tw, eb, tb)


PIPE = [
    ("duf_3d_bn", 2, 5, 20, 40, 64, 32, (3, 3, 3), (1, 1, 1), True, True),
    ("duf_3d_valid", 2, 5, 20, 40, 96, 32, (3, 3, 3), (0, 1, 1), True, True),
    ("edsr_64", 3, 1, 40, 70, 64, 64, (1, 3, 3), (0, 1, 1), False, True),
    ("ragged_ch", 2, 3, 13, 37, 40, 24, (3, 3, 3), (1, 1, 1), True, False),
    ("wide_in", 2, 4, 12, 50, 224, 32, (3, 3, 3), (0, 1, 1), True, True),
]


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("case", PIPE, ids=[c[0] for c in PIPE])
def test_wgrad_pipe_matches_generic(case, dtype):
    """The two-stage pipelined 3x3(x3) weight gradient (conv_wgrad_pipe.hip)
    runs the generic kernel's MFMA sequence on the same staged operands, so
    dW and dbias are bitwise equal to it, for every grid cap (several tiles
    per workgroup drive the ring), and within bf16/fp16 tolerance of fp64."""
    name, n, d, h, w, ci, co, k, pad, bn, bias = case
    g = torch.Generator().manual_seed(11)
    x = torch.randn((n, d, h, w, ci), generator=g)
    do = d + 2 * pad[0] - k[0] + 1
    gy = torch.randn((n, do, h, w, co), generator=g)
    sc = torch.rand(ci, generator=g) + 0.5
    sh = torch.randn(ci, generator=g)
    kw = dict(prologue=F.PRO_AFFINE_RELU, pro_scale=sc.to(DEV), pro_shift=sh.to(DEV)) if bn else {}
    xd, gd = x.to(DEV, dtype), gy.to(DEV, dtype)

    def run(pipe, cap):
        F.set_conv_path("wgrad_pipe", pipe)
        F.set_conv_path("wgrad_roll", 0)  # the rolling 3x3x3 kernel has its own tests (test_wgrad_roll_gpu.py)
        F.set_grid_cap(cap)
        try:
            dw = torch.empty((co, ci, *k), dtype=torch.float32, device=DEV)
            db = torch.empty(co, dtype=torch.float32, device=DEV) if bias else None
            F.conv_wgrad(xd, gd, k, pad, dw, db, **kw)
            return dw.cpu(), (db.cpu() if bias else None)
        finally:
            F.set_conv_path("wgrad_pipe", -1)
            F.set_conv_path("wgrad_roll", -1)
            F.set_grid_cap(0)

    xin = _q(x, dtype)
    if bn:
        xin = torch.relu(xin * sc.double() + sh.double()).to(dtype).double()
    wr = torch.zeros((co, ci, *k), dtype=torch.float64, requires_grad=True)
    br = torch.zeros(co, dtype=torch.float64, requires_grad=True)
    _ref_conv(xin, wr, br, pad).backward(_q(gy, dtype))
    for cap in (0, 3):
        pw, pb = run(1, cap)
        gw, gb = run(0, cap)
        assert torch.equal(pw, gw), (name, cap, (pw - gw).abs().max().item())
        if bias:
            assert torch.equal(pb, gb), (name, cap)
        assert (pw.double() - wr.grad).abs().max().item() <= 1e-2 * (1 + wr.grad.abs().max().item())
        if bias:
            assert (pb.double() - br.grad).abs().max().item() <= 1e-2 * (1 + br.grad.abs().max().item())


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("r,f,ci", [(2, 64, 64), (2, 16, 16), (3, 32, 64)])
def test_wgrad_pipe_subpixel_dy(dtype, r, f, ci):
    """Pipelined wgrad of an up-sampler conv whose output gradient is read
    through a sub-pixel view (edsr_net.py:55-64: conv -> PixelShuffle):
    bitwise equal to the generic kernel, and within bf16/fp16 tolerance of
    fp64 autograd through pixel_shuffle."""
    g = torch.Generator().manual_seed(13)
    n, h, w = 2, 18, 40
    co = f * r * r
    x = torch.randn((n, 1, h, w, ci), generator=g)
    gy = torch.randn((n, f, h * r, w * r), generator=g)
    xd = x.to(DEV, dtype)
    gy_cl = gy.permute(0, 2, 3, 1).unsqueeze(1).contiguous().to(DEV, dtype)

    def run(pipe, cap):
        F.set_conv_path("wgrad_pipe", pipe)
        F.set_grid_cap(cap)
        try:
            dw = torch.empty((co, ci, 1, 3, 3), device=DEV)
            db = torch.empty(co, device=DEV)
            F.conv_wgrad(xd, gy_cl, (1, 3, 3), (0, 1, 1), dw, db, perm_r=r, dy_shuffle=r)
            return dw.cpu(), db.cpu()
        finally:
            F.set_conv_path("wgrad_pipe", -1)
            F.set_grid_cap(0)

    wr = torch.zeros((co, ci, 3, 3), dtype=torch.float64, requires_grad=True)
    br = torch.zeros(co, dtype=torch.float64, requires_grad=True)
    y = Fn.pixel_shuffle(Fn.conv2d(_q(x, dtype)[:, 0].permute(0, 3, 1, 2), wr, br, padding=1), r)
    y.backward(_q(gy, dtype))
    for cap in (0, 5):
        pw, pb = run(1, cap)
        gw, gb = run(0, cap)
        assert torch.equal(pw, gw) and torch.equal(pb, gb), (r, f, cap, (pw - gw).abs().max().item())
        assert (pw[:, :, 0].double() - wr.grad).abs().max().item() <= 1e-2 * (1 + wr.grad.abs().max().item())
        assert (pb.double() - br.grad).abs().max().item() <= 1e-2 * (1 + br.grad.abs().max().item())
