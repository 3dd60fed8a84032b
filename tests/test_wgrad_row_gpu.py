"""The rolling-row Conv2d 3x3 weight gradient (conv_wgrad_row.hip): the
autograd of EDSR's body convs nn.Conv2d(64, 64, 3, padding=1).weight / .bias
(edsr_net.py:41-53) on channels-last views.

Against an fp32 torch reference of the same bf16 / fp16 operands
(torch.nn.grad.conv2d_weight; bias = sum of dy): the kernel multiplies the
16-bit values exactly and sums in fp32 in another order, so the weight
gradient agrees to fp32 summation noise (max |d| <= 1e-4 of the largest
entry) and equals the pipelined kernel it replaces (path "wgrad_row" off)
within the same bound.  Shapes cover: one 128-column segment and two (W =
150), W below a k-chunk multiple, bands of one row up to the whole image (grid
caps), several 64-channel chunks on both sides, 2 depths per sample, channel
slices of wider buffers, dy_scale and accumulation.
"""
import pytest
import torch

from vsr_amd import functional as F

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(autouse=True)
def _row_path():
    F.set_conv_path("wgrad_row", 1)
    yield
    F.set_conv_path("wgrad_row", -1)
    F.set_grid_cap(0)


def _ref(x, dy, scale):
    """fp32 torch weight / bias gradient of a 3x3 pad-1 conv on (N, D, H, W, C) views."""
    n, d, h, w, ci = x.shape
    co = dy.shape[-1]
    xn = x.float().reshape(n * d, h, w, ci).permute(0, 3, 1, 2)
    gn = dy.float().reshape(n * d, h, w, co).permute(0, 3, 1, 2)
    with torch.backends.cudnn.flags(enabled=False):
        torch.backends.cuda.matmul.allow_tf32 = False
        dw = torch.nn.grad.conv2d_weight(xn.double(), (co, ci, 3, 3), gn.double(), padding=1).float()
    db = gn.double().sum((0, 2, 3)).float()
    return dw.view(co, ci, 1, 3, 3) * scale, db * scale


CASES = [
    # (n, d, h, w, ci, co, grid_cap, x channel offset in a wider buffer)
    (2, 1, 19, 45, 64, 64, 0, 0),
    (1, 1, 40, 128, 64, 64, 1, 0),      # one band of 40 rows
    (3, 1, 9, 150, 64, 64, 0, 64),      # two column segments, x a channel slice
    (1, 2, 13, 31, 128, 192, 0, 0),     # 2 x 3 channel chunks, two depths per sample
    (2, 1, 33, 128, 64, 128, 5, 32),    # uneven bands
    (1, 1, 1, 7, 64, 64, 0, 0),         # one row, one partial k-chunk
]


@pytest.mark.parametrize("case", CASES)
@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
def test_wgrad_row_matches_fp32(case, dt):
    n, d, h, w, ci, co, cap, off = case
    g = torch.Generator().manual_seed(n * 1000 + h * 10 + w + ci)
    big = torch.randn((n, d, h, w, ci + off + 16), generator=g).to(DEV, dt)
    x = big[..., off:off + ci]
    dy = (torch.randn((n, d, h, w, co), generator=g) * 0.5).to(DEV, dt)
    F.set_grid_cap(cap)
    dw = torch.empty((co, ci, 1, 3, 3), device=DEV)
    db = torch.empty(co, device=DEV)
    F.conv_wgrad(x, dy, (1, 3, 3), (0, 1, 1), dw, db)
    rw, rb = _ref(x, dy, 1.0)
    tol = 1e-4 * rw.abs().max().item()
    assert (dw - rw).abs().max().item() <= tol, (dw - rw).abs().max().item()
    assert (db - rb).abs().max().item() <= 1e-4 * rb.abs().max().item() + 1e-4
    # the pipelined kernel it replaces
    F.set_conv_path("wgrad_row", 0)
    dw0 = torch.empty_like(dw)
    db0 = torch.empty_like(db)
    F.conv_wgrad(x, dy, (1, 3, 3), (0, 1, 1), dw0, db0)
    assert (dw - dw0).abs().max().item() <= tol
    # deterministic
    F.set_conv_path("wgrad_row", 1)
    dw2 = torch.empty_like(dw)
    F.conv_wgrad(x, dy, (1, 3, 3), (0, 1, 1), dw2, None)
    assert torch.equal(dw, dw2)


def test_wgrad_row_scale_and_accumulate():
    """EDSR's conv2 gradient carries res_scale (edsr_net.py:51): dw += s * dL/dW."""
    n, d, h, w, ci, co = 2, 1, 24, 64, 64, 64
    g = torch.Generator().manual_seed(11)
    x = torch.randn((n, d, h, w, ci), generator=g).to(DEV, torch.bfloat16)
    dy = torch.randn((n, d, h, w, co), generator=g).to(DEV, torch.bfloat16)
    base_w = torch.randn((co, ci, 1, 3, 3), generator=g).to(DEV)
    base_b = torch.randn(co, generator=g).to(DEV)
    dw, db = base_w.clone(), base_b.clone()
    F.conv_wgrad(x, dy, (1, 3, 3), (0, 1, 1), dw, db, dy_scale=0.1, accumulate=True)
    rw, rb = _ref(x, dy, 0.1)
    assert (dw - base_w - rw).abs().max().item() <= 1e-4 * rw.abs().max().item() + 1e-5
    assert (db - base_b - rb).abs().max().item() <= 1e-4 * rb.abs().max().item() + 1e-5


def test_wgrad_row_edsr_layer_size():
    """The bench's EDSR body layer (64 slices of 128 x 128, 64 -> 64): against
    the pipelined kernel (the fp32 reference of 2^20 voxels is slow on CPU-less
    paths; both kernels are checked against fp32 above)."""
    g = torch.Generator().manual_seed(5)
    x = torch.randn((64, 1, 128, 128, 64), generator=g).to(DEV, torch.bfloat16)
    dy = torch.randn((64, 1, 128, 128, 64), generator=g).to(DEV, torch.bfloat16)
    dw = torch.empty((64, 64, 1, 3, 3), device=DEV)
    db = torch.empty(64, device=DEV)
    F.conv_wgrad(x, dy, (1, 3, 3), (0, 1, 1), dw, db)
    F.set_conv_path("wgrad_row", 0)
    dw0, db0 = torch.empty_like(dw), torch.empty_like(db)
    F.conv_wgrad(x, dy, (1, 3, 3), (0, 1, 1), dw0, db0)
    assert (dw - dw0).abs().max().item() <= 1e-4 * dw0.abs().max().item()
    assert (db - db0).abs().max().item() <= 1e-4 * db0.abs().max().item()


# ---- sub-pixel views ----
PROJ = {2: (6, 2, 2), 3: (7, 3, 2), 4: (8, 4, 2), 8: (12, 8, 2)}


def _cl(t):  # (N,C,H,W) -> (N,1,H,W,C)
    return t.permute(0, 2, 3, 1).unsqueeze(1).contiguous()


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("ci", [64, 128])
def test_wgrad_row_edsr_upsampler(dt, ci):
    """EDSR's Upsampler conv (edsr_net.py:15-30, nn.Conv2d(f, 4f, 3) then
    PixelShuffle(2)): its output gradient is read straight from the high-res
    gradient through a shuffle-2 view, the 4f logical channels permuted by
    perm_r=2.  Equal to the pipelined kernel within fp32 summation noise, and
    to the fp64 gradient of conv2d + pixel_shuffle."""
    n, h, w, r = 2, 11, 37, 2
    co = ci * r * r
    g = torch.Generator().manual_seed(ci + 3)
    x = torch.randn((n, 1, h, w, ci), generator=g).to(DEV, dt)
    gy_hr = torch.randn((n, 1, h * r, w * r, ci), generator=g).to(DEV, dt)
    dw = torch.empty((co, ci, 1, 3, 3), device=DEV)
    db = torch.empty(co, device=DEV)
    F.conv_wgrad(x, gy_hr, (1, 3, 3), (0, 1, 1), dw, db, perm_r=r, dy_shuffle=r)
    # fp64: PixelShuffle's channel order c * r^2 + i * r + j
    xn = x.double().cpu()[:, 0].permute(0, 3, 1, 2).requires_grad_(True)
    wr = torch.zeros((co, ci, 3, 3), dtype=torch.float64, requires_grad=True)
    br = torch.zeros(co, dtype=torch.float64, requires_grad=True)
    yo = torch.nn.functional.pixel_shuffle(torch.nn.functional.conv2d(xn, wr, br, padding=1), r)
    yo.backward(gy_hr.double().cpu()[:, 0].permute(0, 3, 1, 2))
    rw = wr.grad.view(co, ci, 1, 3, 3)
    tol = 1e-4 * rw.abs().max().item()
    assert (dw.double().cpu() - rw).abs().max().item() <= tol
    assert (db.double().cpu() - br.grad).abs().max().item() <= 1e-4 * br.grad.abs().max().item()
    F.set_conv_path("wgrad_row", 0)
    dw0, db0 = torch.empty_like(dw), torch.empty_like(db)
    F.conv_wgrad(x, gy_hr, (1, 3, 3), (0, 1, 1), dw0, db0, perm_r=r, dy_shuffle=r)
    assert (dw - dw0).abs().max().item() <= tol
    assert (db - db0).abs().max().item() <= 1e-4 * db0.abs().max().item()


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("r", [2, 3, 4, 8])
@pytest.mark.parametrize("skip", [False, True])
def test_wgrad_row_drf_projections(dt, r, skip):
    """DRF's feedback-block projections (drf_net.py:70-102) at f = 64: the
    ConvTranspose2d(k, s, p) weight gradient with dy a shuffle-s view of the
    high-res gradient, the strided Conv2d's with x a shuffle-s view of the
    high-res input.  With the sub-pixel code passed (a form the router keeps on
    the pipelined kernel unless forced), each phase's zero taps are skipped and
    come out exactly zero, like the pipelined kernel's.  Folded to
    the k x k weights against fp64 autograd; unfolded against the pipelined
    kernel."""
    k, s, p = PROJ[r]
    f = 64
    n, h, w = 2, 7, 23 if r < 8 else 9
    H, W = h * s, w * s
    g = torch.Generator().manual_seed(r * 7 + skip)
    x_lr = torch.randn((n, f, h, w), generator=g)
    x_hr = torch.randn((n, f, H, W), generator=g)
    gy_hr = torch.randn((n, f, H, W), generator=g)
    gy_lr = torch.randn((n, f, h, w), generator=g)
    K3, P1 = (1, 3, 3), (0, 1, 1)
    for tr in (True, False):
        code = F.subpixel_code(k, s, p, tr, False) if skip else 0
        wk = torch.zeros((f, f, k, k), dtype=torch.float64, requires_grad=True)
        bk = torch.zeros(f, dtype=torch.float64, requires_grad=True)
        if tr:
            xin, gin = _cl(x_lr).to(DEV, dt), _cl(gy_hr).to(DEV, dt)
            kw = dict(dy_shuffle=s)
            torch.nn.functional.conv_transpose2d(xin.double().cpu()[:, 0].permute(0, 3, 1, 2), wk, bk, stride=s,
                                                 padding=p).backward(gin.double().cpu()[:, 0].permute(0, 3, 1, 2))
        else:
            xin, gin = _cl(x_hr).to(DEV, dt), _cl(gy_lr).to(DEV, dt)
            kw = dict(x_shuffle=s)
            torch.nn.functional.conv2d(xin.double().cpu()[:, 0].permute(0, 3, 1, 2), wk, bk, stride=s,
                                       padding=p).backward(gin.double().cpu()[:, 0].permute(0, 3, 1, 2))
        weq, beq = F.subpixel_conv_weight(torch.zeros((f, f, k, k), device=DEV), torch.zeros(f, device=DEV),
                                          k, s, p, transposed=tr)
        res = []
        for row in (2, 0):  # 2: the tap-skip forms are forced onto the row kernel
            F.set_conv_path("wgrad_row", row)
            dweq, dbeq = torch.empty_like(weq), torch.empty_like(beq)
            F.conv_wgrad(xin, gin, K3, P1, dweq.view(*weq.shape[:2], 1, 3, 3), dbeq, subpixel=code, **kw)
            res.append((dweq, dbeq))
        F.set_conv_path("wgrad_row", 1)
        (dweq, dbeq), (dweq0, dbeq0) = res
        tol = 1e-4 * dweq0.abs().max().item()
        if skip:  # the skipped taps: exact zeros on both paths
            assert torch.equal(dweq == 0, dweq0 == 0), tr
        assert (dweq - dweq0).abs().max().item() <= tol, tr
        assert (dbeq - dbeq0).abs().max().item() <= 1e-4 * dbeq0.abs().max().item(), tr
        dw = torch.empty((f, f, k, k), device=DEV)
        db = torch.empty(f, device=DEV)
        F.subpixel_wgrad_fold(dweq, dbeq, dw, db, k, s, p, transposed=tr)
        assert (dw.double().cpu() - wk.grad).abs().max().item() <= 1e-4 * wk.grad.abs().max().item(), tr
        assert (db.double().cpu() - bk.grad).abs().max().item() <= 1e-4 * bk.grad.abs().max().item(), tr
