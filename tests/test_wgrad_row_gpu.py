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
