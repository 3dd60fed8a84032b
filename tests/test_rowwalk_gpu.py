"""Edge cases of the row-walking HBM-bound kernels (BatchNorm statistics /
BN+ReLU backward in bn.hip, PReLU backward in drf.hip): ragged channel counts
(a partial last 16-byte chunk), channel slices and depth windows of a wider
buffer, and misaligned views that must take the scalar path.  Reference:
torch fp64 autograd on the CPU on the same dtype-rounded inputs (the oracle
for floating-point kernels).  Tolerances as in test_bn_duf_kernels_gpu /
test_drf_kernels_gpu: rel-L2 1e-4 (fp32) / 2e-2 (bf16) for BN, and
max|d| <= 2^-7 * (1 + max|ref|) for the bf16 PReLU data gradient."""
import pytest
import torch
import torch.nn.functional as Fn

from vsr_amd import functional as F

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _rel(a, b):
    return (a.double().cpu() - b.double().cpu()).norm().item() / max(b.double().norm().item(), 1e-30)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("c,extra,c_off,win", [(20, 12, 0, False), (36, 8, 8, True), (256, 0, 0, False)])
def test_bn_relu_backward_views(dtype, c, extra, c_off, win):
    g = torch.Generator().manual_seed(c)
    shp = (2, 5 if win else 3, 7, 19)
    big = torch.randn((*shp, c + extra), generator=g) * 1.3 + 0.2
    dzb = torch.randn((*shp, c + extra), generator=g)
    sl = (slice(None), slice(1, 4) if win else slice(None), slice(None), slice(None), slice(c_off, c_off + c))
    x, dz = big[sl], dzb[sl]
    gamma = torch.rand(c, generator=g) + 0.5
    beta = torch.randn(c, generator=g) * 0.5
    xq = x.to(dtype).double().requires_grad_(True)
    gm = gamma.double().requires_grad_(True)
    bt = beta.double().requires_grad_(True)
    y = Fn.batch_norm(xq.permute(0, 4, 1, 2, 3), None, None, gm, bt, training=True, eps=1e-5)
    torch.relu(y).backward(dz.to(dtype).double().permute(0, 4, 1, 2, 3))
    xd, dzd = big.to(DEV, dtype)[sl], dzb.to(DEV, dtype)[sl]
    cnt = xd[..., 0].numel()
    st = F.bn_finalize(F.bn_stats(xd), cnt, gamma.to(DEV), beta.to(DEV), 1e-5, 0.1)
    xs = x.to(dtype).double().reshape(-1, c)
    tol = 1e-4 if dtype == torch.float32 else 2e-2
    assert _rel(st[2], xs.mean(0)) <= 1e-5
    red = F.bn_relu_bwd_reduce(xd, dzd, st)
    assert _rel(red[1], gm.grad) <= tol and _rel(red[0], bt.grad) <= tol
    out = torch.zeros((*x.shape[:-1], c), dtype=dtype, device=DEV)
    F.bn_relu_bwd_apply(xd, dzd, st, gamma.to(DEV), red, cnt, out, accumulate=False)
    assert _rel(out, xq.grad) <= tol


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("c,c_off", [(12, 0), (64, 1), (40, 8), (256, 0)])
def test_prelu_backward_views(dtype, c, c_off):
    """c_off = 1 misaligns every view (scalar path); c = 12 leaves a partial chunk."""
    g = torch.Generator().manual_seed(100 + c + c_off)
    shp = (2, 1, 5, 37)
    a = 0.2
    W = c + c_off + 3
    x = torch.randn((*shp, c), generator=g)
    y = torch.where(x > 0, x, a * x).to(dtype)
    gy = torch.randn((*shp, c), generator=g).to(dtype)
    gy2 = torch.randn((*shp, c), generator=g).to(dtype)

    def place(t):
        buf = torch.zeros((*shp, W), dtype=dtype, device=DEV)
        buf[..., c_off:c_off + c] = t.to(DEV)
        return buf[..., c_off:c_off + c]

    dx = place(torch.zeros((*shp, c), dtype=dtype))
    da = torch.zeros(1, device=DEV)
    F.prelu_bwd(place(y), place(gy), torch.tensor([a], device=DEV), dx, da, accumulate_da=False, dy2=place(gy2))
    yd, gd = y.double(), gy.double() + gy2.double()
    refx = torch.where(yd > 0, gd, a * gd)
    tol = 2e-6 if dtype == torch.float32 else 2.0 ** -7
    assert (dx.double().cpu() - refx).abs().max().item() <= tol * (1 + refx.abs().max().item())
    refa = (torch.where(yd < 0, yd / a, torch.zeros_like(yd)) * gd).sum().item()
    assert abs(da.item() - refa) <= (1e-4 if dtype == torch.float32 else 3e-2) * max(abs(refa), 1.0)
