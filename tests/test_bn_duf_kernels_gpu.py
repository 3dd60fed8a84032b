"""BatchNorm3d (+ReLU) statistics/backward kernels and the fused DUF dynamic
upsampling kernels against torch fp64 on the CPU (oracle for floating-point
kernels).  fp32 kernels: rel err <= 1e-5 (reductions) / 1e-4 (outputs);
bf16 inputs: the fp64 reference sees the same bf16-rounded values."""
import numpy as np
import pytest
import torch
import torch.nn.functional as Fn

from vsr_amd import functional as F

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _rel(a, b):
    return (a.double().cpu() - b.double().cpu()).norm().item() / max(b.double().norm().item(), 1e-30)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("c", [32, 64, 200])
def test_bn_stats_depth(dtype, c):
    """Per-depth statistics of a depth window / channel slice of a concat
    buffer (the DUF bn1 cache) vs fp64, and their sum vs the one-pass stats."""
    g = torch.Generator().manual_seed(7 + c)
    big = torch.randn((3, 7, 11, 37, c + 40), generator=g) * 1.5 + 0.3
    xd = big.to(DEV, dtype)[:, 1:6, :, :, 16:16 + c]
    xq = big.to(dtype).double()[:, 1:6, :, :, 16:16 + c]
    sd = F.bn_stats_depth(xd)
    assert sd.shape == (5, 2, c)
    ref1 = xq.sum(dim=(0, 2, 3))
    ref2 = (xq * xq).sum(dim=(0, 2, 3))
    assert _rel(sd[:, 0], ref1) <= 1e-5 and _rel(sd[:, 1], ref2) <= 1e-5
    whole = F.bn_stats(xd)
    assert _rel(sd.double().sum(0), whole) <= 1e-5


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("c", [32, 160, 224])
def test_bn_forward_stats_and_running(dtype, c):
    g = torch.Generator().manual_seed(c)
    big = torch.randn((2, 5, 9, 13, c + 32), generator=g) * 2 + 0.7
    x = big[:, 1:4, :, :, :c]  # depth window + channel slice of a concat buffer
    gamma = torch.rand(c, generator=g) + 0.5
    beta = torch.randn(c, generator=g)
    rm, rv = torch.randn(c, generator=g), torch.rand(c, generator=g) + 0.5
    xd = big.to(DEV, dtype)[:, 1:4, :, :, :c]
    sums = F.bn_stats(xd)
    cnt = x.shape[0] * x.shape[1] * x.shape[2] * x.shape[3]
    rmd, rvd = rm.to(DEV).clone(), rv.to(DEV).clone()
    st = F.bn_finalize(sums, cnt, gamma.to(DEV), beta.to(DEV), 1e-5, 0.1, rmd, rvd)
    xq = x.to(dtype).double().reshape(-1, c)
    mean, var = xq.mean(0), xq.var(0, unbiased=False)
    invstd = 1 / torch.sqrt(var + 1e-5)
    assert _rel(st[2], mean) <= 1e-5 and _rel(st[3], invstd) <= 1e-5
    assert _rel(st[0], gamma.double() * invstd) <= 1e-5
    assert _rel(st[1], beta.double() - mean * gamma.double() * invstd) <= 1e-5
    assert _rel(rmd, 0.9 * rm.double() + 0.1 * mean) <= 1e-5
    assert _rel(rvd, 0.9 * rv.double() + 0.1 * xq.var(0, unbiased=True)) <= 1e-5


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16])
def test_bn_relu_backward(dtype):
    """dx of relu(batchnorm(x)) given dz; dgamma, dbeta; accumulate into a concat slice."""
    g = torch.Generator().manual_seed(9)
    c = 96
    x = torch.randn((2, 3, 8, 11, c), generator=g) * 1.5 + 0.3
    dz = torch.randn((2, 3, 8, 11, c), generator=g)
    gamma = torch.rand(c, generator=g) + 0.5
    beta = torch.randn(c, generator=g) * 0.5
    xq = x.to(dtype).double().requires_grad_(True)
    gm = gamma.double().requires_grad_(True)
    bt = beta.double().requires_grad_(True)
    y = Fn.batch_norm(xq.permute(0, 4, 1, 2, 3), None, None, gm, bt, training=True, eps=1e-5)
    torch.relu(y).backward(dz.to(dtype).double().permute(0, 4, 1, 2, 3))
    xd, dzd = x.to(DEV, dtype), dz.to(DEV, dtype)
    st = F.bn_finalize(F.bn_stats(xd), xd[..., 0].numel(), gamma.to(DEV), beta.to(DEV), 1e-5, 0.1)
    red = F.bn_relu_bwd_reduce(xd, dzd, st)
    base = torch.randn((2, 3, 8, 11, c + 16), generator=g)
    out = base.to(DEV, dtype)
    F.bn_relu_bwd_apply(xd, dzd, st, gamma.to(DEV), red, xd[..., 0].numel(), out[..., 16:], accumulate=True)
    tol = {torch.float32: 1e-4, torch.float16: 4e-3}.get(dtype, 2e-2)
    assert _rel(red[1], gm.grad) <= tol and _rel(red[0], bt.grad) <= tol
    exp = base[..., 16:].to(dtype).double() + xq.grad
    assert _rel(out[..., 16:], exp) <= tol
    assert torch.equal(out[..., :16].cpu(), base[..., :16].to(dtype))  # untouched


def _duf_ref(x, logits, res, k, r):
    """duf_net.py:67-97 restated in fp64: softmax over taps, unfold, contract, shuffle."""
    n, h, w = x.shape
    f = logits.view(n, h, w, k * k, r * r).softmax(3)
    eye = torch.tensor(np.eye(k * k), dtype=x.dtype).view(k * k, 1, k, k)
    p = Fn.conv2d(x.unsqueeze(1), eye, padding=k // 2).permute(0, 2, 3, 1)  # (n,h,w,kk)
    o = torch.einsum("nhwt,nhwts->nshw", p, f)
    return Fn.pixel_shuffle(o, r) + Fn.pixel_shuffle(res.permute(0, 3, 1, 2), r)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16])
def test_duf_dynfilter(dtype):
    g = torch.Generator().manual_seed(5)
    n, h, w, k, r = 2, 9, 13, 5, 4
    x = torch.randn((n, h, w), generator=g)
    lg = torch.randn((n, h, w, k * k * r * r), generator=g) * 2
    res = torch.randn((n, h, w, r * r), generator=g)
    gout = torch.randn((n, 1, h * r, w * r), generator=g)
    x64, lg64, res64 = x.double(), lg.double().requires_grad_(True), res.double().requires_grad_(True)
    out64 = _duf_ref(x64, lg64, res64, k, r)
    out64.backward(gout.double())
    out = F.duf_dynfilter_fwd(x.to(DEV), lg.to(DEV), res.to(DEV), k, r)
    assert _rel(out, out64) <= 1e-5
    dl, dr = F.duf_dynfilter_bwd(x.to(DEV), lg.to(DEV), gout.to(DEV), k, r, dtype)
    tol = {torch.float32: 1e-5, torch.float16: 2e-3}.get(dtype, 8e-3)
    assert _rel(dl, lg64.grad) <= tol and _rel(dr, res64.grad) <= tol


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("ncontrib,cb", [(1, 32), (2, 32), (3, 32), (4, 32), (6, 32), (7, 64), (8, 20)])
def test_bn_apply_multi_equals_sequential_applies(dtype, ncontrib, cb):
    """vsrk_bn_relu_bwd_apply_multi (DUF's deferred bn1 input gradients) vs
    the single-contributor apply run once per contributor: every
    contributor's dz covers its own depth window of the block.  More than
    three contributors take the one-pass LDS-constant form (DUF's head block
    has 7, its first unit blocks 4-6); cb = 20: a partial 16-byte chunk (bf16)."""
    g = torch.Generator().manual_seed(11 + ncontrib)
    n, D, h, w, c = 2, 7, 5, 9, cb + 32
    buf = (torch.randn((n, D, h, w, c + 16), generator=g) * 1.3 + 0.2).to(DEV, dtype)
    x = buf[..., 16:16 + cb]  # the block: a channel slice of a concat buffer
    base = (torch.randn((n, D, h, w, cb), generator=g) * 0.1).to(DEV, dtype)
    cs, seq = [], base.clone()
    for i in range(ncontrib):
        d0, d1 = [(0, 7), (1, 6), (2, 5), (0, 7), (3, 4), (1, 6), (0, 7), (2, 5)][i]
        dz = torch.randn((n, d1 - d0, h, w, c), generator=g).to(DEV, dtype)[..., 8:8 + cb]
        sc = (torch.rand(cb, generator=g) + 0.3).to(DEV)
        sh = torch.randn(cb, generator=g).to(DEV)
        mean, invstd = torch.randn(cb, generator=g).to(DEV), (torch.rand(cb, generator=g) + 0.5).to(DEV)
        st = torch.stack([sc, sh, mean, invstd])
        gamma = (torch.rand(cb, generator=g) + 0.5).to(DEV)
        red = torch.randn((2, cb), generator=g).to(DEV)
        cnt = float(n * (d1 - d0) * h * w)
        cs.append((dz, d0, st, gamma, red, cnt))
        F.bn_relu_bwd_apply(x[:, d0:d1], dz, st, gamma, red, cnt, seq[:, d0:d1], True)
    out = base.clone()
    F.bn_relu_bwd_apply_multi(x, out, True, cs)
    tol = 1e-5 if dtype == torch.float32 else 2e-2
    assert (out.float() - seq.float()).abs().max().item() <= tol * max(1.0, seq.float().abs().max().item())
