"""torch.ops.vsrk / vsr_amd.modules on the GPU against the fp64 torch
reference of the same layers (CPU), one op at a time and as whole reference
generators with swap_modules.

The ops compute in the input's dtype (fp32 here; one bf16 case): fp32 results
are held to 1e-4 relative L2 (outputs and every gradient), bf16 to 2e-2."""
import copy
import sys
from pathlib import Path

import pytest
import torch
import torch.nn as nn
import torch.nn.functional as Fn

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from oracle import cpu_nets  # noqa: E402

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)
TOL = 1e-4


def _rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def _flat(o):
    return torch.cat([t.flatten() for t in o]) if isinstance(o, (list, tuple)) else o


def _compare(ref_mod, inputs, tol=TOL):
    """Run ref_mod in fp64 on the CPU and a swapped fp32 copy on the GPU; same
    inputs, loss = <out, fixed random G>; compare outputs and all gradients."""
    from vsr_amd import modules
    ref = copy.deepcopy(ref_mod).double()
    hip = modules.swap_modules(copy.deepcopy(ref_mod)).to(DEV)
    n_hip = sum(type(m).__name__.startswith("Hip") for m in hip.modules())
    assert n_hip > 0

    def run(net, dev, dt):
        xs = [t.to(dev, dt).requires_grad_(True) for t in inputs]
        as_list = isinstance(ref_mod, cpu_nets.DUFRef) or type(ref_mod) is cpu_nets.DRFRef
        out = net(xs if as_list else xs[0])
        o = _flat(out)
        g = torch.Generator().manual_seed(11)
        G = torch.randn(o.shape, generator=g, dtype=torch.float64).to(dev, dt)
        (o * G).sum().backward()
        return o, [t.grad for t in xs], {k: p.grad for k, p in net.named_parameters()}

    o64, gx64, gp64 = run(ref, "cpu", torch.float64)
    o32, gx32, gp32 = run(hip, DEV, torch.float32)
    assert _rel(o32, o64) <= tol, ("out", _rel(o32, o64))
    for a, b in zip(gx32, gx64):
        if b is not None and b.norm() > 0:
            assert _rel(a, b) <= tol, ("grad_in", _rel(a, b))
    gmax = max(b.norm().item() for b in gp64.values())
    for k, b in gp64.items():
        assert gp32[k] is not None, k
        if b.norm().item() <= 1e-9 * gmax:
            # exact gradient 0 (a conv bias feeding a train-mode BatchNorm): fp32 noise only
            assert gp32[k].norm().item() <= 1e-5 * gmax, k
            continue
        assert _rel(gp32[k], b) <= tol, (k, _rel(gp32[k], b))
    return ref, hip


@pytest.mark.parametrize("mod,shape", [
    (lambda: nn.Conv2d(16, 32, 3, padding=1), (2, 16, 13, 17)),
    (lambda: nn.Conv2d(1, 16, 3, padding=1), (2, 1, 13, 17)),
    (lambda: nn.Conv2d(16, 1, 3, padding=1), (2, 16, 13, 17)),
    (lambda: nn.Conv2d(24, 16, 1), (2, 24, 13, 17)),
    (lambda: nn.Conv3d(32, 16, 3, padding=(1, 1, 1)), (2, 32, 5, 9, 11)),
    (lambda: nn.Conv3d(32, 16, 3, padding=(0, 1, 1)), (2, 32, 5, 9, 11)),
    (lambda: nn.Conv3d(32, 64, 1), (2, 32, 3, 9, 11)),
    (lambda: nn.Conv3d(64, 32, (1, 3, 3), padding=(0, 1, 1)), (1, 64, 1, 9, 11)),
    (lambda: nn.ConvTranspose2d(16, 16, 8, stride=4, padding=2), (2, 16, 6, 7)),
    (lambda: nn.ConvTranspose2d(16, 16, 6, stride=2, padding=2), (2, 16, 6, 7)),
    (lambda: nn.Conv2d(16, 16, 8, stride=4, padding=2), (2, 16, 24, 28)),
    (lambda: nn.Conv2d(16, 16, 6, stride=2, padding=2), (2, 16, 12, 14)),
])
def test_layer(mod, shape):
    torch.manual_seed(3)
    m = mod()
    g = torch.Generator().manual_seed(4)
    _compare(m, [torch.randn(shape, generator=g)])


def test_conv_relu_pixelshuffle_op():
    """vsrk::conv with a fused ReLU and a PixelShuffle(2) output view vs
    Conv2d -> ReLU -> PixelShuffle in fp64 (edsr_net.py:26-27 up-sampler order)."""
    torch.manual_seed(5)
    w = torch.randn(4 * 16, 16, 3, 3) * 0.1
    b = torch.randn(4 * 16) * 0.1
    x = torch.randn(2, 16, 9, 10)
    G = torch.randn(2, 16, 18, 20)
    ref = [t.double().requires_grad_(True) for t in (x, w, b)]
    (Fn.pixel_shuffle(torch.relu(Fn.conv2d(ref[0], ref[1], ref[2], padding=1)), 2) * G.double()).sum().backward()
    hip = [t.to(DEV).requires_grad_(True) for t in (x, w, b)]
    y = torch.ops.vsrk.conv(hip[0], hip[1], hip[2], [1, 1], "relu", 1, 2)
    (y * G.to(DEV)).sum().backward()
    yr = Fn.pixel_shuffle(torch.relu(Fn.conv2d(ref[0], ref[1], ref[2], padding=1)), 2)
    assert _rel(y, yr) <= TOL
    for a, r in zip(hip, ref):
        assert _rel(a.grad, r.grad) <= TOL


def test_conv_bf16():
    torch.manual_seed(6)
    m = nn.Conv2d(64, 64, 3, padding=1)
    x = torch.randn(2, 64, 16, 20)
    yr = m.double()(x.double())
    from vsr_amd import modules
    h = modules.swap_modules(nn.Sequential(copy.deepcopy(m).float())).to(DEV)
    y = h(x.to(DEV, torch.bfloat16))
    assert y.dtype == torch.bfloat16
    assert _rel(y.float(), yr) <= 2e-2


@pytest.mark.parametrize("train", [True, False])
def test_batch_norm(train):
    torch.manual_seed(7)
    bn = nn.BatchNorm3d(32)
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.5, 0.5)
        bn.running_mean.uniform_(-0.2, 0.2)
        bn.running_var.uniform_(0.5, 2.0)
    bn.train(train)
    g = torch.Generator().manual_seed(8)
    x = torch.randn((2, 32, 3, 9, 11), generator=g) * 2 + 0.5
    ref, hip = _compare(bn, [x])
    for k in ("running_mean", "running_var"):
        assert _rel(getattr(hip, k), getattr(ref, k)) <= TOL, k
    assert int(hip.num_batches_tracked) == int(ref.num_batches_tracked)


@pytest.mark.parametrize("kind,param,fn", [
    (0, 0.0, lambda o, t: Fn.l1_loss(o, t)),
    (1, 0.0, lambda o, t: Fn.mse_loss(o, t)),
    (2, 0.5, lambda o, t: Fn.smooth_l1_loss(o, t, beta=0.5) * 0.5),  # = Huber(delta 0.5), losses.py:5-20
    (3, 1e-3, lambda o, t: torch.sqrt((o - t) ** 2 + 1e-3).mean()),  # losses.py:23-34
])
def test_loss_op(kind, param, fn):
    g = torch.Generator().manual_seed(9)
    o, t = torch.randn(2, 1, 33, 41, generator=g), torch.randn(2, 1, 33, 41, generator=g)
    od = o.double().requires_grad_(True)
    lr = fn(od, t.double())
    lr.backward()
    oh = o.to(DEV).requires_grad_(True)
    lh = torch.ops.vsrk.loss(oh, t.to(DEV), kind, param)
    lh.backward()
    assert abs(lh.item() - lr.item()) <= 1e-5 * max(1.0, abs(lr.item()))
    assert _rel(oh.grad, od.grad) <= TOL


def test_metric_ops():
    g = torch.Generator().manual_seed(10)
    o, t = torch.randn(3, 1, 40, 44, generator=g), torch.randn(3, 1, 40, 44, generator=g) * 0.5
    mean, std = cpu_nets.DATASET_STATS["acdc"]
    od, td = cpu_nets.denormalize(o.double(), "acdc"), cpu_nets.denormalize(t.double(), "acdc")
    p = torch.ops.vsrk.psnr(o.to(DEV), t.to(DEV), mean, std, 255.0, True)
    assert _rel(p, cpu_nets.psnr(od, td, size_average=False)) <= 1e-5
    s = torch.ops.vsrk.ssim(o.to(DEV), t.to(DEV), mean, std, 255.0, True)
    assert _rel(s, cpu_nets.ssim(od, td, size_average=False)) <= 1e-4


def test_duf_dynfilter_op():
    """duf_net.py:67-97 (the DUFRef tail) vs vsrk::duf_dynfilter, fp64 reference."""
    k, r = 5, 4
    g = torch.Generator().manual_seed(12)
    x = torch.randn(2, 1, 9, 10, generator=g)
    lg = torch.randn(2, k * k * r * r, 9, 10, generator=g)
    res = torch.randn(2, r * r, 9, 10, generator=g)
    G = torch.randn(2, 1, 9 * r, 10 * r, generator=g)

    def ref_fn(x, lg, res):
        f = torch.softmax(lg.reshape(2, k * k, r * r, 9, 10), dim=1)
        eye = torch.eye(k * k, dtype=x.dtype).reshape(k * k, 1, k, k)
        pt = Fn.conv2d(x, eye, padding=k // 2).permute(0, 2, 3, 1).unsqueeze(-2)
        o = torch.matmul(pt, f.permute(0, 3, 4, 1, 2)).squeeze(-2).permute(0, 3, 1, 2)
        return Fn.pixel_shuffle(o, r) + Fn.pixel_shuffle(res, r)

    rd = [t.double().requires_grad_(True) for t in (lg, res)]
    yr = ref_fn(x.double(), *rd)
    (yr * G.double()).sum().backward()
    hd = [t.to(DEV).requires_grad_(True) for t in (lg, res)]
    y = torch.ops.vsrk.duf_dynfilter(x.to(DEV), hd[0], hd[1], k, r)
    (y * G.to(DEV)).sum().backward()
    assert _rel(y, yr) <= TOL
    for a, b in zip(hd, rd):
        assert _rel(a.grad, b.grad) <= TOL


@pytest.mark.parametrize("name", ["edsr", "duf", "drf", "drf_sisr"])
def test_reference_generator_swapped(name):
    """A reference generator (oracle restatement of src/model/nets/*.py, same
    module tree) with every conv / deconv / BN swapped runs forward + backward
    on the HIP ops and matches its own fp64 CPU run."""
    torch.manual_seed(13)
    g = torch.Generator().manual_seed(14)
    if name == "edsr":
        net, xs = cpu_nets.EDSRRef(1, 1, 2, 16, 4), [torch.randn(2, 1, 10, 12, generator=g)]
    elif name == "duf":
        net = cpu_nets.DUFRef(1, 1, 7, 5, 4, "_DenseLayer16").train()
        xs = [torch.randn(2, 1, 8, 9, generator=g) for _ in range(7)]
    elif name == "drf":
        net, xs = cpu_nets.DRFRef(1, 1, 16, 3, 4), [torch.randn(2, 1, 8, 10, generator=g) for _ in range(3)]
    else:
        net, xs = cpu_nets.DRFSISRRef(1, 1, 2, 16, 2, 2), [torch.randn(2, 1, 8, 10, generator=g)]
    _compare(net, xs)
