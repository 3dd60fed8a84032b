"""torch.ops.vsrk registry, fake (meta) shapes and swap_modules on the
reference generators' module trees -- no kernel launches (CPU container)."""
import copy
import sys
from pathlib import Path

import pytest
import torch
import torch.nn as nn

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from oracle import cpu_nets  # noqa: E402
from vsr_amd import modules, ops  # noqa: E402,F401

META = torch.device("meta")


def test_registry():
    names = {"conv", "conv_backward", "subpixel_weight", "batch_norm_stats", "batch_norm",
             "batch_norm_backward", "duf_dynfilter", "loss", "psnr", "ssim"}
    for n in names:
        assert hasattr(torch.ops.vsrk, n), n


@pytest.mark.parametrize("xs,ws,pad,xsh,ysh,exp", [
    ((2, 16, 9, 11), (64, 16, 3, 3), [1, 1], 1, 2, (2, 16, 18, 22)),
    ((2, 16, 9, 11), (8, 16, 1, 1), [0, 0], 1, 1, (2, 8, 9, 11)),
    ((2, 64, 7, 9, 11), (32, 64, 3, 3, 3), [0, 1, 1], 1, 1, (2, 32, 5, 9, 11)),
    ((2, 64, 7, 9, 11), (32, 64, 3, 3, 3), [1, 1, 1], 1, 1, (2, 32, 7, 9, 11)),
    ((1, 8, 32, 48), (8, 128, 3, 3), [1, 1], 4, 1, (1, 8, 8, 12)),
])
def test_conv_fake_shapes(xs, ws, pad, xsh, ysh, exp):
    x, w = torch.empty(xs, device=META), torch.empty(ws, device=META)
    y = torch.ops.vsrk.conv(x, w, torch.empty(ws[0], device=META), pad, "relu", xsh, ysh)
    assert tuple(y.shape) == exp
    g = torch.ops.vsrk.conv_backward(y, x, w, y, pad, "relu", xsh, ysh, False, True)
    assert [tuple(t.shape) for t in g] == [xs, ws, (ws[0],)]


@pytest.mark.parametrize("r", [2, 4, 8])
def test_subpixel_weight_fake_shapes(r):
    k, s, p = cpu_nets._PROJ[r]
    w = torch.empty((16, 16, k, k), device=META)
    weq, beq = torch.ops.vsrk.subpixel_weight(w, torch.empty(16, device=META), k, s, p, True)
    assert tuple(weq.shape) == (s * s * 16, 16, 3, 3) and tuple(beq.shape) == (s * s * 16,)
    weq, beq = torch.ops.vsrk.subpixel_weight(w, None, k, s, p, False)
    assert tuple(weq.shape) == (16, s * s * 16, 3, 3) and tuple(beq.shape) == (16,)


def test_batch_norm_fake_shapes():
    x = torch.empty((2, 64, 7, 9, 11), device=META)
    rm, rv = torch.empty(64, device=META), torch.empty(64, device=META)
    st = torch.ops.vsrk.batch_norm_stats(x, None, None, rm, rv, True, 0.1, 1e-5)
    assert tuple(st.shape) == (4, 64)
    assert torch.ops.vsrk.batch_norm(x, None, None, st, True, True).shape == x.shape


def _swapped_types(net):
    return sorted({type(m).__name__ for m in net.modules()})


@pytest.mark.parametrize("name,make,expect", [
    ("edsr", lambda: cpu_nets.EDSRRef(1, 1, 2, 16, 4), {"HipConv2d"}),
    ("duf", lambda: cpu_nets.DUFRef(1, 1, 7, 5, 4, "_DenseLayer16"), {"HipConv2d", "HipConv3d", "HipBatchNorm3d"}),
    ("drf", lambda: cpu_nets.DRFRef(1, 1, 16, 3, 4), {"HipConv2d", "HipConvTranspose2d"}),
])
def test_swap_modules_reference_trees(name, make, expect):
    torch.manual_seed(0)
    net = make()
    before = {k: v for k, v in net.state_dict().items()}
    n_before = sum(isinstance(m, (nn.Conv2d, nn.Conv3d, nn.ConvTranspose2d, nn.BatchNorm3d)) for m in net.modules())
    modules.swap_modules(net)
    hip = [m for m in net.modules() if type(m).__name__.startswith("Hip")]
    assert len(hip) == n_before  # every conv / deconv / BN of these generators is supported
    assert {type(m).__name__ for m in hip} == expect
    after = net.state_dict()
    assert list(after) == list(before)
    for k in before:
        assert after[k].data_ptr() == before[k].data_ptr(), k  # the same tensors, not copies
    # the swapped modules are still the torch classes they replace
    assert all(isinstance(m, (nn.Conv2d, nn.Conv3d, nn.ConvTranspose2d, nn.BatchNorm3d)) for m in hip)


def test_swap_leaves_unsupported_layers():
    net = nn.Sequential(nn.Conv2d(8, 8, 5, padding=2), nn.Conv2d(8, 8, 3, padding=2, dilation=2),
                        nn.Conv2d(8, 8, 3, groups=2, padding=1), nn.ConvTranspose2d(8, 8, 3, 1, 1),
                        nn.BatchNorm2d(8))
    ref = copy.deepcopy(net)
    modules.swap_modules(net)
    assert [type(m) for m in net] == [type(m) for m in ref]


def test_ops_refuse_cpu_tensors():
    """No CPU fallback: the ops launch HIP kernels or raise."""
    x = torch.randn(1, 8, 4, 4)
    w = torch.randn(8, 8, 3, 3)
    with pytest.raises(Exception):
        torch.ops.vsrk.conv(x, w, None, [1, 1], "none", 1, 1)
