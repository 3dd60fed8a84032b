"""DCNv2 / DCNv1 on HIP (vsr_amd.dcn: vsrk_dcn_im2col + MFMA 1x1 conv +
vsrk_dcn_col2im / vsrk_dcn_coord_grad) against the fp64 torch restatement of
deform_conv_cuda_kernel.cu (oracle/dcn_ref.py), forward and every gradient.
fp32 tolerances: output max |d| <= 1e-4 * max|ref|, gradients rel-L2 <= 1e-4
(the input gradient's float atomics change only the summation order).
Offsets are drawn so that samples fall off the image and straddle the -1 / H
borders, and no sample lies within 1e-3 of a grid line (where the
interpolation's derivative jumps)."""
import pytest
import torch

from oracle.dcn_ref import modulated_deform_conv_ref
from vsr_amd import dcn

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return ((a.double().cpu() - b.double()).norm() / b.double().norm().clamp_min(1e-30)).item()


def _offsets(g, n, dg, K, ho, wo, scale):
    off = torch.randn((n, dg * 2 * K, ho, wo), generator=g, dtype=torch.float64) * scale
    frac = off - off.floor()
    bad = (frac < 1e-3) | (frac > 1 - 1e-3)
    return torch.where(bad, off + 0.01, off)


@pytest.mark.parametrize("n,c,h,w,co,k,stride,pad,dil,dg,modulated", [
    (2, 16, 12, 13, 24, 3, 1, 1, 1, 1, True),
    (1, 32, 9, 10, 16, 3, 1, 1, 1, 4, True),   # EDVR-like: deformable groups
    (2, 8, 11, 9, 8, 3, 2, 1, 1, 2, True),     # strided
    (1, 16, 10, 10, 8, 3, 1, 2, 2, 1, True),   # dilated
    (2, 16, 12, 12, 16, 3, 1, 1, 1, 2, False),  # DCNv1 (deform_conv)
])
def test_dcn_forward_backward(n, c, h, w, co, k, stride, pad, dil, dg, modulated):
    g = torch.Generator().manual_seed(n * 1000 + c + dg)
    x = torch.randn((n, c, h, w), generator=g, dtype=torch.float64)
    wt = torch.randn((co, c, k, k), generator=g, dtype=torch.float64) * 0.2
    b = torch.randn(co, generator=g, dtype=torch.float64) if modulated else None
    ho = (h + 2 * pad - (dil * (k - 1) + 1)) // stride + 1
    wo = (w + 2 * pad - (dil * (k - 1) + 1)) // stride + 1
    off = _offsets(g, n, dg, k * k, ho, wo, 2.5)
    m = torch.rand((n, dg * k * k, ho, wo), generator=g, dtype=torch.float64) if modulated else None
    gy = torch.randn((n, co, ho, wo), generator=g, dtype=torch.float64)

    leaves = [t.clone().requires_grad_(True) for t in (x, off, wt)]
    mr = m.clone().requires_grad_(True) if modulated else None
    br = b.clone().requires_grad_(True) if modulated else None
    ref = modulated_deform_conv_ref(leaves[0], leaves[1], mr, leaves[2], br, stride, pad, dil, dg)
    ref.backward(gy)

    dev = [t.float().cuda().requires_grad_(True) for t in (x, off, wt)]
    md = m.float().cuda().requires_grad_(True) if modulated else None
    bd = b.float().cuda().requires_grad_(True) if modulated else None
    if modulated:
        out = dcn.modulated_deform_conv(dev[0], dev[1], md, dev[2], bd, stride, pad, dil, 1, dg)
    else:
        out = dcn.deform_conv(dev[0], dev[1], dev[2], stride, pad, dil, 1, dg)
    out.backward(gy.float().cuda())
    torch.cuda.synchronize()
    assert (out.double().cpu() - ref.detach()).abs().max().item() <= 1e-4 * ref.abs().max().item()
    for d, r, name in zip(dev, leaves, ("x", "offset", "weight")):
        assert _rel(d.grad, r.grad) <= 1e-4, name
    if modulated:
        assert _rel(md.grad, mr.grad) <= 1e-4
        assert _rel(bd.grad, br.grad) <= 1e-4


def test_pack_modules_zero_init_equal_plain_conv():
    """DCNv2Pack starts as a plain conv (zero offsets, sigmoid(0) = 0.5 masks)."""
    torch.manual_seed(0)
    m = dcn.ModulatedDeformConvPack(16, 8, 3, padding=1, deformable_groups=2).cuda()
    x = torch.randn((2, 16, 10, 12), device="cuda")
    y = m(x)
    ref = torch.nn.functional.conv2d(x.double().cpu(), m.weight.double().cpu(), m.bias.double().cpu(), 1, 1) * 1.0
    ref = 0.5 * (ref - m.bias.double().cpu().view(1, -1, 1, 1)) + m.bias.double().cpu().view(1, -1, 1, 1)
    assert (y.double().cpu() - ref).abs().max().item() < 1e-4
    assert set(n for n, _ in m.named_parameters()) == {"weight", "bias", "conv_offset_mask.weight",
                                                        "conv_offset_mask.bias"}
    v1 = dcn.DeformConvPack(16, 8, 3, padding=1).cuda()
    assert torch.allclose(v1(x).double().cpu(), torch.nn.functional.conv2d(x.double().cpu(), v1.weight.double().cpu(),
                                                                           None, 1, 1), atol=1e-4)
