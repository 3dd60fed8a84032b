"""The DCN oracle (oracle/dcn_ref.py, a restatement of
deform_conv_cuda_kernel.cu) on the CPU: zero offsets and unit masks give
nn.functional.conv2d; integer offsets shift the sampling grid exactly;
positions at or beyond -1 / H read as zero.  (The reference's CUDA extension
cannot be built here: parity of DCN is pinned to its source, not to its
outputs.)"""
import pytest
import torch
import torch.nn.functional as Fn

from oracle.dcn_ref import modulated_deform_conv_ref


@pytest.mark.parametrize("stride,padding,dilation,dg", [(1, 1, 1, 1), (2, 1, 1, 2), (1, 2, 2, 4)])
def test_zero_offset_is_conv2d(stride, padding, dilation, dg):
    g = torch.Generator().manual_seed(0)
    x = torch.randn((2, 8, 9, 11), generator=g, dtype=torch.float64)
    wt = torch.randn((5, 8, 3, 3), generator=g, dtype=torch.float64)
    b = torch.randn(5, generator=g, dtype=torch.float64)
    ref = Fn.conv2d(x, wt, b, stride, padding, dilation)
    ho, wo = ref.shape[2:]
    off = torch.zeros((2, dg * 18, ho, wo), dtype=torch.float64)
    m = torch.ones((2, dg * 9, ho, wo), dtype=torch.float64)
    out = modulated_deform_conv_ref(x, off, m, wt, b, stride, padding, dilation, dg)
    assert torch.allclose(out, ref, atol=1e-12)


def test_integer_offset_shifts_and_border():
    x = torch.arange(1.0, 1 + 6 * 7, dtype=torch.float64).view(1, 1, 6, 7)
    wt = torch.zeros((1, 1, 1, 1), dtype=torch.float64)
    wt[0, 0, 0, 0] = 1.0
    off = torch.zeros((1, 2, 6, 7), dtype=torch.float64)
    off[0, 0] = 1.0  # every sample one row down
    out = modulated_deform_conv_ref(x, off, None, wt)
    assert torch.equal(out[0, 0, :5], x[0, 0, 1:])
    assert torch.equal(out[0, 0, 5], torch.zeros(7, dtype=torch.float64))  # row 6 == H: outside
    off[0, 0] = -0.5  # half a row up: row 0 blends with the zero row above (h = -0.5 > -1)
    out = modulated_deform_conv_ref(x, off, None, wt)
    assert torch.allclose(out[0, 0, 0], 0.5 * x[0, 0, 0])
