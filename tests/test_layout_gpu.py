"""Layout moves at the network edges (NCDHW fp32 <-> channels-last views):
`functional.to_view` / `from_view` are exact copies (bf16 rounding only), so
they are compared bit-exactly against torch's permute + cast.  Covers the
dense fast path (zero-padded 8-channel storage of the 1-channel LR input and
HR gradient, 2D and 3D) and the generic strided path (a channel slice)."""
import pytest
import torch

from vsr_amd import functional as F

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("shape,cpad", [((3, 1, 37, 29), 8), ((2, 1, 5, 17, 9), 8), ((2, 3, 11, 13), 8),
                                        ((2, 16, 9, 7), None), ((1, 5, 3, 6, 10), 8)])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_to_view_dense(shape, cpad, dtype):
    g = torch.Generator().manual_seed(7)
    x = torch.randn(shape, generator=g)
    v = F.to_view(x.to(DEV), dtype, cpad)
    xc = x if x.dim() == 5 else x.unsqueeze(2)
    ref = xc.permute(0, 2, 3, 4, 1).to(dtype)
    c = x.shape[1]
    assert v.shape[-1] == (cpad or c)
    assert torch.equal(v[..., :c].cpu(), ref)
    if cpad and cpad > c:
        assert not v[..., c:].any()  # padding channels are zero
    back = F.from_view(v, c, two_d=x.dim() == 4)
    assert torch.equal(back.cpu(), ref.float().permute(0, 4, 1, 2, 3).reshape(x.shape))


def test_to_view_generic_slice():
    """A channel slice of a wider buffer is not dense: the generic kernel writes
    only its own channels."""
    import ctypes as C

    from vsr_amd import _native as N
    g = torch.Generator().manual_seed(3)
    x = torch.randn((2, 4, 1, 9, 11), generator=g)
    buf = torch.full((2, 1, 9, 11, 16), 7.0, device=DEV)
    view = buf[..., 4:8]
    tv = N.t5(view)
    lib = N.load()
    N.check(lib.vsrk_ncdhw_to_view(x.to(DEV).data_ptr(), 2, 4, 1, 9, 11, C.byref(tv), N.stream_ptr(torch.device(DEV))),
            "ncdhw_to_view")
    out = buf.cpu()
    assert torch.equal(out[..., 4:8], x.permute(0, 2, 3, 4, 1))
    assert (out[..., :4] == 7).all() and (out[..., 8:] == 7).all()
