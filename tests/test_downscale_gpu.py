"""vsrk_resize_bicubic and the device Downscale (torch.fft + the HIP resize)
against the reference's Downscale outputs (tests/golden/downscale.pt).  The
resize is bit-exact given the same input; the whole pipeline is compared
exactly too (the FFTs differ from numpy's only in the last bits, far from
the .5 rounding ties of integer-valued images), and the numpy front end keeps
the reference's type checks."""
import numpy as np
import pytest
import torch

from oracle import downscale as D
from tests.conftest import load_golden
from vsr_amd.data import Downscale, downscale_tensor
from vsr_amd.data.downscale import resize_bicubic

pytestmark = pytest.mark.gpu
DEV = "cuda"


def test_resize_kernel_bit_exact():
    fx = load_golden("downscale")
    for c in fx["cases"]:
        t = c["kspace_truncated"][..., 0]
        h, w = t.shape
        r = c["r"]
        got = resize_bicubic(t[None].to(DEV), h // r, w // r, round_clip=False)[0].cpu().numpy()
        np.testing.assert_array_equal(got, D.resize_cubic(t.numpy(), w // r, h // r))
        got = resize_bicubic(t[None].to(DEV), h // r, w // r, round_clip=True)[0].cpu().numpy()
        np.testing.assert_array_equal(got, c["lr"][..., 0].numpy())


def test_resize_kernel_upscale_and_ragged():
    rng = np.random.default_rng(1)
    img = rng.random((3, 13, 17)) * 255
    got = resize_bicubic(torch.from_numpy(img).to(DEV), 29, 11).cpu().numpy()
    want = np.stack([D.resize_cubic(i, 11, 29) for i in img])
    np.testing.assert_array_equal(got, want)


def test_device_downscale_matches_reference():
    fx = load_golden("downscale")
    for c in fx["cases"]:
        hr = c["hr"].numpy().astype(np.float32)
        (got,) = Downscale(c["r"])(hr)
        assert got.shape == c["lr"].shape
        np.testing.assert_array_equal(got, c["lr"].numpy())
    c = fx["cases"][0]
    batch = torch.stack([c["hr"][..., 0]] * 3).to(DEV)
    got = downscale_tensor(batch, c["r"]).cpu()
    assert torch.equal(got, c["lr"][..., 0].expand(3, -1, -1))


def test_downscale_type_checks():
    with pytest.raises(TypeError):
        Downscale(4)(torch.zeros(8, 8, 1))
    with pytest.raises(ValueError):
        Downscale(4)(np.zeros((8, 8)))
