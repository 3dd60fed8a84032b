"""The CPU restatement of Downscale (oracle/downscale.py) against the golden
vectors that the reference's own Downscale produced (tests/golden/downscale.pt,
oracle/make_downscale_golden.py; the cv2 resize step inside it is the
restatement itself, so that step is parity unpinned), plus properties of the
OpenCV INTER_CUBIC restatement."""
import numpy as np
import pytest

from oracle import downscale as D
from tests.conftest import load_golden


def test_oracle_matches_reference_vectors():
    fx = load_golden("downscale")
    assert len(fx["cases"]) >= 5
    for c in fx["cases"]:
        hr = c["hr"].numpy().astype(np.float32)
        np.testing.assert_array_equal(D.kspace_truncate(hr, c["r"]), c["kspace_truncated"].numpy())
        np.testing.assert_array_equal(D.downscale(hr, c["r"]), c["lr"].numpy())


def test_resize_constant_and_identity():
    img = np.full((12, 20), 37.0)
    np.testing.assert_allclose(D.resize_cubic(img, 5, 3), 37.0, rtol=0, atol=1e-12)
    rng = np.random.default_rng(0)
    img = rng.random((9, 7))
    np.testing.assert_array_equal(D.resize_cubic(img, 7, 9), img)  # scale 1: weights (0, 1, 0, 0)


def test_resize_rejects_multichannel():
    with pytest.raises(ValueError):
        D.resize_cubic(np.zeros((4, 4, 3)), 2, 2)
