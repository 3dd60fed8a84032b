"""TEST INFRASTRUCTURE ONLY — golden vectors for the k-space Downscale.

Run in the build container (needs /root/reference):
    python -m oracle.make_downscale_golden

Loads acdc_preprocess.py by path and runs the reference's own `Downscale`
(acdc_preprocess.py:102-180) on seeded images.  OpenCV and nibabel are not
installed here: `cv2` is a stand-in module whose `resize` is the OpenCV
INTER_CUBIC restatement of oracle/downscale.py (so the resize step itself is
parity unpinned), `nibabel` an empty module (unused by Downscale).  Asserts
the reference's pipeline equals oracle.downscale.downscale bit for bit and
writes tests/golden/downscale.pt (inputs and LR outputs, float64).  The
images go in as float64, so the FFTs run in complex128 as under the
reference's pinned numpy 1.16 (env.yml:112).
"""
from __future__ import annotations

import importlib.util
import os
import sys
import types
from pathlib import Path

import numpy as np
import torch

from . import downscale as D
from .ref_loader import REF

OUT = Path(__file__).resolve().parent.parent / "tests" / "golden" / "downscale.pt"

# (H, W, r): even / odd k-space rectangles, non-square, r = 2, 3, 4
CASES = [(64, 64, 4), (48, 40, 4), (30, 33, 3), (36, 20, 2), (128, 96, 4)]


def _load_reference():
    sys.dont_write_bytecode = True
    cv2 = types.ModuleType("cv2")
    cv2.INTER_CUBIC = 2

    def resize(img, dsize, interpolation):
        assert interpolation == cv2.INTER_CUBIC
        return D.resize_cubic(img, dsize[0], dsize[1])

    cv2.resize = resize
    sys.modules.setdefault("cv2", cv2)
    sys.modules.setdefault("nibabel", types.ModuleType("nibabel"))
    spec = importlib.util.spec_from_file_location("acdc_preprocess", os.path.join(REF, "src", "acdc_preprocess.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def _image(h, w, rng):
    """A smooth, MRI-like 8-bit image: blurred noise plus a bright disc."""
    z = rng.standard_normal((h + 4, w + 4))
    k = np.ones(5) / 5.0
    z = np.apply_along_axis(lambda v: np.convolve(v, k, "valid"), 0, z)
    z = np.apply_along_axis(lambda v: np.convolve(v, k, "valid"), 1, z) * 5.0
    yy, xx = np.mgrid[:h, :w]
    disc = ((yy - h / 2) ** 2 + (xx - w / 2) ** 2 < (min(h, w) / 4) ** 2) * 120.0
    return np.clip(np.round(50 + 40 * z + disc), 0, 255).astype(np.float32)[..., None]


def main():
    ref = _load_reference()
    rng = np.random.default_rng(2024)
    fx = {"cases": []}
    for h, w, r in CASES:
        img = _image(h, w, rng)
        # float64 in: numpy 1.16 (env.yml:112) runs the FFTs in complex128 for
        # any real input, numpy 2 would drop to complex64 for float32 images.
        (want,) = ref.Downscale(r)(img.astype(np.float64))
        got = D.downscale(img, r)
        assert want.shape == (h // r, w // r, 1), want.shape
        assert np.array_equal(want, got), (h, w, r)
        trunc = D.kspace_truncate(img, r)
        fx["cases"].append({"r": r, "hr": torch.from_numpy(img.astype(np.float64)),
                            "kspace_truncated": torch.from_numpy(trunc), "lr": torch.from_numpy(want)})
        print(f"downscale {h}x{w} /{r}: lr mean {want.mean():.3f}, range [{want.min()}, {want.max()}]")
    torch.save(fx, OUT)
    print(f"wrote {OUT}")


if __name__ == "__main__":
    main()
