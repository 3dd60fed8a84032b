"""TEST INFRASTRUCTURE ONLY — CPU restatement of the reference's LR synthesis.

`Downscale` (acdc_preprocess.py:102-180): per 2-D image (H, W, C)
  1. kspace = fftshift(fftn(ifftshift(img), norm='ortho'))          (:141-150)
  2. keep the centred lx x ly rectangle, lx = H // r, ly = W // r     (:152-170)
  3. img = around(abs(fftshift(ifftn(ifftshift(k), norm='ortho'))))  (:172-180)
  4. cv2.resize(img, (W // r, H // r), INTER_CUBIC)[..., None]        (:131)
  5. np.clip(img.round(), 0, 255)                                     (:132)

Steps 1-3 and 5 are the reference's own numpy calls.  Step 4 restates
OpenCV's resize for float64 input with INTER_CUBIC (OpenCV is not installed
here: this step is **parity unpinned** against cv2 itself): for output index
d the source coordinate is fx = float32((d + 0.5) * scale - 0.5) with
scale = 1 / (dst / src) in double, sx = floor(fx), the Keys cubic weights
(A = -0.75) of fx - sx evaluated in float32, source indices clamped to the
image (border replicate), a horizontal pass per source row and then the
vertical pass, each a left-to-right sum of double products.

`oracle/make_downscale_golden.py` runs the reference's own Downscale (loaded
by path, with this resize standing in for the absent cv2 module) and asserts
it equals `downscale` bit for bit, which pins steps 1-3 and 5.
"""
from __future__ import annotations

import numpy as np
from numpy.fft import fftn, fftshift, ifftn, ifftshift


def _cubic_weights(x: np.ndarray) -> np.ndarray:
    """(n,) float32 fractions -> (n, 4) float32 weights, OpenCV interpolateCubic."""
    x = x.astype(np.float32)
    A, one = np.float32(-0.75), np.float32(1)
    w0 = ((A * (x + one) - np.float32(5) * A) * (x + one) + np.float32(8) * A) * (x + one) - np.float32(4) * A
    w1 = ((A + np.float32(2)) * x - (A + np.float32(3))) * x * x + one
    w2 = ((A + np.float32(2)) * (one - x) - (A + np.float32(3))) * (one - x) * (one - x) + one
    w3 = one - w0 - w1 - w2
    return np.stack([w0, w1, w2, w3], axis=1).astype(np.float32)


def _axis_taps(n_src: int, n_dst: int):
    scale = 1.0 / (n_dst / n_src)
    f = ((np.arange(n_dst, dtype=np.float64) + 0.5) * scale - 0.5).astype(np.float32)
    s = np.floor(f).astype(np.int64)
    w = _cubic_weights(f - s.astype(np.float32))
    idx = np.clip(s[:, None] + np.arange(-1, 3)[None, :], 0, n_src - 1)
    return idx, w.astype(np.float64)


def resize_cubic(img: np.ndarray, out_w: int, out_h: int) -> np.ndarray:
    """cv2.resize(img, (out_w, out_h), interpolation=INTER_CUBIC) for a 2-D
    float64 image (or (H, W, 1), returned as 2-D like OpenCV does)."""
    if img.ndim == 3:
        if img.shape[2] != 1:
            raise ValueError("resize_cubic restates single-channel images only")
        img = img[..., 0]
    img = np.asarray(img, dtype=np.float64)
    ih, iw = img.shape
    yi, wy = _axis_taps(ih, out_h)
    xi, wx = _axis_taps(iw, out_w)
    # horizontal pass: rows[r, d] = sum_k S[r, xi[d, k]] * wx[d, k], left to right
    g = img[:, xi]  # (ih, out_w, 4)
    rows = ((g[..., 0] * wx[:, 0] + g[..., 1] * wx[:, 1]) + g[..., 2] * wx[:, 2]) + g[..., 3] * wx[:, 3]
    v = rows[yi]  # (out_h, 4, out_w)
    out = ((v[:, 0] * wy[:, 0:1] + v[:, 1] * wy[:, 1:2]) + v[:, 2] * wy[:, 2:3]) + v[:, 3] * wy[:, 3:4]
    return out


def kspace_truncate(img: np.ndarray, r: int) -> np.ndarray:
    """Steps 1-3: the image band-limited to the centred 1/r of k-space."""
    # numpy 1.16 (env.yml:112, the reference's pin) transforms in complex128
    # whatever the input precision; numpy >= 2 keeps float32 as complex64.
    k = fftshift(fftn(ifftshift(np.asarray(img, dtype=np.float64)), norm="ortho"))
    rect = np.zeros_like(k)
    kx, ky = k.shape[0] // 2, k.shape[1] // 2
    lx, ly = k.shape[0] // r, k.shape[1] // r
    rect[kx - lx // 2: kx + (lx - lx // 2), ky - ly // 2: ky + (ly - ly // 2)] = 1
    out = fftshift(ifftn(ifftshift(rect * k), norm="ortho"))
    return np.around(np.abs(out))


def downscale(img: np.ndarray, r: int) -> np.ndarray:
    """One (H, W, 1) image -> its (H // r, W // r, 1) LR image."""
    t = kspace_truncate(img, r)
    h, w, _ = t.shape
    out = resize_cubic(t, w // r, h // r)[..., np.newaxis]
    return np.clip(out.round(), 0, 255)
