"""k-space LR synthesis on the GPU: the mirror of `Downscale`
(acdc_preprocess.py:102-180).

Per image: centred FFT (``fftshift(fftn(ifftshift(img), norm='ortho'))``),
keep the centred (H // r) x (W // r) rectangle of k-space, inverse FFT,
``around(abs(.))``, then OpenCV's INTER_CUBIC resize to (H // r, W // r) and
``clip(round(.), 0, 255)``.  The FFTs are torch.fft (rocFFT) in complex128 on
the device; the truncation is a slice fill; the resize + round + clip is the
HIP kernel ``vsrk_resize_bicubic`` (fp64, OpenCV's float coordinate and
weight arithmetic).  Images are single-channel (the reference's fftn over an
(H, W, 1) array is the 2-D transform).
"""
from __future__ import annotations

import numpy as np
import torch

from .. import _native as N


def resize_bicubic(src: torch.Tensor, out_h: int, out_w: int, round_clip: bool = False) -> torch.Tensor:
    """cv2.resize(INTER_CUBIC) of (N, H, W) float64 device images -> (N, out_h, out_w)."""
    if src.dtype != torch.float64 or src.dim() != 3 or not src.is_cuda:
        raise ValueError("resize_bicubic expects a (N, H, W) float64 CUDA tensor")
    lib = N.load()
    s = src.contiguous()
    dst = torch.empty((s.shape[0], out_h, out_w), dtype=torch.float64, device=s.device)
    N.check(lib.vsrk_resize_bicubic(s.data_ptr(), s.shape[0], s.shape[1], s.shape[2], out_h, out_w, dst.data_ptr(),
                                    int(round_clip), N.stream_ptr(s.device)), "resize_bicubic")
    return dst


def kspace_truncate(img: torch.Tensor, r: int) -> torch.Tensor:
    """(N, H, W) real device images -> around(abs(band-limited image)), float64
    (acdc_preprocess.py:141-180)."""
    dims = (-2, -1)
    k = torch.fft.fftshift(torch.fft.fftn(torch.fft.ifftshift(img.to(torch.complex128), dim=dims), dim=dims,
                                          norm="ortho"), dim=dims)
    h, w = k.shape[-2:]
    kx, ky, lx, ly = h // 2, w // 2, h // r, w // r
    band = torch.zeros_like(k)
    sl = (Ellipsis, slice(kx - lx // 2, kx + (lx - lx // 2)), slice(ky - ly // 2, ky + (ly - ly // 2)))
    band[sl] = k[sl]
    out = torch.fft.fftshift(torch.fft.ifftn(torch.fft.ifftshift(band, dim=dims), dim=dims, norm="ortho"), dim=dims)
    return torch.round(out.abs())


def downscale_tensor(hr: torch.Tensor, r: int) -> torch.Tensor:
    """(N, H, W) HR images on the device -> (N, H // r, W // r) LR images, float64."""
    t = kspace_truncate(hr, r)
    return resize_bicubic(t, t.shape[-2] // r, t.shape[-1] // r, round_clip=True)


class Downscale:
    """acdc_preprocess.py:102-139: ``Downscale(r)(*imgs)`` maps numpy (H, W, 1)
    images to their (H // r, W // r, 1) LR images (float64), on ``device``."""

    def __init__(self, downscale_factor: int, device: str | torch.device = "cuda"):
        self.downscale_factor = downscale_factor
        self.device = torch.device(device)

    def __call__(self, *imgs):
        if not all(isinstance(img, np.ndarray) for img in imgs):
            raise TypeError('All of the images should be numpy.ndarray.')
        if not all(img.ndim == 3 for img in imgs):
            raise ValueError("All of the images' dimensions should be 3 (2D images).")
        if not all(img.shape[2] == 1 for img in imgs):
            raise ValueError("Downscale handles single-channel (H, W, 1) images.")
        out = []
        for img in imgs:
            x = torch.from_numpy(np.ascontiguousarray(img[..., 0], dtype=np.float64)).to(self.device)[None]
            out.append(downscale_tensor(x, self.downscale_factor)[0, ..., None].cpu().numpy())
        return tuple(out)


__all__ = ["Downscale", "downscale_tensor", "kspace_truncate", "resize_bicubic"]
