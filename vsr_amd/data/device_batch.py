"""Training batches assembled on the GPU from HBM-resident cine volumes.

The reference assembles every sample on CPU DataLoader workers: read the
NIfTI volume, cut the temporal window, crop / flip with numpy, normalise,
collate, copy to the device (acdc_*_dataset.py, transforms.py,
base_trainer.py:120-124).  With 288 GB of HBM a whole preprocessed dataset
fits on one GPU, so here the normalised volumes stay resident and a batch
is one ``vsrk_gather_windows`` launch per side (LR, HR): the host only
replays the augment draws (vsr_amd.data.transforms.plan_augments, the same
Python ``random`` calls in the same order as the CPU pipeline) into 24-byte
index maps.  The result equals the CPU pipeline's batch bit for bit
(tests/test_device_batch_gpu.py).

Normalize commutes with the gathers (a per-image affine of the values), so it
is applied to the volumes once, before they are made resident.
"""
from __future__ import annotations

import torch

from .. import _native as N
from .datasets import _window
from .transforms import Compose, Normalize, ToTensor, compose, plan_augments


def _normalize(v: torch.Tensor, mean: float, std: float) -> torch.Tensor:
    """(v - mean) / (std + 1e-10) with the reference's float32 rounding
    (transforms.py:164-168 on float32 images: numpy casts both Python scalars
    to float32, subtracts, then divides correctly rounded).  A device kernel
    dividing by a Python scalar multiplies by its reciprocal instead (1 ulp
    apart on some values), so the quotient is taken in float64 -- exact
    division of two float32 values, then one rounding to float32, which is the
    correctly rounded float32 quotient."""
    dev = v.device
    m = torch.tensor(mean, dtype=torch.float32, device=dev)
    s = torch.tensor(std + 1e-10, dtype=torch.float32, device=dev).double()
    return ((v.float() - m).double() / s).float()


class DeviceCineBatcher:
    """Batches of (volume, target frame) items for one task.

    lr: (V, T, h, w) and hr: (V, T, H, W) fp32 device tensors (normalised, or
    raw with `normalize` given as (mean, std) to apply here once).
    task: 'sisr' (frame t alone), 'misr' (n-frame window around t, target the
    window's centre frame; acdc_misr_dataset.py) or 'vsr' (n-frame window,
    n targets; acdc_vsr_dataset.py).  augments: the dataset's augment list
    (Compose, list of transforms or config dicts), applied per sample.
    Returns the reference's batch dict: 'lr_img'/'hr_img' (B,1,.,.) for SISR,
    'lr_imgs' (n x (B,1,h,w)) + 'hr_img' for MISR, 'lr_imgs' + 'hr_imgs' for VSR.
    """

    def __init__(self, lr: torch.Tensor, hr: torch.Tensor, task: str, num_frames: int = 5,
                 temporal_order: str | None = None, augments=None, normalize=None):
        if task not in ("sisr", "misr", "vsr"):
            raise ValueError(f"task {task!r}")
        if lr.dim() != 4 or hr.dim() != 4 or lr.shape[:2] != hr.shape[:2]:
            raise ValueError("lr (V,T,h,w) and hr (V,T,H,W) volumes of the same V, T expected")
        if not lr.is_cuda or not hr.is_cuda:
            raise RuntimeError("DeviceCineBatcher keeps the volumes in device memory (no CPU fallback)")
        if normalize is not None:
            lr, hr = _normalize(lr, *normalize), _normalize(hr, *normalize)
        self.lr = lr.float().contiguous()
        self.hr = hr.float().contiguous()
        self.task = task
        self.n = 1 if task == "sisr" else num_frames
        self.order = temporal_order or ("middle" if task == "misr" else "last")
        if augments is not None and not isinstance(augments, Compose):
            augments = compose(augments) if augments and isinstance(augments[0], dict) else Compose(list(augments))
        self.augments = augments
        for t in (augments.transforms if augments is not None else []):
            if isinstance(t, (Normalize, ToTensor)):
                raise ValueError("value transforms belong to the resident volumes, not to the per-sample augments")

    def _gather(self, src: torch.Tensor, maps: list, frames: int, oh: int, ow: int) -> torch.Tensor:
        lib = N.load()
        V, T, h, w = src.shape
        for vol, t0, y0, dy, x0, dx in maps:  # every source index inside its volume
            ys = (y0, y0 + dy * (oh - 1))
            xs = (x0, x0 + dx * (ow - 1))
            if not (0 <= vol < V and 0 <= min(ys) and max(ys) < h and 0 <= min(xs) and max(xs) < w):
                raise ValueError(f"index map {(vol, t0, y0, dy, x0, dx)} leaves the ({V},{T},{h},{w}) volumes")
        m = torch.tensor(maps, dtype=torch.int32).to(src.device, non_blocking=True)
        out = torch.empty((len(maps), frames, oh, ow), dtype=torch.float32, device=src.device)
        N.check(lib.vsrk_gather_windows(src.data_ptr(), V, T, h, w, m.data_ptr(), len(maps), frames, oh, ow,
                                        out.data_ptr(), N.stream_ptr(src.device)), "gather_windows")
        return out

    def __call__(self, items) -> dict:
        """items: list of (volume index, target frame)."""
        V, T, h, w = self.lr.shape
        H, W = self.hr.shape[2:]
        lmaps, hmaps, size = [], [], None
        c = self.n // 2 if self.n % 2 == 1 else self.n // 2 - 1
        for vol, t in items:
            s = t if self.task == "sisr" else _window(t, self.n, T, self.order)[0]
            lm, hm = plan_augments(self.augments, (h, w), (H, W))
            if size is None:
                size = (lm.h, lm.w, hm.h, hm.w)
            elif size != (lm.h, lm.w, hm.h, hm.w):
                raise ValueError("every sample of a batch must have the same output size")
            lmaps.append([vol, s, lm.y0, lm.dy, lm.x0, lm.dx])
            hmaps.append([vol, s + (c if self.task == "misr" else 0), hm.y0, hm.dy, hm.x0, hm.dx])
        oh, ow, OH, OW = size
        lr = self._gather(self.lr, lmaps, self.n, oh, ow)
        hr = self._gather(self.hr, hmaps, 1 if self.task == "misr" else self.n, OH, OW)
        if self.task == "sisr":
            return {"lr_img": lr, "hr_img": hr}
        lr_list = [lr[:, k:k + 1] for k in range(self.n)]
        if self.task == "misr":
            return {"lr_imgs": lr_list, "hr_img": hr}
        return {"lr_imgs": lr_list, "hr_imgs": [hr[:, k:k + 1] for k in range(self.n)]}
