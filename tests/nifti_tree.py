"""A small NIfTI tree in the reference's on-disk layout (acdc_preprocess.py:55-85),
shared by the config and predictor tests."""
from pathlib import Path

import numpy as np

from vsr_amd.data import nifti


def make_tree(root: Path, T=30, H=32, W=32, patients=2, seed=0):
    """acdc_preprocess.py:55-85 layout: imgs/{split}/{HR,LR/X{r}}/<patient>/<patient>_2d_slice01_frameNN.nii.gz
    and videos/{split}/.../<patient>_2d+1d_sequence01.nii.gz (1-based ids), r = 2 and 4, T = 30 (DSB15 keeps
    sequences of >= 30 frames, dsb15_preprocess.py:28)."""
    rng = np.random.default_rng(seed)
    for split in ("train", "valid", "test"):
        for i in range(patients):
            pid = f"patient{i:03d}"
            hr = rng.integers(0, 255, (H, W, 1, T)).astype(np.float32)
            vols = [(hr, "HR")]
            for r in (2, 4):
                vols.append((hr.reshape(H // r, r, W // r, r, 1, T).mean(axis=(1, 3)).astype(np.float32), f"LR/X{r}"))
            for vol, sub in vols:
                d = root / "videos" / split / sub / pid
                d.mkdir(parents=True, exist_ok=True)
                nifti.save(vol, d / f"{pid}_2d+1d_sequence01.nii.gz")
                d = root / "imgs" / split / sub / pid
                d.mkdir(parents=True, exist_ok=True)
                for t in range(T):
                    nifti.save(vol[..., t], d / f"{pid}_2d_slice01_frame{t + 1:02d}.nii.gz")
    return root
