"""The data path pinned by the reference's own code: tests/golden/data_path.pt
holds sample dicts produced by the reference's src/data/transforms.py and
src/data/datasets/acdc_{sisr,misr,vsr}_dataset.py (oracle/make_data_golden.py,
nibabel and SimpleITK replaced by stand-ins, see there) under per-sample
Python ``random`` seeds.  The vsr_amd Datasets over the same volumes, written
as real NIfTI files by vsr_amd.data.nifti, must give bitwise the same
samples: windows with cyclic wrap, flips, the LR/HR crop pair, Normalize and
ToTensor.  (tests/test_device_batch_gpu.py holds the GPU gather to the same
fixture.)"""
import random
from pathlib import Path

import numpy as np
import pytest
import torch

from vsr_amd import data as D
from vsr_amd.data import nifti

GOLDEN = Path(__file__).resolve().parent / "golden" / "data_path.pt"


@pytest.fixture(scope="module")
def fx():
    return torch.load(GOLDEN, weights_only=True)


def write_tree(root: Path, fx):
    """The fixture's volumes as NIfTI files at the fixture's relative paths."""
    T = fx["geometry"]["T"]
    r = fx["geometry"]["r"]
    for split in ("train", "valid"):
        for i, v in enumerate(fx["volumes"]):
            pid = f"patient{i + 1:03d}"
            for arr, sub in ((v["hr"].numpy(), "HR"), (v["lr"].numpy(), f"LR/X{r}")):
                d = root / "videos" / split / sub / pid
                d.mkdir(parents=True, exist_ok=True)
                nifti.save(arr, d / f"{pid}_2d+1d_sequence01.nii.gz")
                d = root / "imgs" / split / sub / pid
                d.mkdir(parents=True, exist_ok=True)
                for t in range(T):
                    nifti.save(arr[..., t], d / f"{pid}_2d_slice01_frame{t + 1:02d}.nii.gz")
    return root


def _case_ids():
    return [c["name"] for c in torch.load(GOLDEN, weights_only=True)["cases"]]


@pytest.mark.parametrize("name", _case_ids())
def test_dataset_samples_equal_reference(name, fx, tmp_path):
    case = next(c for c in fx["cases"] if c["name"] == name)
    root = write_tree(tmp_path, fx)
    cls = getattr(D, case["cls"])
    ds = cls(downscale_factor=fx["geometry"]["r"], transforms=fx["transforms"],
             augments=fx["augments"] if case["split"] == "train" else None, data_dir=root / case["kind"],
             type=case["split"], **case["kwargs"])
    got_entries = [(str(Path(e[0]).relative_to(root)),) + tuple(e[2:]) for e in ds.data]
    assert got_entries == [tuple(e) for e in case["data"]]
    for idx, (seed, want) in enumerate(zip(case["seeds"], case["samples"])):
        random.seed(seed)
        np.random.seed(seed)
        s = ds[idx]
        assert sorted(s) == sorted(want)
        for k, v in want.items():
            g = torch.stack(s[k]) if isinstance(s[k], list) else s[k]
            if k == "index":
                assert int(g) == v
            else:
                assert g.dtype == v.dtype and torch.equal(g, v), (name, idx, k)
