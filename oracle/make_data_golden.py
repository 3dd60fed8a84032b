"""TEST INFRASTRUCTURE ONLY — golden samples of the reference's data path.

Run in the build container (needs /root/reference):
    python -m oracle.make_data_golden

Loads the reference's own src/data/transforms.py and
src/data/datasets/{base,acdc_sisr,acdc_misr,acdc_vsr}_dataset.py by path and
runs their seeded ``__getitem__`` (windowing with cyclic wrap, the numpy
augments RandomHorizontalFlip / RandomVerticalFlip / RandomCropPatch, then
Normalize + ToTensor) over small synthetic cine volumes.  Two libraries the
files import are absent here:
  * ``SimpleITK`` (transforms.py:5, used only by RandomElasticDeformation,
    which is not exercised) is an empty module;
  * ``nibabel`` (datasets' ``nib.load(path).get_data()`` and
    ``.header.get_data_shape()``) is a stand-in that serves the synthetic
    arrays by file path -- so the NIfTI *reader* is not what this pins; the
    windowing, augment draws and transforms are.
The directory tree the datasets glob is created with empty files named as
acdc_preprocess.py:70-85 writes them.  Writes tests/golden/data_path.pt:
the volumes, each case's dataset kwargs, the Python ``random`` seed of each
sample and the reference's sample dicts (tensors).  Nothing from the
reference is copied into the repository.
"""
from __future__ import annotations

import importlib.util
import os
import random
import sys
import tempfile
import types
from pathlib import Path

import numpy as np
import torch

from .ref_loader import REF

OUT = Path(__file__).resolve().parent.parent / "tests" / "golden" / "data_path.pt"

PATIENTS, T, H, W, R = 2, 6, 40, 48, 4
AUG = [{"name": "RandomHorizontalFlip"}, {"name": "RandomVerticalFlip"},
       {"name": "RandomCropPatch", "kwargs": {"size": [6, 5], "ratio": R}}]
TF = [{"name": "Normalize", "kwargs": {"means": [54.089], "stds": [48.084]}}, {"name": "ToTensor"}]
# (case name, dataset class, directory kind, split, kwargs)
CASES = [
    ("misr_middle5_train", "AcdcMISRDataset", "videos", "train", dict(num_frames=5, temporal_order="middle")),
    ("misr_last4_train", "AcdcMISRDataset", "videos", "train", dict(num_frames=4, temporal_order="last")),
    ("vsr_last3_train", "AcdcVSRDataset", "videos", "train", dict(num_frames=3, temporal_order="last")),
    ("vsr_middle5_train", "AcdcVSRDataset", "videos", "train", dict(num_frames=5, temporal_order="middle")),
    ("vsr_valid", "AcdcVSRDataset", "videos", "valid", dict(num_frames=3)),
    ("sisr_train", "AcdcSISRDataset", "imgs", "train", {}),
]


class _Box(dict):
    """The attribute dict the reference's compose() reads ({name, kwargs})."""

    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError:
            raise AttributeError(k) from None


def _volumes():
    rng = np.random.default_rng(7)
    vols = []
    for _ in range(PATIENTS):
        hr = rng.integers(0, 256, (H, W, 1, T)).astype(np.float32)
        lr = hr.reshape(H // R, R, W // R, R, 1, T).mean(axis=(1, 3)).round().astype(np.float32)
        vols.append((lr, hr))
    return vols


def _tree(root: Path, vols):
    """Empty files in the reference's layout + the path -> array map of the nibabel stand-in."""
    arrays = {}
    for split in ("train", "valid"):
        for i, (lr, hr) in enumerate(vols):
            pid = f"patient{i + 1:03d}"
            for arr, sub in ((hr, "HR"), (lr, f"LR/X{R}")):
                d = root / "videos" / split / sub / pid
                d.mkdir(parents=True, exist_ok=True)
                p = d / f"{pid}_2d+1d_sequence01.nii.gz"
                p.touch()
                arrays[str(p)] = arr
                d = root / "imgs" / split / sub / pid
                d.mkdir(parents=True, exist_ok=True)
                for t in range(T):
                    p = d / f"{pid}_2d_slice01_frame{t + 1:02d}.nii.gz"
                    p.touch()
                    arrays[str(p)] = arr[..., t]
    return arrays


def _load_reference(arrays):
    sys.dont_write_bytecode = True
    nib = types.ModuleType("nibabel")

    class _Img:
        def __init__(self, a):
            self._a = a
            self.header = types.SimpleNamespace(get_data_shape=lambda: a.shape)

        def get_data(self):
            return self._a.copy()

    nib.load = lambda path: _Img(arrays[str(path)])
    sys.modules["nibabel"] = nib
    sys.modules.setdefault("SimpleITK", types.ModuleType("SimpleITK"))
    pkgs = {}
    for pkg in ("src", "src.data", "src.data.datasets"):
        m = types.ModuleType(pkg)
        m.__path__ = []
        sys.modules[pkg] = m
        pkgs[pkg] = m
    pkgs["src"].data = pkgs["src.data"]
    pkgs["src.data"].datasets = pkgs["src.data.datasets"]

    def load(name, rel):
        spec = importlib.util.spec_from_file_location(name, os.path.join(REF, rel))
        mod = importlib.util.module_from_spec(spec)
        sys.modules[name] = mod
        parent, _, leaf = name.rpartition(".")
        setattr(sys.modules[parent], leaf, mod)
        spec.loader.exec_module(mod)
        return mod

    load("src.data.transforms", "src/data/transforms.py")
    load("src.data.datasets.base_dataset", "src/data/datasets/base_dataset.py")
    mods = {}
    for cls, rel in (("AcdcSISRDataset", "acdc_sisr_dataset"), ("AcdcMISRDataset", "acdc_misr_dataset"),
                     ("AcdcVSRDataset", "acdc_vsr_dataset")):
        mods[cls] = getattr(load(f"src.data.datasets.{rel}", f"src/data/datasets/{rel}.py"), cls)
    return mods


def _tensors(sample):
    out = {}
    for k, v in sample.items():
        if isinstance(v, list):
            out[k] = torch.stack(v)
        elif torch.is_tensor(v):
            out[k] = v
        else:
            out[k] = int(v)
    return out


def main():
    vols = _volumes()
    with tempfile.TemporaryDirectory() as tmp:
        root = Path(tmp)
        arrays = _tree(root, vols)
        classes = _load_reference(arrays)
        fx = {"volumes": [{"lr": torch.from_numpy(lr), "hr": torch.from_numpy(hr)} for lr, hr in vols],
              "geometry": {"T": T, "H": H, "W": W, "r": R}, "augments": AUG, "transforms": TF, "cases": []}
        for name, cls, kind, split, kw in CASES:
            ds = classes[cls](downscale_factor=R, transforms=[_Box(t) for t in TF],
                              augments=[_Box(a) for a in AUG] if split == "train" else None,
                              data_dir=root / kind, type=split, **kw)
            samples, seeds = [], []
            for idx in range(len(ds)):
                seed = 1000 * (len(fx["cases"]) + 1) + idx
                random.seed(seed)
                np.random.seed(seed)
                samples.append(_tensors(ds[idx]))
                seeds.append(seed)
            entries = [(str(Path(e[0]).relative_to(root)),) + tuple(e[2:]) for e in ds.data]
            fx["cases"].append({"name": name, "cls": cls, "kind": kind, "split": split, "kwargs": kw,
                                "seeds": seeds, "samples": samples, "data": entries})
            print(f"{name}: {len(ds)} samples, keys {sorted(samples[0])}")
    torch.save(fx, OUT)
    print(f"wrote {OUT} ({OUT.stat().st_size / 1024:.0f} KiB)")


if __name__ == "__main__":
    main()
