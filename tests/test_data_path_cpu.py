"""Data path on the CPU: the NIfTI restatement, the
Dataset mirrors over a NIfTI tree laid out as acdc_preprocess.py writes it,
and the augment index maps against the numpy transforms they replace.
nibabel is absent here: the reader is pinned by round trips and by the
header fields' byte offsets of the NIfTI-1 standard (parity of the reader
itself: unpinned by a reference fixture)."""
import random
import struct

import numpy as np
import pytest

from vsr_amd.data import nifti
from vsr_amd.data import transforms as T
from vsr_amd.data.datasets import AcdcMISRDataset, AcdcSISRDataset, AcdcVSRDataset


@pytest.mark.parametrize("suffix", [".nii", ".nii.gz"])
@pytest.mark.parametrize("dtype", [np.float32, np.int16, np.float64])
def test_nifti_round_trip(tmp_path, suffix, dtype):
    rng = np.random.default_rng(0)
    a = (rng.standard_normal((7, 5, 1, 4)) * 100).astype(dtype)
    p = tmp_path / f"x_2d+1d{suffix}"
    nifti.save(a, p)
    img = nifti.load(p)
    assert img.header.get_data_shape() == (7, 5, 1, 4)
    b = img.get_data()
    assert b.dtype == a.dtype and np.array_equal(a, b)
    raw = (nifti.gzip.open(p, "rb") if suffix.endswith(".gz") else open(p, "rb")).read()
    assert struct.unpack("<i", raw[:4])[0] == 348
    assert struct.unpack("<8h", raw[40:56])[:5] == (4, 7, 5, 1, 4)
    # Fortran order on disk: the first axis varies fastest
    off = int(struct.unpack("<f", raw[108:112])[0])
    first = np.frombuffer(raw[off:off + 2 * a.itemsize], dtype=a.dtype)
    assert first[0] == a[0, 0, 0, 0] and first[1] == a[1, 0, 0, 0]


def test_nifti_scaling(tmp_path):
    a = np.arange(24, dtype=np.int16).reshape(2, 3, 4)
    p = tmp_path / "s.nii"
    nifti.save(a, p)
    raw = bytearray(open(p, "rb").read())
    struct.pack_into("<2f", raw, 112, 0.5, 3.0)
    open(p, "wb").write(bytes(raw))
    assert np.allclose(nifti.load(p).get_data(), a * 0.5 + 3.0)


def _tree(root, T_=6, h=8, w=10, r=2, patients=2, slices=False):
    """acdc_preprocess.py:55-85 layout: sequences under videos/, 2-D slices
    under imgs/ (the SISR glob *2d* would also match *2d+1d*)."""
    rng = np.random.default_rng(1)
    vols = {}
    for i in range(patients):
        hr = rng.integers(0, 255, (h * r, w * r, 1, T_)).astype(np.float32)
        lr = hr.reshape(h, r, w, r, 1, T_).mean(axis=(1, 3)).astype(np.float32)
        pid = f"patient{i:03d}"
        for kind, vol, sub in (("HR", hr, "HR"), ("LR", lr, f"LR/X{r}")):
            d = root / "train" / sub / pid
            d.mkdir(parents=True, exist_ok=True)
            if slices:
                for t in range(T_):
                    nifti.save(vol[..., t], d / f"{pid}_2d_frame{t:02d}.nii.gz")
            else:
                nifti.save(vol, d / f"{pid}_2d+1d_sequence.nii.gz")
        vols[pid] = (lr, hr)
    return vols


def _cyc(v, idx):
    return np.stack([v[..., i % v.shape[-1]] for i in idx], -1)


def test_vsr_and_misr_windows(tmp_path):
    vols = _tree(tmp_path / "videos")
    _tree(tmp_path / "imgs", slices=True)
    lr0, hr0 = vols["patient000"]
    # (augments=None would compose a ToTensor ahead of the transforms' own,
    # as in the reference: training configs always list their augments)
    vsr = AcdcVSRDataset(downscale_factor=2, transforms=None, augments=[], num_frames=3, data_dir=tmp_path / "videos",
                         type="train")
    assert len(vsr) == 12
    s = vsr[0]  # patient 0, t = 0, 'last': frames {-2, -1, 0}
    got = np.stack([x.numpy()[0] for x in s["lr_imgs"]], -1)
    assert np.array_equal(got, _cyc(lr0, [-2, -1, 0])[:, :, 0])
    assert len(s["hr_imgs"]) == 3 and s["hr_imgs"][0].shape == (1, 16, 20)
    misr = AcdcMISRDataset(downscale_factor=2, transforms=None, augments=[], num_frames=5, data_dir=tmp_path / "videos",
                           type="train")
    m = misr[5]  # patient 0, t = 5, 'middle': frames {3..7} mod 6, target frame 5
    got = np.stack([x.numpy()[0] for x in m["lr_imgs"]], -1)
    assert np.array_equal(got, _cyc(lr0, [3, 4, 5, 6, 7])[:, :, 0])
    assert np.array_equal(m["hr_img"].numpy()[0], hr0[:, :, 0, 5])
    sisr = AcdcSISRDataset(downscale_factor=2, transforms=None, augments=[], data_dir=tmp_path / "imgs", type="train")
    assert len(sisr) == 12 and sisr[0]["lr_img"].shape == (1, 8, 10) and sisr[0]["hr_img"].shape == (1, 16, 20)
    with pytest.raises(ValueError):
        AcdcVSRDataset(downscale_factor=5, transforms=None, data_dir=tmp_path / "videos", type="train")


def _apply(img, m, oh, ow):
    ys = m.y0 + m.dy * np.arange(oh)
    xs = m.x0 + m.dx * np.arange(ow)
    return img[np.ix_(ys, xs)]


@pytest.mark.parametrize("seed", range(6))
@pytest.mark.parametrize("order", ["crop_first", "flip_first"])
def test_augment_maps_equal_numpy_transforms(seed, order):
    rng = np.random.default_rng(seed)
    n, h, w, r = 3, 12, 14, 4
    lr = [rng.standard_normal((h, w, 1)).astype(np.float32) for _ in range(n)]
    hr = [rng.standard_normal((h * r, w * r, 1)).astype(np.float32) for _ in range(n)]
    crop = T.RandomCropPatch(size=[6, 5], ratio=r)
    flips = [T.RandomHorizontalFlip(0.5), T.RandomVerticalFlip(0.5)]
    aug = T.Compose([crop] + flips if order == "crop_first" else flips + [crop])
    random.seed(seed)
    ref = aug(*lr, *hr)
    random.seed(seed)
    lm, hm = T.plan_augments(aug, (h, w), (h * r, w * r))
    assert (lm.h, lm.w, hm.h, hm.w) == (6, 5, 24, 20)
    for k in range(n):
        assert np.array_equal(_apply(lr[k][..., 0], lm, 6, 5), np.asarray(ref[k])[..., 0])
        assert np.array_equal(_apply(hr[k][..., 0], hm, 24, 20), np.asarray(ref[n + k])[..., 0])


def test_compose_from_config_dicts():
    c = T.compose([{"name": "RandomCropPatch", "kwargs": {"size": [4, 4], "ratio": 2}},
                   {"name": "RandomHorizontalFlip"}])
    assert [type(t).__name__ for t in c.transforms] == ["RandomCropPatch", "RandomHorizontalFlip"]
    x = np.zeros((8, 8, 1), np.float32)
    out = T.compose(None)(x)
    assert tuple(out.shape) == (8, 8, 1)
