"""GPU batch gather (include/vsrk_data.h, vsr_amd.data.DeviceCineBatcher)
against the CPU pipeline it replaces: the reference's windowing
(acdc_{misr,vsr}_dataset.py) and numpy augments (transforms.py:321-450)
under the same Python `random` seed -- the build's CPU restatement, and the
reference's own code through the committed fixture tests/golden/data_path.pt
(oracle/make_data_golden.py).  Pure gathers: bit-exact."""
import random

import numpy as np
import pytest
import torch

from vsr_amd.data import DeviceCineBatcher
from vsr_amd.data import transforms as T
from vsr_amd.data.datasets import _take, _window

pytestmark = pytest.mark.gpu


def _aug():
    return T.Compose([T.RandomCropPatch(size=[6, 5], ratio=4), T.RandomHorizontalFlip(0.5),
                      T.RandomVerticalFlip(0.5)])


@pytest.mark.parametrize("task", ["sisr", "misr", "vsr"])
@pytest.mark.parametrize("seed", [0, 1, 2])
def test_gather_matches_cpu_pipeline(task, seed):
    rng = np.random.default_rng(seed)
    V, Tn, h, w, r, n = 3, 7, 12, 14, 4, 5
    lr = rng.standard_normal((V, Tn, h, w)).astype(np.float32)
    hr = rng.standard_normal((V, Tn, h * r, w * r)).astype(np.float32)
    items = [(int(rng.integers(V)), int(rng.integers(Tn))) for _ in range(9)]
    aug = _aug()
    b = DeviceCineBatcher(torch.from_numpy(lr).cuda(), torch.from_numpy(hr).cuda(), task, num_frames=n, augments=aug)
    random.seed(seed)
    out = b(items)
    torch.cuda.synchronize()
    random.seed(seed)
    order = "middle" if task == "misr" else "last"
    c = n // 2
    for i, (v, t) in enumerate(items):
        lv = np.moveaxis(lr[v], 0, -1)[:, :, None, :]  # (h, w, 1, T) as the NIfTI volumes
        hv = np.moveaxis(hr[v], 0, -1)[:, :, None, :]
        if task == "sisr":
            lo, ho = aug(lv[..., t], hv[..., t])
            assert np.array_equal(out["lr_img"][i, 0].cpu().numpy(), np.asarray(lo)[..., 0])
            assert np.array_equal(out["hr_img"][i, 0].cpu().numpy(), np.asarray(ho)[..., 0])
            continue
        s, e = _window(t, n, Tn, order)
        lw, hw = _take(lv, s, e), _take(hv, s, e)
        imgs = aug(*[lw[..., k] for k in range(n)], *[hw[..., k] for k in range(n)])
        for k in range(n):
            assert np.array_equal(out["lr_imgs"][k][i, 0].cpu().numpy(), np.asarray(imgs[k])[..., 0])
        if task == "misr":
            assert np.array_equal(out["hr_img"][i, 0].cpu().numpy(), np.asarray(imgs[n + c])[..., 0])
        else:
            for k in range(n):
                assert np.array_equal(out["hr_imgs"][k][i, 0].cpu().numpy(), np.asarray(imgs[n + k])[..., 0])


def test_gather_without_augments_and_normalize():
    V, Tn, h, w = 2, 6, 8, 8
    g = torch.Generator().manual_seed(3)
    lr = torch.rand((V, Tn, h, w), generator=g) * 255
    hr = torch.rand((V, Tn, 2 * h, 2 * w), generator=g) * 255
    b = DeviceCineBatcher(lr.cuda(), hr.cuda(), "vsr", num_frames=3, normalize=(54.089, 48.084))
    out = b([(1, 0), (0, 5)])
    ref = (lr[1, [4, 5, 0]] - 54.089) / (48.084 + 1e-10)
    got = torch.stack([x[0, 0] for x in out["lr_imgs"]]).cpu()
    assert torch.allclose(got, ref, rtol=0, atol=1e-5)
    with pytest.raises(ValueError):
        DeviceCineBatcher(lr.cuda(), hr.cuda(), "vsr", augments=[T.Normalize([0.0], [1.0])])


def _golden():
    from pathlib import Path
    return torch.load(Path(__file__).resolve().parent / "golden" / "data_path.pt", weights_only=True)


@pytest.mark.parametrize("name", ["misr_middle5_train", "misr_last4_train", "vsr_last3_train", "vsr_middle5_train",
                                  "sisr_train"])
def test_gather_matches_reference_fixture(name):
    """vsrk_gather_windows against the reference's own Dataset + transforms
    (tests/golden/data_path.pt, oracle/make_data_golden.py): bitwise, per
    sample under the fixture's Python `random` seed."""
    import re
    fx = _golden()
    case = next(c for c in fx["cases"] if c["name"] == name)
    lr = torch.stack([v["lr"][:, :, 0].permute(2, 0, 1) for v in fx["volumes"]]).cuda()  # (V, T, h, w)
    hr = torch.stack([v["hr"][:, :, 0].permute(2, 0, 1) for v in fx["volumes"]]).cuda()
    task = {"AcdcMISRDataset": "misr", "AcdcVSRDataset": "vsr", "AcdcSISRDataset": "sisr"}[case["cls"]]
    kw = case["kwargs"]
    b = DeviceCineBatcher(lr, hr, task, num_frames=kw.get("num_frames", 1), temporal_order=kw.get("temporal_order"),
                          augments=fx["augments"], normalize=(54.089, 48.084))
    for seed, entry, want in zip(case["seeds"], case["data"], case["samples"]):
        vol = int(re.search(r"patient(\d+)", entry[0]).group(1)) - 1
        t = int(entry[1]) if len(entry) > 1 else int(re.search(r"frame(\d+)", entry[0]).group(1)) - 1
        random.seed(seed)
        out = b([(vol, t)])
        if task == "sisr":
            assert torch.equal(out["lr_img"][0].cpu(), want["lr_img"])
            assert torch.equal(out["hr_img"][0].cpu(), want["hr_img"])
            continue
        got = torch.stack([x[0] for x in out["lr_imgs"]]).cpu()
        assert torch.equal(got, want["lr_imgs"]), (name, seed)
        if task == "misr":
            assert torch.equal(out["hr_img"][0].cpu(), want["hr_img"])
        else:
            assert torch.equal(torch.stack([x[0] for x in out["hr_imgs"]]).cpu(), want["hr_imgs"])
