"""Synthetic cine data: the reference Dataset dict contract and the cyclic
temporal window of acdc_misr_dataset.py:53-68 (restated independently here)."""
import torch

from vsr_amd.data import SyntheticCine, cyclic_windows, synth_cine


def _ref_window(t, n, T):
    # acdc_misr_dataset.py:57-68 'middle' order with cyclic wrap
    start, end = t - (n - 1) // 2, t + ((n - 1) - (n - 1) // 2) + 1
    idx = list(range(T))
    if start < 0:
        return idx[start:] + idx[:end]
    if end > T:
        return idx[start:] + idx[:end % T]
    return idx[start:end]


def test_cyclic_windows_match_reference_order():
    T, n = 16, 7
    vol = torch.arange(T, dtype=torch.float32).view(1, T, 1, 1).expand(2, T, 3, 3).contiguous()
    win = cyclic_windows(vol, n)
    assert len(win) == n
    for t in range(T):
        got = [int(w[t, 0, 0, 0]) for w in win]
        assert got == _ref_window(t, n, T), t


def test_synthetic_statistics_and_shapes():
    lr, hr = synth_cine(2, 4, 16, 16, 4, seed=3)
    assert lr.shape == (2, 4, 16, 16) and hr.shape == (2, 4, 64, 64)
    raw = hr * 48.084 + 54.089
    assert torch.allclose(raw, raw.round(), atol=1e-3) and raw.min() >= -1e-3 and raw.max() <= 255 + 1e-3
    # LR is the 4x4 average of HR (in raw intensity)
    pooled = torch.nn.functional.avg_pool2d(raw.view(8, 1, 64, 64), 4).view(2, 4, 16, 16)
    assert torch.allclose(lr * 48.084 + 54.089, pooled, atol=1e-3)


def test_dict_contract():
    for task, keys in (("sisr", {"lr_img", "hr_img", "index"}), ("misr", {"lr_imgs", "hr_img", "index"}),
                       ("vsr", {"lr_imgs", "hr_imgs", "index"})):
        ds = SyntheticCine(task, volumes=1, frames=5, size=(8, 8), upscale_factor=2, num_frames=3)
        item = ds[0]
        assert set(item) == keys
        if task == "misr":
            assert len(item["lr_imgs"]) == 3 and item["lr_imgs"][0].shape == (1, 8, 8)
        if task == "vsr":
            assert len(item["lr_imgs"]) == 5 and item["hr_imgs"][0].shape == (1, 16, 16)
