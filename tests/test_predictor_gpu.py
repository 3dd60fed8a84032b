"""The predictor mirror (base_predictor.py / acdc_{sisr,vsr}_predictor.py):
batch size 1, eval mode, per-frame losses and HIP metrics, frame-weighted log,
and the exported CSV / PNG / GIF.  The log equals the reference loop's values
computed with the oracle metrics on the same outputs (1e-4 relative)."""
import csv

import pytest
import torch
from torch.utils.data import DataLoader

from oracle import cpu_nets
from vsr_amd import losses, metrics, nets
from vsr_amd.data import SyntheticCine
from vsr_amd.runner import predictors

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")


def _oracle_log(frames):
    acc = {"Loss": 0.0, "L1Loss": 0.0, "PSNR": 0.0, "SSIM": 0.0}
    for o, y in frames:
        o, y = o.cpu(), y.cpu()
        l1 = torch.nn.functional.l1_loss(o, y).item()
        od, yd = cpu_nets.denormalize(o, "acdc"), cpu_nets.denormalize(y, "acdc")
        for k, v in (("Loss", l1), ("L1Loss", l1), ("PSNR", cpu_nets.psnr(od, yd).item()),
                     ("SSIM", cpu_nets.ssim(od, yd).item())):
            acc[k] += v
    return {k: v / len(frames) for k, v in acc.items()}


def _check(log, ref):
    assert list(log) == list(ref)
    for k in ("Loss", "L1Loss", "PSNR"):
        assert abs(log[k] - ref[k]) <= 1e-4 * abs(ref[k]), (k, log[k], ref[k])
    assert abs(log["SSIM"] - ref["SSIM"]) <= 1e-4


def test_sisr_predictor_export(tmp_path):
    torch.manual_seed(0)
    net = nets.EDSRNet(1, 1, num_resblocks=2, num_features=16, upscale_factor=2).to(DEV).set_precision("fp32")
    ds = SyntheticCine("sisr", volumes=1, frames=3, size=(12, 16), upscale_factor=2)
    loader = DataLoader(ds, batch_size=1, shuffle=False)
    pred = predictors.AcdcSISRPredictor(DEV, loader, net, [losses.L1Loss()], [1.0], [metrics.PSNR(), metrics.SSIM()],
                                        saved_dir=tmp_path, exported=True)
    log = pred.predict()
    net.eval()
    with torch.no_grad():
        frames = [(net(b["lr_img"].to(DEV)), b["hr_img"]) for b in loader]
    _check(log, _oracle_log(frames))
    rows = list(csv.reader(open(tmp_path / "results.csv")))
    assert rows[0] == ["name", "PSNR", "SSIM", "L1Loss"]
    assert len(rows) == 1 + len(ds)
    assert len(list((tmp_path / "imgs").rglob("*.png"))) == len(ds)
    assert len(list((tmp_path / "videos").rglob("*.gif"))) == len(ds)


def test_vsr_predictor(tmp_path):
    torch.manual_seed(0)
    net = nets.DRFNet(1, 1, num_features=16, num_groups=2, upscale_factor=2).to(DEV).set_precision("fp32")
    ds = SyntheticCine("vsr", volumes=2, frames=3, size=(12, 16), upscale_factor=2)
    loader = DataLoader(ds, batch_size=1, shuffle=False)
    pred = predictors.AcdcVSRPredictor(DEV, loader, net, [losses.L1Loss()], [1.0], [metrics.PSNR(), metrics.SSIM()],
                                       saved_dir=tmp_path, exported=True)
    log = pred.predict()
    net.eval()
    frames = []
    with torch.no_grad():
        for b in loader:
            outs = net([x.to(DEV) for x in b["lr_imgs"]])
            frames += list(zip(outs, b["hr_imgs"]))
    _check(log, _oracle_log(frames))
    rows = list(csv.reader(open(tmp_path / "results.csv")))
    assert len(rows) == 1 + len(frames)
    assert rows[1][0].endswith("_frame01")
    assert len(list((tmp_path / "imgs").rglob("*.png"))) == len(frames)


def test_predictor_rejects_batched_loader():
    net = nets.EDSRNet(1, 1, num_resblocks=1, num_features=16, upscale_factor=2).to(DEV)
    loader = DataLoader(SyntheticCine("sisr", volumes=1, frames=2, size=(8, 8), upscale_factor=2), batch_size=2)
    with pytest.raises(ValueError):
        predictors.AcdcSISRPredictor(DEV, loader, net, [losses.L1Loss()], [1.0], [metrics.PSNR()])


@pytest.mark.parametrize("kind", ["sisr", "misr"])
def test_export_names_follow_the_reference(kind, tmp_path):
    """ACDC file names (acdc_preprocess.py:70-85) through the SISR / MISR
    predictors: rows named as acdc_{sisr,misr}_predictor.py:66-68 /
    acdc_misr_predictor.py:67-69, one PNG per frame
    imgs/<patient>/<slice>_<frame>.png (no overwrites), one GIF per sequence
    videos/<patient>/<sequence>.gif; a reference checkpoint (pickled Monitor)
    loads through the allow-list."""
    import sys
    import types
    from nifti_tree import make_tree
    from vsr_amd.callbacks.monitor import Monitor
    from vsr_amd.data import AcdcMISRDataset, AcdcSISRDataset

    T = 8  # >= num_frames: a 7-frame window wraps at most once (acdc_misr_dataset.py:61-68)
    root = make_tree(tmp_path / "data", T=T, H=16, W=16, patients=2)
    tf = [{"name": "Normalize", "kwargs": {"means": [54.089], "stds": [48.084]}}, {"name": "ToTensor"}]
    if kind == "sisr":
        ds = AcdcSISRDataset(downscale_factor=2, transforms=tf, data_dir=root / "imgs", type="test")
        net = nets.EDSRNet(1, 1, num_resblocks=1, num_features=16, upscale_factor=2)
        cls = predictors.AcdcSISRPredictor
    else:
        ds = AcdcMISRDataset(downscale_factor=2, transforms=tf, num_frames=7, data_dir=root / "videos", type="test")
        net = nets.DUFNet(1, 1, num_frames=7, size_filter=5, upscale_factor=2, backbone="_DenseLayer16")
        cls = predictors.AcdcMISRPredictor
    net = net.to(DEV).set_precision("fp32")
    # a checkpoint in the reference's format: the Monitor pickled under src.callbacks.monitor
    mod = types.ModuleType("src.callbacks.monitor")
    mod.Monitor = type("Monitor", (), {"__module__": "src.callbacks.monitor"})
    for name in ("src", "src.callbacks"):
        sys.modules.setdefault(name, types.ModuleType(name))
    sys.modules["src.callbacks.monitor"] = mod
    try:
        ref_mon = mod.Monitor()
        ref_mon.__dict__.update(checkpoints_dir=tmp_path / "ck", mode="min", target="Loss", saved_freq=1,
                                early_stop=0, best=1.0, not_improved_count=0)
        torch.save({"net": net.state_dict(), "monitor": ref_mon, "epoch": 1}, tmp_path / "model_best.pth")
    finally:
        for name in ("src.callbacks.monitor", "src.callbacks", "src"):
            sys.modules.pop(name, None)
    loader = DataLoader(ds, batch_size=1, shuffle=False)
    out = tmp_path / "pred"
    pred = cls(DEV, loader, net, [losses.L1Loss()], [1.0], [metrics.PSNR()], saved_dir=out, exported=True)
    pred.load(tmp_path / "model_best.pth")
    pred.predict()
    rows = list(csv.reader(open(out / "results.csv")))
    names = [r[0] for r in rows[1:]]
    want = [f"patient{p:03d}_2d_slice01_frame{t + 1:02d}" for p in range(2) for t in range(T)]
    assert names == want
    pngs = sorted(str(p.relative_to(out / "imgs")) for p in (out / "imgs").rglob("*.png"))
    assert pngs == sorted(f"patient{p:03d}/slice01_frame{t + 1:02d}.png" for p in range(2) for t in range(T))
    gifs = sorted(str(p.relative_to(out / "videos")) for p in (out / "videos").rglob("*.gif"))
    assert gifs == [f"patient{p:03d}/sequence01.gif" for p in range(2)]
    from PIL import Image
    assert Image.open(out / "videos" / "patient000" / "sequence01.gif").n_frames == T
