"""The configs/ drop-in surface (north_star: "configs/ ... stay drop-in
unchanged"; SURVEY §2 row 19, §5 Config/flags).

Every object of a config is ``{name, kwargs}`` resolved by name
(src/main.py:167-178).  These tests load the build's own configs for the
BASELINE configurations and the reference's own training configs
(configs/train/acdc_{sisr,misr,vsr}_config.yaml, with their placeholders --
MyNet, MyLoss, ``value`` -- filled in) and build every object through
vsr_amd.config, as main.py:16-108 does: datasets over a small NIfTI tree in
the reference's on-disk layout, dataloaders, net, losses, metrics,
optimizer, scheduler, logger, monitor and trainer.  Construction only (CPU);
tests/test_configs_gpu.py runs an epoch.
"""
from pathlib import Path

import pytest
import torch
import yaml

from nifti_tree import make_tree
from vsr_amd import config as C

ROOT = Path(__file__).resolve().parent.parent
REF = Path("/root/reference/configs")
OWN = sorted((ROOT / "configs" / "train").glob("*.yaml"))


def _point_data(cfg, tree: Path):
    """data_dir -> the synthetic tree (keeping the imgs / videos choice of the config)."""
    def fix(ds):
        if ds["name"] == "ConcatDataset":
            for p in ds["kwargs"]["datasets"]:
                fix(p)
            return
        kind = "imgs" if "SISR" in ds["name"] else "videos"
        ds["kwargs"]["data_dir"] = str(tree / kind)
    fix(cfg["dataset"])


def _crop_to(cfg, size):
    def fix(ds):
        if ds["name"] == "ConcatDataset":
            for p in ds["kwargs"]["datasets"]:
                fix(p)
            return
        for a in ds["kwargs"].get("augments") or []:
            if a["name"] == "RandomCropPatch":
                a["kwargs"]["size"] = [size, size]
    fix(cfg["dataset"])


@pytest.fixture(scope="module")
def tree(tmp_path_factory):
    return make_tree(tmp_path_factory.mktemp("data"))


def test_box_is_what_main_uses():
    b = C.Box.from_yaml("a: {b: [{name: x, kwargs: {k: 1}}], c: 2}")
    assert b.a.b[0].name == "x" and b.a.b[0].kwargs.k == 1 and b.get("missing") is None
    b.a.update(c=3)
    assert b.a.c == 3 and b.a.pop("c") == 3
    assert b.to_dict() == {"a": {"b": [{"name": "x", "kwargs": {"k": 1}}]}}
    assert C.seed_everything("vsr") == 2613296012  # main.py:29-30


@pytest.mark.parametrize("path", OWN, ids=[p.stem for p in OWN])
def test_own_configs_build(path, tree, tmp_path):
    cfg = yaml.safe_load(path.read_text())
    assert {"main", "dataset", "dataloader", "net", "losses", "metrics", "optimizer", "logger", "monitor",
            "trainer"} <= set(cfg)
    _point_data(cfg, tree)
    _crop_to(cfg, 8)
    cfg["main"]["saved_dir"] = str(tmp_path / "out")
    cfg["dataloader"]["kwargs"]["num_workers"] = 0
    trainer = C.build_train(C.Box(cfg), device="cpu")
    from vsr_amd import nets
    from vsr_amd.runner import trainers
    assert isinstance(trainer.net, getattr(nets, cfg["net"]["name"]))
    assert type(trainer).__name__ == cfg["trainer"]["name"]
    assert isinstance(trainer, trainers.BaseTrainer)
    want = {"fp32": torch.float32, "bf16": torch.bfloat16, "fp16": torch.float16}[cfg.get("precision", "fp32")]
    assert trainer.net.compute_dtype == want
    assert len(trainer.train_dataloader.dataset) > 0 and len(trainer.valid_dataloader.dataset) > 0
    assert trainer.train_dataloader.batch_size == cfg["dataloader"]["kwargs"]["train_batch_size"]
    batch = next(iter(trainer.train_dataloader))
    inputs, targets = trainer._get_inputs_targets(batch)
    assert (tmp_path / "out" / "config.yaml").exists()
    assert [type(f).__name__ for f in trainer.loss_fns] == [c["name"] for c in cfg["losses"]]
    assert [type(f).__name__ for f in trainer.metric_fns] == [c["name"] for c in cfg["metrics"]]


# The reference's own configs with the placeholders filled in the way the
# BASELINE configurations use them (SURVEY §8 canonical constructors).
FILL = {
    "acdc_sisr_config.yaml": ("EDSRNet", dict(in_channels=1, out_channels=1, num_resblocks=2, num_features=16,
                                              upscale_factor=4, res_scale=0.1), {}),
    "acdc_misr_config.yaml": ("DUFNet", dict(in_channels=1, out_channels=1, num_frames=7, size_filter=5,
                                             upscale_factor=4, backbone="_DenseLayer16"), {"num_frames": 7}),
    "acdc_vsr_config.yaml": ("DRFNet", dict(in_channels=1, out_channels=1, num_features=16, num_groups=2,
                                            upscale_factor=4), {"num_frames": 3}),
}


@pytest.mark.skipif(not REF.is_dir(), reason="the reference tree is not on this machine")
@pytest.mark.parametrize("name", sorted(FILL))
def test_reference_train_configs_build(name, tree, tmp_path):
    """configs/train/acdc_*_config.yaml of the reference, read unchanged except
    for its placeholders, resolve every name through vsr_amd."""
    text = (REF / "train" / name).read_text()
    cfg = yaml.safe_load(text)
    net_name, net_kwargs, ds_extra = FILL[name]
    cfg["net"] = {"name": net_name, "kwargs": net_kwargs}
    cfg["losses"] = [{"name": "L1Loss", "weight": 1.0}]
    cfg["main"]["saved_dir"] = str(tmp_path / "out")
    kw = cfg["dataset"]["kwargs"]
    kw["downscale_factor"] = 4
    kw.update(ds_extra)
    for a in kw.get("augments") or []:
        if a["name"] == "RandomCropPatch":
            a["kwargs"].update(size=[8, 8], ratio=4)
    cfg["dataloader"]["kwargs"].update(train_batch_size=2, num_workers=0)
    cfg["optimizer"]["kwargs"]["lr"] = 1e-4
    cfg["trainer"]["kwargs"]["num_epochs"] = 1
    _point_data(cfg, tree)
    # nothing else in the file is a placeholder
    flat = yaml.safe_dump(cfg)
    assert "value" not in flat.split() and "MyNet" not in flat and "MyLoss" not in flat
    trainer = C.build_train(C.Box(cfg), device="cpu")
    assert type(trainer).__name__ == cfg["trainer"]["name"]
    assert type(trainer.logger).__name__ == cfg["logger"]["name"]
    assert type(trainer.monitor).__name__ == "Monitor"
    assert [type(m).__name__ for m in trainer.metric_fns] == ["PSNR", "SSIM"]
    batch = next(iter(trainer.train_dataloader))
    inputs, targets = trainer._get_inputs_targets(batch)
    if isinstance(inputs, list):
        assert len(inputs) == ds_extra["num_frames"]


@pytest.mark.skipif(not REF.is_dir(), reason="the reference tree is not on this machine")
@pytest.mark.parametrize("name", ["acdc_sisr_config.yaml", "acdc_misr_config.yaml", "acdc_vsr_config.yaml"])
def test_reference_test_configs_build(name, tree, tmp_path):
    cfg = yaml.safe_load((REF / "test" / name).read_text())
    net_name, net_kwargs, ds_extra = FILL[name]
    cfg["net"] = {"name": net_name, "kwargs": net_kwargs}
    cfg["losses"] = [{"name": "L1Loss", "weight": 1.0}]
    cfg["metrics"] = [m for m in cfg["metrics"] if m["name"] != "MyMetric"]
    cfg["main"]["saved_dir"] = str(tmp_path / "pred")
    cfg["main"].pop("loaded_path", None)
    cfg["predictor"]["kwargs"].update(saved_dir=str(tmp_path / "pred"), device="cpu")
    kw = cfg["dataset"]["kwargs"]
    kw["downscale_factor"] = 4
    kw.update(ds_extra)
    cfg["dataloader"]["kwargs"]["num_workers"] = 0
    _point_data(cfg, tree)
    pred = C.build_test(C.Box(cfg), device="cpu")
    assert type(pred).__name__ == cfg["predictor"]["name"]


def test_loss_resolution_order():
    """vsr_amd.losses (HIP) first, then torch.nn (e.g. SmoothL1Loss)."""
    fns, w = C.build_losses(C.Box(losses=[{"name": "L1Loss", "weight": 1.0},
                                          {"name": "SmoothL1Loss", "weight": 0.5},
                                          {"name": "CharbonnierLoss", "weight": 2.0, "kwargs": {"epsilon": 1e-3}}]))
    from vsr_amd import losses
    assert isinstance(fns[0], losses.L1Loss) and isinstance(fns[1], torch.nn.SmoothL1Loss)
    assert isinstance(fns[2], losses.CharbonnierLoss) and w == [1.0, 0.5, 2.0]
    with pytest.raises(AttributeError):
        C.build_losses(C.Box(losses=[{"name": "NoSuchLoss", "weight": 1.0}]))


def test_logger_writes_scalars(tmp_path):
    from vsr_amd.callbacks import AcdcVSRLogger
    lg = AcdcVSRLogger(log_dir=tmp_path / "log", net=None, dummy_input=None)
    batch = {"hr_imgs": [torch.rand(2, 1, 8, 8)]}
    lg.write(1, {"Loss": 0.5, "PSNR": 30.0}, batch, [torch.rand(2, 1, 8, 8)], {"Loss": 0.6, "PSNR": 29.0}, batch,
             [torch.rand(2, 1, 8, 8)])
    lg.close()
    lines = (tmp_path / "log" / "scalars.jsonl").read_text().splitlines()
    assert len(lines) == 2 and '"train": 0.5' in lines[0] and '"valid": 0.6' in lines[0]
    img = torch.load(tmp_path / "log" / "images" / "train_0001.pt", weights_only=True)
    assert img.shape[0] == 1 and img.shape[-1] == 2 * 12
