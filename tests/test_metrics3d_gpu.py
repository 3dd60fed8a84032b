"""SSIM(dim=3) and the Cardiac bounding-box metrics against the reference's own
values (tests/golden/metrics3d.pt, written by oracle/make_golden.py from
src/model/metrics.py:39-165 on fixed data).  fp32 kernels with fp64 partial
sums: within 1e-5 relative of the reference."""
import pickle

import pytest
import torch

from tests.conftest import load_golden
from vsr_amd import functional as F
from vsr_amd import metrics
from vsr_amd.utils import DATASET_STATS

pytestmark = pytest.mark.gpu
DEV = "cuda"


def test_ssim3d_denormalized_matches_reference():
    fx = load_golden("metrics3d")
    mean, std = DATASET_STATS["acdc"]
    m, per = F.ssim(fx["out"].to(DEV), fx["target"].to(DEV), mean, std, 255.0, denormalize=True)
    assert abs(m.item() - fx["ssim3d_acdc"]) <= 1e-5 * abs(fx["ssim3d_acdc"]), (m.item(), fx["ssim3d_acdc"])
    assert (per.cpu().double() - fx["ssim3d_acdc_per_sample"].double()).abs().max().item() <= 1e-5


def test_ssim3d_module_on_volumes():
    fx = load_golden("metrics3d")
    from oracle import cpu_nets
    od = cpu_nets.denormalize(fx["out"], "acdc")
    td = cpu_nets.denormalize(fx["target"], "acdc")
    got = metrics.SSIM(dim=3)(od.to(DEV), td.to(DEV)).item()
    assert abs(got - fx["ssim3d_acdc"]) <= 1e-5 * abs(fx["ssim3d_acdc"])
    with pytest.raises(ValueError):
        metrics.SSIM(dim=3)(od[:, :, 0].to(DEV), td[:, :, 0].to(DEV))


@pytest.mark.parametrize("fmt", ["pickle", "json"])
def test_cardiac_metrics(tmp_path, fmt):
    fx = load_golden("metrics3d")
    coords = fx["cardiac_coords"]
    path = tmp_path / f"coords.{fmt}"
    if fmt == "pickle":  # the reference's own format (metrics.py:123-125)
        with open(path, "wb") as fh:
            pickle.dump(dict(coords), fh)
    else:
        import json
        path.write_text(json.dumps({k: list(v) for k, v in coords.items()}))
    o, t = fx["cardiac_out"].to(DEV), fx["cardiac_target"].to(DEV)
    cp, cs = metrics.CardiacPSNR(str(path)), metrics.CardiacSSIM(str(path))
    for name, ref in fx["cardiac"].items():
        assert abs(cp(o, t, name).item() - ref["psnr"]) <= 1e-5 * abs(ref["psnr"]), name
        assert abs(cs(o, t, name).item() - ref["ssim"]) <= 1e-5 * abs(ref["ssim"]), name
