"""Metrics on HIP (PSNR, SSIM, with the trainer's denormalize fused) against
the reference's own values (tests/golden/metrics.pt, made by importing
src/model/metrics.py) and against the oracle restatement on larger random
images.  SSIM tolerance 1e-4 absolute: two fp32 evaluations of E[x^2] - mu^2
on 0..255 images (the reference's own formulation) differ by ~1e-5."""
import pytest
import torch

from oracle import cpu_nets
from tests.conftest import load_golden
from vsr_amd import functional as F
from vsr_amd import metrics

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("ds", ["acdc", "dsb15"])
def test_ssim_psnr_match_reference_fixture(ds):
    fx = load_golden("metrics")
    o, t = fx["out"].to(DEV), fx["target"].to(DEV)
    s = metrics.ssim_denorm(o, t, ds).item()
    assert abs(s - fx[f"ssim_{ds}"]) <= 1e-4, (s, fx[f"ssim_{ds}"])
    p = metrics.psnr_denorm(o, t, ds).item()
    assert abs(p - fx[f"psnr_{ds}"]) <= 1e-3, (p, fx[f"psnr_{ds}"])
    per = metrics.psnr_denorm(o, t, ds, size_average=False).cpu()
    assert torch.allclose(per, fx[f"psnr_{ds}_per_sample"], atol=1e-3)


@pytest.mark.parametrize("shape", [(4, 1, 64, 96), (2, 3, 45, 77), (1, 1, 11, 11), (3, 1, 512, 512)])
def test_ssim_matches_oracle(shape):
    g = torch.Generator().manual_seed(sum(shape))
    o = torch.randn(shape, generator=g)
    t = (o + 0.3 * torch.randn(shape, generator=g))
    od, td = cpu_nets.denormalize(o, "acdc"), cpu_nets.denormalize(t, "acdc")
    ref_all = float(cpu_nets.ssim(od, td, channels=shape[1]))
    ref_per = cpu_nets.ssim(od, td, channels=shape[1], size_average=False)
    m, per = F.ssim(o.to(DEV), t.to(DEV), *metrics.DATASET_STATS["acdc"], 255.0, denormalize=True)
    assert abs(m.item() - ref_all) <= 1e-4
    assert (per.cpu() - ref_per).abs().max().item() <= 1e-4
    # SSIM module on already-denormalized images (size_average False/True)
    mod = metrics.SSIM(channels=shape[1], size_average=False)
    assert (mod(od.to(DEV), td.to(DEV)).cpu() - ref_per).abs().max().item() <= 1e-4
