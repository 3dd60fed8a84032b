"""The CPU oracle (oracle/cpu_nets.py) reproduces the golden fixtures, which
oracle/make_golden.py checked bit-for-bit against the reference itself.
Runs on any host (fp32 CPU; small tolerance for a different host BLAS)."""
import pytest
import torch

from oracle import cpu_nets
from tests.conftest import load_golden

CLASSES = {"EDSRNet": cpu_nets.EDSRRef, "DUFNet": cpu_nets.DUFRef, "DRFNet": cpu_nets.DRFRef,
           "DRFSISRNet": cpu_nets.DRFSISRRef}
CASES = ["edsr_x4_small", "edsr_x3_small", "edsr_x2_cfg1", "duf_x4_canon", "drf_x4_canon", "drf_sisr_x2_small"]


def _flat(x):
    return torch.cat([t.flatten() for t in x]) if isinstance(x, list) else x.flatten()


@pytest.mark.parametrize("name", CASES)
def test_oracle_matches_golden(name):
    fx = load_golden(name)
    torch.manual_seed(fx["seed"])
    net = CLASSES[fx["class"]](**fx["kwargs"]).train()
    for k, v in net.state_dict().items():
        if v.is_floating_point():
            assert abs(float(v.double().sum()) - fx["param_sum"][k]) <= 1e-9 * (1 + abs(fx["param_sum"][k])), k
    out = net(fx["lr"])
    hr = fx["hr"]
    if isinstance(out, list) and not isinstance(hr, list):
        loss = torch.stack([torch.nn.functional.l1_loss(o, hr) for o in out]).mean()
    elif isinstance(out, list):
        loss = torch.stack([torch.nn.functional.l1_loss(o, t) for o, t in zip(out, hr)]).mean()
    else:
        loss = torch.nn.functional.l1_loss(out, hr)
    loss.backward()
    d = (_flat(out).detach() - _flat(fx["output"])).abs().max().item()
    assert d <= 1e-5, d
    assert abs(loss.item() - fx["loss_l1"]) <= 1e-6
    for k, p in net.named_parameters():
        ref = fx["grad_norm"][k]
        assert abs(p.grad.double().norm().item() - ref) <= 1e-4 * (1 + ref), k
    for k, v in fx["running_stats"].items():
        assert torch.allclose(net.state_dict()[k].float(), v.float(), atol=1e-6), k


def test_metrics_golden():
    fx = load_golden("metrics")
    for ds in ("acdc", "dsb15"):
        o, t = cpu_nets.denormalize(fx["out"], ds), cpu_nets.denormalize(fx["target"], ds)
        assert abs(cpu_nets.psnr(o, t).item() - fx[f"psnr_{ds}"]) <= 1e-5


def test_oracle_ssim_matches_reference_fixture():
    """The SSIM restatement (oracle/cpu_nets.ssim) against the reference's own
    metrics.SSIM output recorded in tests/golden/metrics.pt."""
    from oracle import cpu_nets
    fx = load_golden("metrics")
    for ds in ("acdc", "dsb15"):
        o = cpu_nets.denormalize(fx["out"], ds)
        t = cpu_nets.denormalize(fx["target"], ds)
        assert abs(float(cpu_nets.ssim(o, t)) - fx[f"ssim_{ds}"]) <= 1e-6
