"""Loss kernels (vsrk_loss_fwd / vsrk_loss_bwd through vsr_amd.losses) against
the reference's own values: tests/golden/metrics.pt holds torch.nn.L1Loss /
MSELoss and the reference's HuberLoss(delta=0.7) / CharbonnierLoss(1e-3)
(src/model/losses.py:5-34) evaluated on fixed data, with their input
gradients (oracle/make_golden.py run_metrics).  fp32 kernels with
double-precision partial sums: loss within 1e-6 relative, gradient within
1e-6 relative of its max (the gradient of a mean is O(1/count))."""
import pytest
import torch

from tests.conftest import load_golden
from vsr_amd import losses

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _make(name, params):
    if name == "HuberLoss":
        return losses.HuberLoss(delta=params[name])
    if name == "CharbonnierLoss":
        return losses.CharbonnierLoss(epsilon=params[name])
    return getattr(losses, name)()


@pytest.mark.parametrize("name", ["L1Loss", "MSELoss", "HuberLoss", "CharbonnierLoss"])
def test_loss_matches_reference(name):
    fx = load_golden("metrics")
    fn = _make(name, fx["loss_params"])
    o = fx["out"].to(DEV).requires_grad_(True)
    t = fx["target"].to(DEV)
    val = fn(o, t)
    val.backward()
    ref = fx["loss"][name]
    assert abs(val.item() - ref) <= 1e-6 * max(1.0, abs(ref)), (name, val.item(), ref)
    g, gr = o.grad.cpu(), fx["grad"][name]
    assert (g - gr).abs().max().item() <= 1e-6 * gr.abs().max().item() + 1e-12, name


@pytest.mark.parametrize("name", ["L1Loss", "MSELoss"])
def test_loss_upstream_gradient_scale(name):
    """backward multiplies by the upstream gradient (weighted loss sums, base_trainer.py:126)."""
    fx = load_golden("metrics")
    fn = _make(name, fx["loss_params"])
    o = fx["out"].to(DEV).requires_grad_(True)
    (0.25 * fn(o, fx["target"].to(DEV))).backward()
    assert torch.allclose(o.grad.cpu(), 0.25 * fx["grad"][name], rtol=1e-5, atol=1e-12)
