"""End-to-end parity of the fused generators against the golden fixtures made
from the reference itself (oracle/make_golden.py): same seed -> same initial
weights (checked), then forward output, L1 loss, PSNR and every parameter
gradient through the HIP path.

Tolerances: fp32 path: output max |d| <= 1e-4 (normalized units),
gradient rel-L2 <= 1e-4 per parameter; bf16 path: output max |d| <= 3e-2,
mean |d| <= 3e-3; PSNR within 0.01 dB for both.  bf16 gradients (§8d states
no bound) are held to rel-L2 <= 8e-2: every layer stores its activation and
data-gradient in bf16 (2^-9 relative rounding), which over the ~35 layers of
EDSR random-walks to the measured 3-4.5 %.  bf16 bias gradients are sums of
B*H*W per-voxel terms with heavy cancellation, so their relative error is
larger (measured up to 8.8 %): held to rel-L2 <= 0.15.
"""
import pytest
import torch

from tests.conftest import load_golden
from vsr_amd import nets

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _build(fx, precision):
    torch.manual_seed(fx["seed"])
    net = getattr(nets, fx["class"])(**fx["kwargs"])
    for k, v in net.state_dict().items():
        if v.is_floating_point():
            assert abs(float(v.double().sum()) - fx["param_sum"][k]) <= 1e-9 * (1 + abs(fx["param_sum"][k])), k
    return net.to(DEV).set_precision(precision).train()


def _to(x):
    return [t.to(DEV) for t in x] if isinstance(x, list) else x.to(DEV)


def _l1(out, hr):
    if isinstance(out, list) and not isinstance(hr, list):
        return torch.stack([torch.nn.functional.l1_loss(o, hr) for o in out]).mean()
    if isinstance(out, list):
        return torch.stack([torch.nn.functional.l1_loss(o, t) for o, t in zip(out, hr)]).mean()
    return torch.nn.functional.l1_loss(out, hr)


def _flat(x):
    return torch.cat([t.flatten() for t in x]) if isinstance(x, list) else x.flatten()


def _psnr(out, hr):
    from vsr_amd.metrics import psnr_denorm
    if isinstance(out, list) and not isinstance(hr, list):
        out = out[-1]
    if isinstance(out, list):
        return torch.stack([psnr_denorm(o, t, "acdc") for o, t in zip(out, hr)]).mean()
    return psnr_denorm(out, hr, "acdc")


CASES = ["edsr_x4_small", "edsr_x3_small", "edsr_x2_cfg1", "edsr_x4_canon"]


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
@pytest.mark.parametrize("name", CASES)
def test_net_matches_golden(name, precision):
    fx = load_golden(name)
    net = _build(fx, precision)
    lr, hr = _to(fx["lr"]), _to(fx["hr"])
    out = net(lr)
    loss = _l1(out, hr)
    loss.backward()
    torch.cuda.synchronize()
    got, exp = _flat(out).detach().cpu().double(), _flat(fx["output"]).double()
    d = (got - exp).abs()
    if precision == "fp32":
        assert d.max().item() <= 1e-4, d.max().item()
    else:
        assert d.max().item() <= 3e-2 and d.mean().item() <= 3e-3, (d.max().item(), d.mean().item())
    assert abs(_psnr([o.detach() for o in out] if isinstance(out, list) else out.detach(), hr).item()
               - fx["psnr_acdc"]) <= 0.01
    for k, p in net.named_parameters():
        tol = 1e-4 if precision == "fp32" else (0.15 if k.endswith("bias") else 8e-2)
        gn = fx["grad_norm"][k]
        if k in fx["grad_full"]:
            ref = fx["grad_full"][k].double()
            rel = (p.grad.detach().cpu().double() - ref).norm().item() / max(ref.norm().item(), 1e-12)
        else:
            rel = abs(p.grad.double().norm().item() - gn) / max(gn, 1e-12)
        assert rel <= tol, (k, rel)
