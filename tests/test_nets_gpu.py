"""End-to-end parity of the fused generators against golden fixtures made from
the reference itself (oracle/make_golden.py): same seed -> same initial
weights (checked), then forward output, L1 loss, PSNR, BatchNorm running
statistics and every parameter gradient through the HIP path.

Yardstick: an fp64 evaluation of the (bitwise-pinned) CPU restatement.  The
fixture records how far the reference's own fp32 CPU path is from it
(out_err32, ref32_err[param]); DUF's gradients are ill-conditioned (ReLU
masks of near-zero pre-activations flip with summation order) and the fp32
reference itself is up to 1e-2 away, while EDSR's is ~1e-5.

fp32 HIP path: output max |d| <= max(1e-4, 3*out_err32); gradient rel-L2 <=
  max(1e-4, 3*ref32_err) per parameter (SURVEY §8d's 1e-4 wherever the
  reference itself is that accurate).  ref32_err is the reference
  algorithm's fp32 envelope: the worst of its own fp32 runs at 1/2/4/8 CPU
  threads and of 8 fp64 runs with fp32-scale noise injected at every conv /
  BatchNorm output and input gradient (oracle/make_golden.py).  The envelope
  matters for DUF only: one filter-head pre-activation sits at 1.6e-7 against
  5e-7 fp32 error, so its ReLU mask legitimately flips with summation order
  (tools/duf_mask_flips.py), which moves filterNet.conv1.bias by 2.3e-3 and
  everything upstream by ~3e-4.  The BN and dynamic-filter kernels alone are
  checked at 1e-5..1e-4 against fp64 in test_bn_duf_kernels_gpu.py.
  Parameters whose exact gradient is 0 (conv biases feeding a BatchNorm):
  |g| <= 1e-4 * max gradient norm.
bf16 HIP path: output max |d| <= 3e-2, mean |d| <= 3e-3; gradient rel-L2 <=
  max(8e-2, 2*bf16_env) where bf16_env is the error of an *ideal*
  bf16-storage implementation (fp64 math, bf16 weights, every conv/BN output
  and input gradient rounded to bf16; worst of 4 dithered draws, in the
  fixture).  Every layer stores activations and data-gradients in bf16
  (2^-9 relative rounding), which over ~35 layers random-walks to a few % on
  well-conditioned parameters and ~25% on DUF's BatchNorm parameters and
  EDSR's final bias; zero-gradient parameters <= 2e-2 * max norm.
PSNR within 0.01 dB of the reference's fp32 PSNR for both.
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


CASES = ["edsr_x4_small", "edsr_x3_small", "edsr_x2_cfg1", "edsr_x4_canon", "duf_x4_canon", "drf_x4_canon",
         "drf_sisr_x2_small"]


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
    got, exp = _flat(out).detach().cpu().double(), _flat(fx["output64"]).double()
    d = (got - exp).abs()
    if precision == "fp32":
        assert d.max().item() <= max(1e-4, 3 * fx["out_err32"]), d.max().item()
    else:
        assert d.max().item() <= 3e-2 and d.mean().item() <= 3e-3, (d.max().item(), d.mean().item())
    assert abs(_psnr([o.detach() for o in out] if isinstance(out, list) else out.detach(), hr).item()
               - fx["psnr_acdc"]) <= 0.01
    for key, ref in fx["running_stats"].items():  # BatchNorm running statistics after the step
        got_rs = net.state_dict()[key].detach().cpu().double()
        assert (got_rs - ref.double()).abs().max().item() <= (1e-5 if precision == "fp32" else 2e-2) * (
            1 + ref.double().abs().max().item()), key
    gmax = fx["grad_max64"]
    for k, p in net.named_parameters():
        g = p.grad.detach().cpu().double()
        r32 = fx["ref32_err"][k]
        if r32 is None:  # exact gradient is zero
            assert g.norm().item() <= (1e-4 if precision == "fp32" else 2e-2) * gmax, (k, g.norm().item())
            continue
        if k in fx["grad_full64"]:
            ref = fx["grad_full64"][k].double()
            rel = (g - ref).norm().item() / ref.norm().item()
        else:
            n64 = fx["grad_norm64"][k]
            rel = abs(g.norm().item() - n64) / n64
        if precision == "fp32":
            tol = max(1e-4, 3 * r32)
        else:
            tol = max(8e-2, 2 * fx["bf16_env"][k])
        assert rel <= tol, (k, rel, tol)
