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
fp16 HIP path (loss-scaled backward, BaseNet._loss_scale): output max |d| <=
  5e-3, mean <= 5e-4; gradient rel-L2 <= max(3e-2, 3*fp16_env), fp16_env the
  ideal fp16-storage envelope (as bf16_env, with fp16 rounding of the
  loss-scaled gradients; oracle/add_fp16_env.py).  It is not 8x below
  bf16_env everywhere: a 16-bit rounding of an activation near zero flips
  its mask whatever the significand width (DRF in_block: 3.9e-2 for both the
  ideal fp16 model and the HIP path).  The 3e-2 floor is measured, not
  derived: on edsr_x4_small the HIP fp16 path sits at 1.7e-2 on one weight
  where the 4-draw ideal model predicts 6e-4 (5e-2 in bf16; loss scale 1 to
  2^18 does not move it); on edsr_x4_canon it tracks the envelope (2-3e-2 vs
  1.5-3e-2, tools/diag/f16_edsr.py), hence the 3x multiplier.
bf16 HIP path: output max |d| <= 3e-2, mean |d| <= 3e-3; gradient rel-L2 <=
  max(5e-2, 2*bf16_env) (round 6; 8e-2 before) where bf16_env is the error of an *ideal*
  bf16-storage implementation (fp64 math, bf16 weights, every conv/BN output
  and input gradient rounded to bf16; worst of 4 dithered draws, in the
  fixture).  Every layer stores activations and data-gradients in bf16
  (2^-9 relative rounding), which over ~35 layers random-walks to a few % on
  well-conditioned parameters and ~25% on DUF's BatchNorm parameters and
  EDSR's final bias; zero-gradient parameters <= 2e-2 * max norm.
PSNR within 0.01 dB of the reference's fp32 PSNR for both.

Well-conditioned fixtures (duf_x4_cond, drf_x4_cond; oracle/make_golden.py
find_seed): the seed is chosen so that no ReLU / PReLU input lies within
1e-5 * rms of zero, so no fp32 rounding can flip an activation mask and the
reference's own fp32 gradients sit within 2e-5 of fp64.  There the fp32 HIP
path is held to SURVEY §8d's 1e-4 rel-L2 on EVERY parameter, with no
envelope term.

Gradients stored in full (<= 20000 elements) are compared element-wise;
larger ones through 16 fixed random projections of the fp64 gradient
(rms of the projected error estimates the rel-L2 error; a wrong gradient
with the right norm cannot pass).

Also: the eval-mode forward after the step (BatchNorm from the updated
running statistics, the validation step base_trainer.py:130-134) and one
Adam step (main.py:73) on the HIP gradients against the reference's update.
"""
import hashlib

import pytest
import torch

from vsr_amd import functional as F

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
         "drf_sisr_x2_small", "duf_x4_cond", "drf_x4_cond"]
COND = {"duf_x4_cond", "drf_x4_cond"}
FP16_OUT_EPS = 1e-3  # EDSR fixtures: fp16 output max|d| against fp64 (canon: 4.5e-4)


def _proj(t, key, n):
    """Same directions as oracle/make_golden.py proj() (seed = digest of the name)."""
    seed = int.from_bytes(hashlib.sha256(key.encode()).digest()[:4], "little")
    g = torch.Generator().manual_seed(seed)
    flat = t.detach().double().flatten().cpu()
    return torch.stack([torch.dot(flat, torch.randn(flat.numel(), generator=g, dtype=torch.float64))
                        for _ in range(n)])


def _rel(g, fx, k, full_key="grad_full64", proj_key="grad_proj64", norm_key="grad_norm64"):
    """rel-L2 of g against the fixture's fp64 value: exact when stored in full,
    else estimated from the projections."""
    if k in fx[full_key]:
        ref = fx[full_key][k].double()
        return (g - ref).norm().item() / ref.norm().item()
    e = _proj(g, k, fx["proj_n"]) - fx[proj_key][k]
    return e.pow(2).mean().sqrt().item() / fx[norm_key][k]


@pytest.mark.parametrize("precision", ["fp32", "bf16", "fp16"])
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
    elif precision == "fp16":
        assert d.max().item() <= 5e-3 and d.mean().item() <= 5e-4, (d.max().item(), d.mean().item())
        if name.startswith("edsr"):  # (bounds the tail-bias sign-flip allowance below)
            assert d.max().item() <= FP16_OUT_EPS, d.max().item()
    else:
        assert d.max().item() <= 3e-2 and d.mean().item() <= 3e-3, (d.max().item(), d.mean().item())
    assert abs(_psnr([o.detach() for o in out] if isinstance(out, list) else out.detach(), hr).item()
               - fx["psnr_acdc"]) <= 0.01
    for key, ref in fx["running_stats"].items():  # BatchNorm running statistics after the step
        got_rs = net.state_dict()[key].detach().cpu().double()
        assert (got_rs - ref.double()).abs().max().item() <= {"fp32": 1e-5, "fp16": 3e-3}.get(precision, 2e-2) * (
            1 + ref.double().abs().max().item()), key
    gmax = fx["grad_max64"]
    for k, p in net.named_parameters():
        g = p.grad.detach().cpu().double()
        r32 = fx["ref32_err"][k]
        if r32 is None:  # exact gradient is zero
            assert g.norm().item() <= {"fp32": 1e-4, "fp16": 3e-3}.get(precision, 2e-2) * gmax, (k, g.norm().item())
            continue
        rel = _rel(g, fx, k)
        if precision == "fp32":
            tol = 1e-4 if name in COND else max(1e-4, 3 * r32)
        elif precision == "fp16":
            tol = max(3e-2, 3 * fx["fp16_env"][k])
        else:
            tol = max(5e-2, 2 * fx["bf16_env"][k])
        if precision == "fp16" and k == "tail.conv.bias" and not isinstance(out, list):
            # The bias of the conv feeding the L1 loss gets sum_v sign(o_v - hr_v) / N,
            # and on these fixtures the signs nearly cancel (edsr_x4_canon: N = 6144,
            # |grad| = 2.3e-3), so one residual flipping sign moves the gradient by
            # 2 / N / |grad| = 14 % -- a residual the 16-bit output error can flip for
            # ANY implementation at this precision (canon: the flip is a residual of
            # 4.4e-5 against an fp16 output rms error of 8.9e-5, stencil and tile tail
            # kernels alike: tools/diag/tailbias_fp16.py, profiles/r6_tailbias_fp16.txt);
            # the ideal-16-bit envelope's four draws happened to flip none.  Fixed,
            # fixture-derived allowance: every fixture residual within FP16_OUT_EPS
            # (the fp16 output bound asserted above for the EDSR fixtures) may flip.
            o64, h64 = _flat(fx["output64"]).double(), _flat(fx["hr"]).double()
            near = ((o64 - h64).abs() <= FP16_OUT_EPS).sum().item()
            ref_b = fx["grad_full64"][k].double().norm().item() if k in fx["grad_full64"] else None
            if ref_b:
                tol += 2.0 * near / o64.numel() / ref_b
        assert rel <= tol, (k, rel, tol)


@pytest.mark.parametrize("precision", ["bf16", "fp16"])
@pytest.mark.parametrize("name", [c for c in CASES if c.startswith("edsr")])
def test_stencil_tail_output_error_matches_tile_path(name, precision):
    """the one-channel stencil tail kernels' 16-bit output
    error against fp64 is no larger than the tile kernels' (stencil off) on
    every EDSR fixture -- max and rms per voxel within 10 % -- so a residual
    sign flip on the tail bias gradient is the precision's, not the kernel's
    (see the FP16_OUT_EPS allowance in test_net_matches_golden)."""
    fx = load_golden(name)
    exp = _flat(fx["output64"]).double()
    stats = []
    for mode in (1, 0):
        F.set_conv_path("stencil", mode)
        try:
            net = _build(fx, precision)
            with torch.no_grad():
                out = net(_to(fx["lr"]))
            torch.cuda.synchronize()
        finally:
            F.set_conv_path("stencil", -1)
        d = _flat(out).detach().cpu().double() - exp
        stats.append((d.abs().max().item(), d.pow(2).mean().sqrt().item()))
    (mx_s, rms_s), (mx_t, rms_t) = stats
    assert mx_s <= 1.1 * mx_t and rms_s <= 1.1 * rms_t, stats


def test_cond_fixtures_are_well_conditioned():
    for name in COND:
        fx = load_golden(name)
        assert fx["act_margin"] >= 1e-5 and fx["cond_worst"] <= 5e-5, (name, fx["act_margin"], fx["cond_worst"])


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
@pytest.mark.parametrize("name", ["duf_x4_canon", "duf_x4_cond", "edsr_x4_small", "drf_x4_cond"])
def test_eval_forward_after_step(name, precision):
    """Train step (updates BatchNorm running statistics), then net.eval() forward
    against the fixture's eval output: exercises vsrk_bn_fold_running."""
    fx = load_golden(name)
    net = _build(fx, precision)
    lr, hr = _to(fx["lr"]), _to(fx["hr"])
    _l1(net(lr), hr).backward()
    net.eval()
    with torch.no_grad():
        out = net(lr)
    got, exp = _flat(out).cpu().double(), _flat(fx["output_eval"]).double()
    d = (got - exp).abs()
    if precision == "fp32":
        assert d.max().item() <= 1e-4 * (1 + exp.abs().max().item()), d.max().item()
    else:
        assert d.max().item() <= 3e-2 * (1 + exp.abs().max().item()) and d.mean().item() <= 3e-3, (
            d.max().item(), d.mean().item())


@pytest.mark.parametrize("name", ["edsr_x4_small", "duf_x4_cond", "drf_x4_cond"])
def test_adam_step_on_hip_gradients(name):
    """One torch.optim.Adam step (main.py:73; fp32 master weights) on the fp32
    HIP gradients reproduces the reference's update.  Adam's first step is
    lr * g / (|g| + eps) per element, so only elements whose gradient is below
    fp32 noise can differ (by up to 2 lr); rel-L2 of the update <= 1e-3.
    Parameters whose exact gradient is zero have no defined update and are
    skipped."""
    fx = load_golden(name)
    net = _build(fx, "fp32")
    lr, hr = _to(fx["lr"]), _to(fx["hr"])
    _l1(net(lr), hr).backward()
    a = fx["adam"]
    opt = torch.optim.Adam(net.parameters(), lr=a["lr"], betas=tuple(a["betas"]), eps=a["eps"])
    p0 = {k: p.detach().clone() for k, p in net.named_parameters()}
    opt.step()
    for k, p in net.named_parameters():
        if fx["ref32_err"][k] is None:  # exact gradient 0 (a conv bias feeding a BatchNorm): the
            continue                    # update is lr * noise / (|noise| + eps), no reference value
        upd = (p.detach() - p0[k]).cpu().double()
        if k in fx["adam_update_full"] and k in fx["grad_full64"]:
            # elements whose exact gradient is 0 (e.g. a bias fed by an L1 loss whose signs
            # cancel) get lr * noise / (|noise| + eps): no reference value, left out
            gref, uref = fx["grad_full64"][k].double(), fx["adam_update_full"][k].double()
            keep = gref.abs() > 1e-6 * gref.abs().max()
            assert (upd.abs() <= a["lr"] * 1.001).all(), k
            rel = ((upd - uref)[keep].norm() / uref[keep].norm()).item()
        else:
            rel = _rel(upd, fx, k, "adam_update_full", "adam_update_proj", "adam_update_norm")
        assert rel <= 1e-3, (k, rel)
