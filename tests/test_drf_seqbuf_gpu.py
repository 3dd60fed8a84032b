"""DRF backward with its sequence buffers in chunks (the
frame-major buffers the run-batched weight gradients read are allocated in
chunks of Kg frames under VSR_DRF_SEQ_BUDGET_GB and dropped once every run over
a chunk is launched).  Against the default (one chunk of all T frames) and
against per-frame weight gradients (VSR_DRF_SEQ_WGRAD=0): every weight gradient
agrees to fp32 summation order (the runs partition the frames
differently); the chunked run keeps fewer bytes alive.  (The nets return no
input gradient -- the reference's trainers never ask for one.)"""
import pytest
import torch

from vsr_amd import nets
from vsr_amd.losses import L1Loss

pytestmark = pytest.mark.gpu

T = 6


def _grads(monkeypatch, budget_gb=None, seq=True, run_cap=0, with_k=False):
    monkeypatch.setenv("VSR_DRF_RUN_FRAMES", str(run_cap))
    if budget_gb is not None:
        monkeypatch.setenv("VSR_DRF_SEQ_BUDGET_GB", str(budget_gb))
    else:
        monkeypatch.delenv("VSR_DRF_SEQ_BUDGET_GB", raising=False)
    torch.manual_seed(0)
    net = nets.DRFNet(in_channels=1, out_channels=1, num_features=32, num_groups=2,
                      upscale_factor=4).cuda().set_precision("bf16").train()
    net.SEQ_WGRAD = seq
    g = torch.Generator().manual_seed(1)
    x = [torch.randn((2, 1, 12, 16), generator=g).cuda() for _ in range(T)]
    y = [torch.randn((2, 1, 48, 64), generator=g).cuda() for _ in range(T)]
    l1 = L1Loss()
    torch.cuda.synchronize()
    torch.cuda.reset_peak_memory_stats()
    base = torch.cuda.memory_allocated()
    out = net(x)
    torch.stack([l1(o, t) for o, t in zip(out, y)]).mean().backward()
    torch.cuda.synchronize()
    peak = torch.cuda.max_memory_allocated() - base
    res = ({k: p.grad.detach().clone() for k, p in net.named_parameters()},
           getattr(net, "_seq_run_frames", None), peak)
    return (*res, dict(getattr(net, "_seq_run_k", {}))) if with_k else res


def test_chunked_sequence_buffers(monkeypatch):
    gw, k_all, peak_all = _grads(monkeypatch)
    assert k_all == T
    # one frame of this net's backward sequence buffers is ~0.3 MB: budgets
    # of 2 and 1 frames' worth force Kg = 2 and Kg = 1
    fb = None
    for kg in (2, 1):
        budget = (kg + 0.5) * _frame_bytes() / 2 ** 30
        gw2, k2, peak2 = _grads(monkeypatch, budget)
        assert k2 == kg
        for k, v in gw.items():
            err = (gw2[k] - v).norm() / v.norm().clamp_min(1e-30)
            assert err < 2e-5, (kg, k, float(err))
        fb = peak2
    assert fb < peak_all, (fb, peak_all)
    gw3, _, _ = _grads(monkeypatch, seq=False)
    for k, v in gw.items():
        err = (gw3[k] - v).norm() / v.norm().clamp_min(1e-30)
        assert err < 2e-5, (k, float(err))


def test_runs_need_not_divide_chunks(monkeypatch):
    """a run length that does not divide the chunk (Kg = 5 of
    T = 6, runs of 2 frames: [0,2) [2,4) [4,5) | [5,6)) -- round 5 lowered K
    until it divided Kg, down to single frames for a prime Kg"""
    gw, _, _ = _grads(monkeypatch)
    budget = 5.5 * _frame_bytes() / 2 ** 30
    gw2, kg, _, run_k = _grads(monkeypatch, budget, run_cap=2, with_k=True)
    assert kg == 5
    assert run_k and set(run_k.values()) == {2}, run_k
    for k, v in gw.items():
        err = (gw2[k] - v).norm() / v.norm().clamp_min(1e-30)
        assert err < 2e-5, (k, float(err))


def _frame_bytes():
    # DRFNet(f=32, G=2, r=4) at b=2, 12x16 LR: mirrors the estimate in
    # _DRFBase's backward (dup*, low-res gradients, high-res gh* / dt2_*)
    b, h, w, f, G, s = 2, 12, 16, 32, 2, 4
    H, W = h * s, w * s
    fe = H * W * f + (H // 2) * (W // 2) * f + h * w * f
    fe += (2 * G + 2) * h * w * f + h * w * 4 * f
    fe += (2 * G - 1) * H * W * f
    return fe * b * 2
