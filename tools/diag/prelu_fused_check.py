"""Diagnose vsrk_conv_fwd_prelu_bwd vs conv + prelu_bwd (slope gradient)."""
import sys
from pathlib import Path
import torch
sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
from vsr_amd import _native, functional as F  # noqa: E402
_native.load()
DEV, dt = "cuda", torch.bfloat16
for form in ("plain", "up_dgrad", "down_dgrad"):
    g = torch.Generator().manual_seed(11)
    f, n, h, w, r = 64, 2, 13, 37, 4
    if form == "plain":
        x = torch.randn((n, 1, h, w, f), generator=g).to(DEV, dt)
        wt = torch.randn((f, f, 1, 3, 3), generator=g) / (9 * f) ** 0.5
        wp, kw, yshape = F.pack_weight(wt.to(DEV), 1, dt), {}, (n, 1, h, w, f)
    else:
        k, s, p = 8, 4, 2
        tr = form == "up_dgrad"
        wt = torch.randn((f, f, k, k), generator=g) / (f * k) ** 0.5
        weq, _ = F.subpixel_conv_weight(wt.to(DEV), None, k, s, p, transposed=tr)
        wp = F.pack_weight(weq, 1, dt)
        code = F.subpixel_code(k, s, p, tr, True)
        if tr:
            x = torch.randn((n, 1, h * s, w * s, f), generator=g).to(DEV, dt)
            kw, yshape = dict(x_shuffle=s, subpixel=code), (n, 1, h, w, f)
        else:
            x = torch.randn((n, 1, h, w, f), generator=g).to(DEV, dt)
            kw, yshape = dict(y_shuffle=s, subpixel=code), (n, 1, h * s, w * s, f)
    y_fwd = torch.randn(yshape, generator=g).to(DEV, dt)
    a = torch.tensor([0.2], device=DEV)
    y_ref = torch.empty(yshape, dtype=dt, device=DEV)
    F.conv(x, wp, y_ref, (1, 3, 3), (0, 1, 1), **kw)
    t_plain = y_ref.clone()
    da_ref = torch.zeros(1, device=DEV)
    F.prelu_bwd(y_fwd, y_ref, a, y_ref, da_ref, False)
    y = torch.empty(yshape, dtype=dt, device=DEV)
    da = torch.zeros(1, device=DEV)
    ok = F.conv_prelu_bwd(x, wp, y, (1, 3, 3), (0, 1, 1), y_fwd, a, da, False, **kw)
    m = y_fwd.float()
    torch_da = lambda yy: ((yy.float() * m)[m < 0].double().sum() / 0.2 ** 2).item()
    exp = torch.where(m > 0, t_plain.float(), 0.2 * t_plain.float())
    print(form, "ok", ok, "da_ref", da_ref.item(), "da_fused", da.item(), "torch(y_ref)", torch_da(y_ref),
          "torch(y_fused)", torch_da(y), "torch(exp)", torch_da(exp),
          "max|y-y_ref|", (y.float() - y_ref.float()).abs().max().item(),
          "n big", int(((y.float() - y_ref.float()).abs() > 0.05).sum()), flush=True)
