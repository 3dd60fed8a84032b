"""TEST INFRASTRUCTURE ONLY — add the fp16 storage envelope ("fp16_env") to
the committed golden fixtures.

The fixtures were written by oracle.make_golden (which pins the CPU
restatement oracle.cpu_nets bit for bit to the reference); this script needs
only the restatement: for each case it rebuilds the fp64 model from the
fixture's seed and inputs, recomputes the fp64 parameter gradients, and runs
make_golden's dithered 16-bit envelope with fp16 rounding (2^-11 relative,
dither 2^-15).  The fp16 HIP path's gradient bound is a multiple of it, as
the bf16 path's is of "bf16_env".

    python -m oracle.add_fp16_env
"""
from __future__ import annotations

import torch

from . import make_golden as mg


def main():
    import os
    only = os.environ.get("GOLDEN_ONLY")
    for name, spec in mg.CASES.items():
        if only and name not in only.split(","):
            continue
        path = mg.OUT / f"{name}.pt"
        fx = torch.load(path, weights_only=True)
        _, _, cls, kwargs, _, _ = spec
        seed = fx["seed"]
        lr64 = [t.double() for t in fx["lr"]] if isinstance(fx["lr"], list) else fx["lr"].double()
        hr64 = [t.double() for t in fx["hr"]] if isinstance(fx["hr"], list) else fx["hr"].double()
        torch.manual_seed(seed)
        m64 = cls(**kwargs).double().train()
        mg._loss(m64(lr64), hr64).backward()
        g64 = {k: p.grad.detach().clone() for k, p in m64.named_parameters()}
        # same yardstick as the fixture's: its full fp64 gradients where stored
        for k, v in fx["grad_full64"].items():
            assert (g64[k] - v.double()).abs().max().item() <= 1e-9 * (1 + v.abs().max().item()), (name, k)
        fx["fp16_env"] = mg._bf16_envelope(cls, kwargs, lr64, hr64, g64, fx["ref32_err"], seed,
                                           dtype=torch.float16)
        torch.save(fx, path)
        worst = max(v for v in fx["fp16_env"].values() if v is not None)
        print(f"{name}: fp16_env max {worst:.3e}", flush=True)


if __name__ == "__main__":
    main()
