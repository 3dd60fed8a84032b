"""bench.py's host-side plumbing (no GPU): the BASELINE configs, their
propagation to spawned ranks, the roofline matchers and the traffic files."""
import argparse
import importlib.util
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
spec = importlib.util.spec_from_file_location("bench_mod", ROOT / "bench.py")
bench = importlib.util.module_from_spec(spec)
spec.loader.exec_module(bench)


def test_configs_cover_the_one_node_baseline_configs():
    assert set(bench.CONFIGS) == {"cfg2", "cfg3", "cfg4", "cfg5"}
    assert bench.CONFIGS["cfg2"]["B"] * bench.CONFIGS["cfg2"]["T"] * 128 * 128 == 1048576
    assert bench.CONFIGS["cfg5"]["precision"] == "fp16" and bench.CONFIGS["cfg5"]["B"] == 8
    assert bench.CONFIGS["cfg3"]["T"] == 30 and bench.CONFIGS["cfg3"]["models"] == "drf"
    # cfg 4: DUF on whole (uncropped) ACDC cine volumes: 256 x 256 HR at 4x
    c4 = bench.CONFIGS["cfg4"]
    assert c4["models"] == "duf" and c4["H"] * 4 == 256 and c4["W"] * 4 == 256 and c4["T"] == 30


def test_apply_config_sets_the_workload():
    args = argparse.Namespace(config="cfg3")
    bench.apply_config(args)
    assert (bench.B, bench.T, bench.DATASET) == (4, 30, "dsb15")
    bench.apply_config(argparse.Namespace(config="cfg4"))
    assert (bench.B, bench.T, bench.H, bench.W) == (2, 30, 64, 64)
    bench.apply_config(argparse.Namespace(config="cfg2"))
    assert (bench.B, bench.T, bench.DATASET, bench.H, bench.W) == (4, 16, "acdc", 128, 128)


class _V:
    def __init__(self, n, d, h, w, c, shuffle=1):
        self.n, self.d, self.h, self.w, self.c, self.shuffle = n, d, h, w, c, shuffle


def test_roofline_matchers_count_the_named_convs():
    m, _ = bench.dominant("edsr")
    assert m(("conv_fwd", (1, 3, 3)), _V(64, 1, 128, 128, 64), _V(64, 1, 128, 128, 64)) == 2 * 64 * 64 * 9 * 64 * 128 * 128
    assert m(("conv_fwd", (1, 3, 3)), _V(64, 1, 128, 128, 64), _V(64, 1, 128, 128, 256)) == 0
    m, _ = bench.dominant("duf")
    x, y = _V(64, 7, 128, 128, 96), _V(64, 7, 128, 128, 32)
    f = m(("conv_fwd", (3, 3, 3)), x, y)
    assert f == 2 * 27 * 96 * 32 * 64 * 7 * 128 * 128
    assert m(("conv_wgrad", (3, 3, 3)), x, y) == f
    assert m(("conv_fwd", (3, 3, 3)), y, x) == f  # data gradient: x = dy (32 channels)


def test_traffic_files_are_per_launch_bytes():
    for model in ("edsr", "duf"):
        t, k = bench._traffic(model, "bf16")
        # the forward roofline kernel: the rolling conv (round 3) or the tile kernel
        assert t is None or (t > 1e8 and k.startswith(("conv_roll_kernel", "conv_fast_kernel")))


def test_every_conv_entry_point_is_timed():
    """The north-star roofline counts the fused data gradients too: every conv
    entry point that can run a roofline kernel launches through timer.wrap
    (conv_reduce / conv_prelu_bwd were not, so the DUF line
    counted 12 of its 18 Conv3d 3x3x3 launches)."""
    import inspect

    from vsr_amd import functional as F
    for fn in (F.conv, F.conv_reduce, F.conv_prelu_bwd, F.conv_wgrad):
        assert "timer.wrap(" in inspect.getsource(fn), fn.__name__
