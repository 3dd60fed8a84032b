"""Captured vs eager DRF train step (tests/test_graph_gpu.py's f = 32 case):
per-parameter gradient differences after each of three replays / eager
steps, to find where the two first part."""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
sys.path.insert(0, str(Path(__file__).resolve().parents[2] / "tests"))
from test_graph_gpu import _setup  # noqa: E402

kw = dict(in_channels=1, out_channels=1, num_features=32, num_groups=2, upscale_factor=4)
ref_net, ref_step = _setup("DRFNet", kw, (2, 1, 12, 16), (2, 1, 48, 64), 3)
net, step = _setup("DRFNet", kw, (2, 1, 12, 16), (2, 1, 48, 64), 3)
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    for _ in range(2):
        step()
        ref_step()
torch.cuda.current_stream().wait_stream(s)
for (k, p), (_, q) in zip(net.named_parameters(), ref_net.named_parameters()):
    assert torch.equal(p, q), ("params before capture", k)
graph = torch.cuda.CUDAGraph()
with torch.cuda.graph(graph):
    step()
for it in range(3):
    graph.replay()
    ref_step()
    torch.cuda.synchronize()
    bad = []
    for (k, p), (_, q) in zip(net.named_parameters(), ref_net.named_parameters()):
        d = (p.grad - q.grad).abs().max().item()
        if d > 0 or not torch.equal(p, q):
            bad.append(f"{k} grad max|d| {d:.3e} |g| {q.grad.abs().max().item():.3e} param equal {torch.equal(p, q)}")
    print(f"replay {it}: {len(bad)} parameters differ")
    for b in bad[:40]:
        print("  ", b)
