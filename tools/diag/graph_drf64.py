"""DRF f = 64: eager vs eager (determinism) and graph vs eager parameters
after a few train steps; which parameters differ and by how much."""
import sys

import torch

sys.path.insert(0, ".")  # run from the repo root
sys.path.insert(0, "tests")
import test_graph_gpu as T  # noqa: E402
from vsr_amd import functional as F  # noqa: E402

if len(sys.argv) > 1:  # e.g. wgrad_row=0 (vsrk_conv_set_path)
    for kv in sys.argv[1].split(","):
        p_, m_ = kv.split("=")
        F.set_conv_path(p_, int(m_))

kw = dict(in_channels=1, out_channels=1, num_features=64, num_groups=3, upscale_factor=4)
xs, ys, seq = (2, 1, 12, 16), (2, 1, 48, 64), 3


def diff(a, b):
    out = []
    for (k, p), (_, q) in zip(a.named_parameters(), b.named_parameters()):
        d = (p.detach() - q.detach()).abs().max().item()
        if d > 0:
            out.append((k, d))
    return out


n1, s1 = T._setup("DRFNet", kw, xs, ys, seq)
n2, s2 = T._setup("DRFNet", kw, xs, ys, seq)
for _ in range(5):
    s1()
    s2()
torch.cuda.synchronize()
print(sys.argv[1:], "eager vs eager:", diff(n1, n2)[:3], flush=True)
n3, s3 = T._setup("DRFNet", kw, xs, ys, seq)
n4, s4 = T._setup("DRFNet", kw, xs, ys, seq)
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    for _ in range(2):
        s3()
        s4()
torch.cuda.current_stream().wait_stream(s)
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    s3()
for _ in range(3):
    g.replay()
torch.cuda.synchronize()
for _ in range(3):
    s4()
torch.cuda.synchronize()
print(sys.argv[1:], "graph vs eager:", len(diff(n3, n4)), diff(n3, n4)[:3], flush=True)
