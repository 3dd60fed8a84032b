"""The cfg 3 DRF train step (B = 4, T = 30, 128^2 LR, F = 64, G = 4, bf16)
captured into a HIP graph vs the same steps run eagerly: parameters after
two steps compared bitwise (the bench's default for cfg 3 replays the graph)."""
import sys

import torch

sys.path.insert(0, ".")  # run from the repo root
sys.path.insert(0, "tests")
import test_graph_gpu as T  # noqa: E402

kw = dict(in_channels=1, out_channels=1, num_features=64, num_groups=4, upscale_factor=4)
xs, ys, seq = (4, 1, 128, 128), (4, 1, 512, 512), 30
n3, s3 = T._setup("DRFNet", kw, xs, ys, seq)
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    s3()
torch.cuda.current_stream().wait_stream(s)
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    s3()
g.replay()
g.replay()
torch.cuda.synchronize()
pg = {k: p.detach().clone() for k, p in n3.named_parameters()}
del g, n3, s3
torch.cuda.empty_cache()
n4, s4 = T._setup("DRFNet", kw, xs, ys, seq)
for _ in range(3):  # warm-up step + the two the graph replayed (the capture itself ran no kernels)
    s4()
torch.cuda.synchronize()
bad = [(k, (pg[k] - p.detach()).abs().max().item()) for k, p in n4.named_parameters() if not torch.equal(pg[k], p.detach())]
print("cfg3 graph vs eager: differing params", len(bad), bad[:3], flush=True)
