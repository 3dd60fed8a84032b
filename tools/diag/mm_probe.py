"""Probe: hipBLASLt (torch.mm) on DUF's 1x1 head shapes, channels-last rows,
against the tile kernel's times (conv_fast 512 -> 400 fp32 out 1.8 ms,
512 -> 256 / 400 -> 512 data gradients 1.1 ms, r5z_duf_bf16_kernel_summary)."""
import torch


def t(fn, it=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it * 1e3


dev = "cuda"
M = 64 * 128 * 128
for K, N in ((512, 400), (512, 256), (400, 512), (256, 512)):
    x = torch.randn((M, K), device=dev, dtype=torch.bfloat16)
    w = torch.randn((N, K), device=dev, dtype=torch.bfloat16)
    y = torch.empty((M, N), device=dev, dtype=torch.bfloat16)
    res = {"bf16": t(lambda: torch.mm(x, w.t(), out=y))}
    try:
        yf = torch.empty((M, N), device=dev, dtype=torch.float32)
        res["f32out"] = t(lambda: torch.mm(x, w.t(), out_dtype=torch.float32, out=yf))
    except Exception as ex:  # noqa: BLE001
        res["f32out"] = f"n/a ({type(ex).__name__}: {str(ex)[:80]})"
    print((K, N), res, flush=True)
