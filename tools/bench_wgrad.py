"""Weight-gradient GEMM timings (HIP events) at the update's shapes: the
hand-written mm_gemm_wgrad (x3, f16) against the fp32 library GEMM
(torch dY^T X on hipBLASLt) that it replaced."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "marl-maze_amd"))
from marlmaze import x3  # noqa: E402


def t(f, n=10):
    for _ in range(3):
        f()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        f()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


for M, N, K in ((419430, 264, 264), (419430, 264, 460), (419430, 6, 264), (209715, 64, 130), (209715, 64, 64),
                (209715, 1, 64)):
    dy = torch.randn(M, N, device="cuda")
    x = torch.randn(M, K, device="cuda")
    fl = 2.0 * M * N * K
    r = [f"M={M} {N}x{K}:"]
    for name, f in (("lib", lambda: dy.t().mm(x)), ("x3", lambda: x3.wgrad(dy, x)),
                    ("f16", lambda: x3.wgrad(dy, x, prec="f16"))):
        us = t(f)
        r.append(f"{name} {us:8.1f} us ({fl / us / 1e6:6.1f} TF/s, {4.0 * M * (N + K) / us / 1e3:6.0f} GB/s)")
    print("  ".join(r), flush=True)
