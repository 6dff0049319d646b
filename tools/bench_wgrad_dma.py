"""x2 trunk weight gradients: k_wgrad_dma (LDS-DMA staging, two raw stages in flight) against k_wgrad_rect
(register staging), alternating in one process (x3.set_wgrad_algo), HIP events, median of ROUNDS x 10
launches; algorithmic bytes 4 M (N + K) per launch.  One JSON line per shape.

  python tools/bench_wgrad_dma.py [M]
"""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "marl-maze_amd"))
from marlmaze import x3  # noqa: E402

ROUNDS = 7


def timed(f, n=10):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        f()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


M = int(sys.argv[1]) if len(sys.argv) > 1 else 419430
s = float(2 ** (M.bit_length() - 1))
for N, K in ((264, 264), (264, 460)):
    g = torch.Generator(device="cuda").manual_seed(N + K)
    dy = torch.randn(M, N, device="cuda", generator=g) / M
    x = torch.randn(M, K, device="cuda", generator=g)
    out = torch.empty(N, K, device="cuda")
    res = {"dma": [], "reg": []}
    for algo in res:  # warm-up (kernel attributes, first launches)
        x3.set_wgrad_algo(algo)
        timed(lambda: x3.wgrad(dy, x, prec="x2", dscale=s, out=out), 3)
    for _ in range(ROUNDS):
        for algo in res:
            x3.set_wgrad_algo(algo)
            res[algo].append(timed(lambda: x3.wgrad(dy, x, prec="x2", dscale=s, out=out)))
    x3.set_wgrad_algo("dma")
    byt = 4.0 * M * (N + K)
    line = {"M": M, "N": N, "K": K}
    for algo, v in res.items():
        med = statistics.median(v)
        line[algo + "_us"] = round(med, 1)
        line[algo + "_TBps"] = round(byt / med / 1e6, 3)
    line["speedup"] = round(line["reg_us"] / line["dma_us"], 3)
    print(json.dumps(line), flush=True)
