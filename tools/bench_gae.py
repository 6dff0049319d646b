"""GAE kernel timings (HIP events): the three mm_gae_ex algorithms on the
rollout shape (T=16, 65,536 columns) and on whole-episode batches (few
columns, long T, episodes of up to 1,200 steps)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "marl-maze_amd"))
from marlmaze import ops  # noqa: E402

rng = np.random.default_rng(0)
for T, N, algos in ((16, 65536, ("column", "walk")), (32, 4096, ("column", "walk", "scan")),
                    (400, 4096, ("column", "walk", "scan")), (15600, 1, ("column", "walk", "scan")),
                    (15600, 16, ("column", "walk", "scan"))):
    r = torch.as_tensor(rng.choice(np.float32([0, 0.5, 1]), size=(T, N))).cuda()
    v = torch.randn(T, N, device="cuda")
    d = torch.zeros(T, N, dtype=torch.uint8)
    for n in range(N):
        t = -1
        while True:
            t += int(rng.integers(1, 1201 if T > 1000 else 60))
            if t >= T:
                break
            d[t, n] = 1
    d = d.cuda()
    for a in algos:
        for _ in range(3):
            ops.gae(r, v, d, algo=a)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            ops.gae(r, v, d, algo=a)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / 20 * 1e3
        print(f"T={T:6d} N={N:6d} {a:7s} {us:9.1f} us  {17 * T * N / us / 1e3:8.1f} GB/s (17 B per position)",
              flush=True)
