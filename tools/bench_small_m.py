"""Small-M GEMM table: the hand-written engine (csrc/x3mlp.hip, x3 = fp32-class
bf16x3) against the fp32 library GEMM (torch on hipBLASLt) at the row counts
the reference's own configuration produces:

* M = 1, 2: the single-sample API (get_action, Maze.step-driven inference);
* M = 300 / 3,000 / 6,000: main.py's PPO(batch_size=15000): 3,000-sample
  minibatches (6,000 actor rows, 3,000 critic rows);
* M = 4,096 / 8,192: a 4,096-maze rollout step (critic / actor trunk rows).

Per shape: forward with bias + ReLU (+ bits), the input-gradient form through
the ReLU bits (+ bias column sums) and the weight gradient.  HIP events, mean
of 20 launches after 5 warm-ups, one process.  Prints a markdown table.
"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "marl-maze_amd"))
from marlmaze import x3  # noqa: E402


def t(f, n=20):
    for _ in range(5):
        f()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        f()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


SHAPES = [("actor L0", 264, 460), ("actor L1/L2", 264, 264), ("heads", 6, 264), ("critic L0", 64, 130),
          ("critic L1", 64, 64), ("value", 1, 64)]
print("| M | layer (N x K) | fwd engine us | fwd lib us | dX engine us | dX lib us | dW engine us | dW lib us |")
print("|---|---|---|---|---|---|---|---|")
for M in (1, 2, 300, 3000, 4096, 6000, 8192, 16384):
    for name, N, K in SHAPES:
        g = torch.Generator(device="cuda").manual_seed(M + N + K)
        a = torch.randn(M, K, device="cuda", generator=g)
        w = torch.randn(N, K, device="cuda", generator=g) * 0.1
        b = torch.randn(N, device="cuda", generator=g)
        dy = torch.randn(M, N, device="cuda", generator=g)
        bits = x3.mbits(M, "cuda") if N <= 272 else None
        tw = x3.pack(w)
        tt = x3.pack(w, trans=True)
        fe = t(lambda: x3.gemm(a, tw, bias=b, relu=True, mbits_out=bits))
        fl = t(lambda: torch._addmm_activation(b, a, w.t()))
        # dX for this layer's input: dY [M, N] . W [N, K]; through the ReLU bits of a [M, K] layer when K <= 272
        xb = x3.mbits(M, "cuda")
        if K % 4 == 0 and K <= 272:
            x3.gemm(a, x3.pack(torch.randn(K, K, device="cuda") * 0.1), relu=True, mbits_out=xb)
        cs = x3.colsum_buf(M, K, "cuda")
        if N % 4 == 0:
            kw = dict(mbits_in=xb, colsum=cs) if K <= 272 and K % 4 == 0 else {}
            de = t(lambda: x3.gemm(dy, tt, **kw))
        else:
            de = float("nan")  # (dY of the heads / value head goes through mm_x3_heads_bwd)
        y = torch.relu(a)
        dl = t(lambda: torch.ops.aten.threshold_backward(dy.mm(w), y, 0))
        we = t(lambda: x3.wgrad(dy, a))
        wl = t(lambda: dy.t().mm(a))
        print(f"| {M} | {name} ({N} x {K}) | {fe:.1f} | {fl:.1f} | {de:.1f} | {dl:.1f} | {we:.1f} | {wl:.1f} |",
              flush=True)
