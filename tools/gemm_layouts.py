"""Which operand layout gives the fastest fp32 GEMM for the actor's MLP shapes
(M = 419,430 rows)?  Tunes each candidate with TunableOp (in-process), then
times it with HIP events."""
import json
import os
import sys

import torch

torch.cuda.tunable.enable(True)
torch.cuda.tunable.tuning_enable(True)
torch.cuda.tunable.set_filename(os.path.join(os.environ.get("TMPDIR", "/tmp"), "gemm_layouts_tune.csv"))
M = 419430
res = {}


def timeit(fn, n=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n


for K, N in ((460, 264), (264, 264)):
    x = torch.randn(M, K, device="cuda")
    W = torch.randn(N, K, device="cuda")
    b = torch.randn(N, device="cuda")
    Wt = W.t().contiguous()
    xt = x.t().contiguous()
    dy = torch.randn(M, N, device="cuda")
    fl = 2.0 * M * N * K
    cands = {
        "fwd addmm(b, x, W.t())": lambda: torch.addmm(b, x, W.t()),
        "fwd addmm(b, x, Wt)": lambda: torch.addmm(b, x, Wt),
        "fwd addmm_act(b, x, W.t())": lambda: torch._addmm_activation(b, x, W.t()),
        "fwd addmm_act(b, x, Wt)": lambda: torch._addmm_activation(b, x, Wt),
        "dX dy @ W": lambda: dy.mm(W),
        "dW dy.t() @ x": lambda: dy.t().mm(x),
        "dW bmm16": lambda: torch.bmm(dy.view(16, M // 16 if M % 16 == 0 else 0, N).transpose(1, 2),
                                      x.view(16, -1, K)).sum(0) if M % 16 == 0 else None,
    }
    for name, fn in cands.items():
        if fn() is None:
            continue
        ms = timeit(fn)
        res[f"K{K} N{N} {name}"] = {"ms": round(ms, 4), "TFLOPs": round(fl / ms / 1e9, 1)}
        print(name, K, N, res[f"K{K} N{N} {name}"], flush=True)
print(json.dumps(res))
