"""Diagnostic: signed (systematic) error of the x3 GEMM vs the fp32 library GEMM,
against fp64.  Positive operands make a truncating accumulation show up as a
negative mean error.  Usage: python tools/diag_x3_bias.py"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "marl-maze_amd"))
import torch  # noqa: E402

from marlmaze import x3  # noqa: E402

torch.backends.cuda.matmul.allow_tf32 = False
g = torch.Generator(device="cuda").manual_seed(0)
for sign in ("pos", "mixed"):
    for K in (32, 264, 460):
        M, N = 65536, 264
        a = torch.rand(M, K, device="cuda", generator=g)
        w = torch.rand(N, K, device="cuda", generator=g)
        if sign == "mixed":
            a = a * 2 - 1
            w = w * 2 - 1
        ref = a.double() @ w.double().t()
        scale = a.double().abs() @ w.double().abs().t()
        c3, _ = x3.nt(a, x3.pack(w))
        cl = a @ w.t()
        for nm, c in (("x3", c3), ("lib", cl)):
            e = (c.double() - ref) / scale
            print(f"{sign:5s} K={K:3d} {nm:3s} mean(err)/eps={e.mean().item() / 2**-24:+8.3f} "
                  f"rms/eps={e.pow(2).mean().sqrt().item() / 2**-24:7.3f} max/eps={e.abs().max().item() / 2**-24:7.3f}")
