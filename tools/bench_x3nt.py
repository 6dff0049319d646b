"""Microbench + accuracy check of the x3 GEMMs (mm_x3_nt / mm_x3_nt_f32a) on the MLP shapes.

python tools/bench_x3nt.py  -> one line per shape: us per launch and TFLOP/s (fp32-equivalent)
for A pre-split (TP) and A fp32 (split in the GEMM), with and without the fused ReLU-backward
mask, the torch fp32 GEMM of the same shape, and max |err| / sum|ab| vs fp64.
SHAPES=264x264,... selects shapes (N x K); M=... the row count.
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "marl-maze_amd"))
import torch  # noqa: E402

from marlmaze import x3  # noqa: E402


def timeit(fn, iters=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def main():
    torch.backends.cuda.matmul.allow_tf32 = False
    M = int(os.environ.get("M", 419430))
    g = torch.Generator(device="cuda").manual_seed(0)
    shapes = [(264, 264), (264, 460), (460, 264), (64, 64)]
    if os.environ.get("SHAPES"):
        shapes = [tuple(int(v) for v in t.split("x")) for t in os.environ["SHAPES"].split(",")]
    for N, K in shapes:
        a = torch.randn(M, K, device="cuda", generator=g)
        w = torch.randn(N, K, device="cuda", generator=g) * 0.05
        bias = torch.randn(N, device="cuda", generator=g)
        mask = torch.relu(torch.randn(M, N, device="cuda", generator=g))
        ta, tw = x3.pack(a), x3.pack(w)
        out = torch.empty(M, N, device="cuda")
        rows = torch.arange(0, M, 997, device="cuda")
        ref = torch.relu(a[rows].double() @ w.double().t() + bias.double())
        scale = a[rows].double().abs() @ w.double().abs().t() + bias.double().abs()
        errs = []
        for src in (ta, a):
            c, _ = x3.nt(src, tw, bias=bias, relu=True, out=out)
            errs.append(((c[rows].double() - ref).abs() / scale).max().item())
        c, _ = x3.nt(a, tw, bias=bias, relu=True, mask=mask, out=out)
        errs.append(((c[rows].double() - ref * (mask[rows] > 0)).abs() / scale).max().item())
        if N <= 272:  # ReLU bit masks: written by a relu GEMM, applied by a second GEMM of the same shape
            mb = x3.mbits(M, "cuda")
            y, _ = x3.nt(a, tw, bias=bias, relu=True, mbits_out=mb)
            c2, _ = x3.nt(a, tw, mbits_in=mb)
            ref2 = (a[rows].double() @ w.double().t()) * (y[rows] > 0)
            errs.append(((c2[rows].double() - ref2).abs() / scale).max().item())
        flop = 2.0 * M * N * K
        t_tp = timeit(lambda: x3.nt(ta, tw, bias=bias, relu=True, out=out))
        t_f32 = timeit(lambda: x3.nt(a, tw, bias=bias, relu=True, out=out))
        t_mask = timeit(lambda: x3.nt(a, tw, bias=bias, relu=True, mask=mask, out=out))
        line = (f"M={M} N={N} K={K}: A=TP {t_tp:6.1f}us {flop / t_tp / 1e6:5.1f} TF | A=f32 {t_f32:6.1f}us "
                f"{flop / t_f32 / 1e6:5.1f} TF | +mask {t_mask:6.1f}us")
        if N <= 272:
            t_bo = timeit(lambda: x3.nt(a, tw, bias=bias, relu=True, out=out, mbits_out=mb))
            t_bi = timeit(lambda: x3.nt(a, tw, out=out, mbits_in=mb))
            line += f" | bits out {t_bo:6.1f}us in {t_bi:6.1f}us"
        if not os.environ.get("ONLY_NT"):
            t_lib = timeit(lambda: torch.addmm(bias, a, w.t()))
            line += f" | lib fp32 {t_lib:6.1f}us {flop / t_lib / 1e6:5.1f} TF"
        print(line + " | err " + " ".join(f"{e:.1e}" for e in errs), flush=True)
        del a, w, ta, tw, out, mask


if __name__ == "__main__":
    main()
