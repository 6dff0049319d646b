"""A/B timing of the fp32-class GEMM arithmetics, x3 (three bf16 planes, six MFMAs per product) against x2
(two fp16 planes, three MFMAs), at the update's shapes, in ONE process, alternating, median of REPS rounds
of 10 launches (HIP events).

python tools/bench_prec.py        M=rows (default 419,430: one update minibatch of actor rows)
"""
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "marl-maze_amd"))
import torch  # noqa: E402

from marlmaze import x3  # noqa: E402

# (form, N, K): fwd = bias + ReLU + bits, bwd = input gradient through bits + column sums, plain = no bits,
# wgrad = dW [N, K] = dY^T X
CASES = [("fwd", 264, 460), ("fwd", 264, 264), ("bwd", 264, 264), ("plain", 460, 264), ("wgrad", 264, 264),
         ("wgrad", 264, 460), ("wgrad", 6, 264), ("fwd", 64, 130), ("wgrad", 64, 130)]


def case(prec, form, N, K, M, g):
    s = 1.0 if prec == "x3" else float(2 ** 18)
    if form == "wgrad":
        dy = torch.randn(M, N, device="cuda", generator=g) / s
        x = torch.randn(M, K, device="cuda", generator=g)
        out = torch.empty(N, K, device="cuda")
        return lambda: x3.wgrad(dy, x, prec=prec, dscale=s, out=out)
    a = torch.randn(M, K, device="cuda", generator=g)
    w = x3.pack(torch.randn(N, K, device="cuda", generator=g) * 0.05, prec=prec)
    bias = torch.randn(N, device="cuda", generator=g)
    out = torch.empty(M, N, device="cuda")
    mb = x3.mbits(M, "cuda")
    cs = x3.colsum_buf(M, N, "cuda")
    if form == "bwd":
        x3.gemm(a, w, bias=bias, relu=True, mbits_out=mb, out=out)
        return lambda: x3.gemm(a, w, mbits_in=mb, colsum=cs, out=out)
    if form == "fwd":
        return lambda: x3.gemm(a, w, bias=bias, relu=True, mbits_out=mb, out=out)
    return lambda: x3.gemm(a, w, bias=bias, out=out)


def timed(fn, n=10):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


def main():
    M = int(os.environ.get("M", 419430))
    reps = int(os.environ.get("REPS", 5))
    g = torch.Generator(device="cuda").manual_seed(0)
    print(f"M = {M}: median us of {reps} x 10 launches; x2 / x3")
    tot = {"x3": 0.0, "x2": 0.0}
    for form, N, K in CASES:
        fns = {p: case(p, form, N, K, M, g) for p in ("x3", "x2")}
        t = {p: [] for p in fns}
        for p in fns:
            fns[p]()
        torch.cuda.synchronize()
        for _ in range(reps):
            for p in fns:
                t[p].append(timed(fns[p]))
        med = {p: statistics.median(v) for p, v in t.items()}
        for p in med:
            tot[p] += med[p]
        fl = 2.0 * M * N * K
        print(f"{form:5s} {N:3d} x {K:3d}: x3 {med['x3']:8.1f} us  x2 {med['x2']:8.1f} us  ratio "
              f"{med['x2'] / med['x3']:.3f}   (x2 {fl / med['x2'] / 1e6:6.1f} TFLOP/s fp32-class)", flush=True)
        del fns
        torch.cuda.empty_cache()
    print(f"sum: x3 {tot['x3']:.1f} us  x2 {tot['x2']:.1f} us  ratio {tot['x2'] / tot['x3']:.3f}")


if __name__ == "__main__":
    main()
