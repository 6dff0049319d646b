"""A/B timing of the two forward-GEMM kernels (mm_gemm_nt_algo: "auto" = B-resident k_bres where it
fits, "stream" = k_x3nt) in ONE process, alternating, median of REPS rounds of 10 launches each.

python tools/bench_gemm_ab.py      CASES="x3:fwd:264x264,f16:bwd:264x264,..." (prec:form:NxK), M=rows
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "marl-maze_amd"))
import torch  # noqa: E402

from marlmaze import x3  # noqa: E402

DEFAULT = ("x3:fwd:264x264,x3:bwd:264x264,x3:fwd:264x460,x3:plain:460x264,x3:fwd:6x264,x3:fwd:64x64,"
           "x3:fwd:64x130,f16:fwd:264x264,f16:bwd:264x264,f16:fwd:264x460,f16:plain:460x264,f16:fwd:6x264,"
           "f16:fwd:64x64,f16:fwd:64x130")


def case(prec, form, N, K, M, g):
    a = torch.randn(M, K, device="cuda", generator=g)
    w = x3.pack(torch.randn(N, K, device="cuda", generator=g) * 0.05, prec=prec)
    bias = torch.randn(N, device="cuda", generator=g)
    out = torch.empty(M, N, device="cuda")
    mb = x3.mbits(M, "cuda")
    cs = x3.colsum_buf(M, N, "cuda")
    if form == "bwd":
        x3.gemm(a, w, bias=bias, relu=True, mbits_out=mb, out=out)
        return lambda: x3.gemm(a, w, mbits_in=mb, colsum=cs, out=out)
    if form == "fwd" and N <= 272:
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
    for c in os.environ.get("CASES", DEFAULT).split(","):
        prec, form, shape = c.split(":")
        N, K = (int(v) for v in shape.split("x"))
        fn = case(prec, form, N, K, M, g)
        t = {"auto": [], "stream": []}
        for algo in ("auto", "stream"):
            x3.set_algo(algo)
            fn()
        torch.cuda.synchronize()
        for _ in range(reps):
            for algo in ("auto", "stream"):
                x3.set_algo(algo)
                t[algo].append(timed(fn))
        x3.set_algo("auto")
        med = {k: sorted(v)[len(v) // 2] for k, v in t.items()}
        print(f"{prec:3s} {form:5s} M={M} N={N:3d} K={K:3d}: auto {med['auto']:7.1f} us  stream {med['stream']:7.1f} us"
              f"  ratio {med['auto'] / med['stream']:.3f}", flush=True)
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
