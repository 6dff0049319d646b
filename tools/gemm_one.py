"""One actor-trunk GEMM shape launched repeatedly (for rocprofv3 --pmc passes).

SHAPE=NxK (default 264x264), M rows (default 419,430), PREC=x3|x2|f16, FORM=fwd (bias + ReLU +
bits out) | bwd (bits in + column sums) | plain | wgrad (dW [N, K] = dY^T X, dY [M, N], X [M, K]);
MARLMAZE_GEMM_BRES=0 selects k_x3nt.
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "marl-maze_amd"))
import torch  # noqa: E402

from marlmaze import x3  # noqa: E402


def main():
    N, K = (int(v) for v in os.environ.get("SHAPE", "264x264").split("x"))
    M = int(os.environ.get("M", 419430))
    prec = os.environ.get("PREC", "x3")
    form = os.environ.get("FORM", "fwd")
    g = torch.Generator(device="cuda").manual_seed(0)
    a = torch.randn(M, K, device="cuda", generator=g)
    w = x3.pack(torch.randn(N, K, device="cuda", generator=g) * 0.05, prec=prec)
    bias = torch.randn(N, device="cuda", generator=g)
    out = torch.empty(M, N, device="cuda")
    mb = x3.mbits(M, "cuda")
    if N <= 272:
        x3.gemm(a, w, bias=bias, relu=True, mbits_out=mb, out=out)
    cs = x3.colsum_buf(M, N, "cuda")
    ascale = 1.0

    if form == "wgrad":
        dy = torch.randn(M, N, device="cuda", generator=g) / M
        dsc = 1.0 if prec == "x3" else float(2.0 ** int(torch.tensor(float(M)).log2().floor()))

    def one():
        if form == "wgrad":
            x3.wgrad(dy, a, prec=prec, dscale=dsc)
        elif form == "fwd":
            x3.gemm(a, w, bias=bias, relu=True, mbits_out=mb, out=out)
        elif form == "bwd":
            x3.gemm(a, w, mbits_in=mb, colsum=cs, ascale=ascale, out=out)
        else:
            x3.gemm(a, w, out=out)

    for _ in range(int(os.environ.get("ITERS", 20))):
        one()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        one()
    e1.record()
    torch.cuda.synchronize()
    print(f"{prec} {form} M={M} N={N} K={K}: {e0.elapsed_time(e1) / 20 * 1e3:.1f} us", flush=True)


if __name__ == "__main__":
    main()
