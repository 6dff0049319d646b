"""In-process A/B timing of library builds (tools/ab_build.py) on the update's kernels, alternating
builds, median of REPS rounds of 10 launches each (HIP events):

  LIBS=tools/_var/base.so,marl-maze_amd/libmarlmaze.so CASES=... python tools/ab_libs.py

CASES (comma-separated; M = rows, default 419,430):
  gemm:PREC:FORM:NxK[:ALGO]   FORM fwd (bias+ReLU+bits), bwd (through bits + column sums), plain; ALGO auto
                       (default) or stream (x3.set_algo)
  wgrad:PREC:NxK       dW = dY^T X
  front:fwd / front:bwd  the fused actor front-end (M samples)
"""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "marl-maze_amd"))
import torch  # noqa: E402

from marlmaze import _lib, x3  # noqa: E402

DEFAULT = ("gemm:x3:fwd:264x264,gemm:x3:bwd:264x264,gemm:x3:plain:460x264,gemm:x3:fwd:264x460,"
           "wgrad:x3:264x264,wgrad:x3:264x460,front:fwd,front:bwd")


def load(path):
    _lib.LIB_PATH = path
    _lib._LIB = None
    return _lib.lib()


def make(c, M, g):
    parts = c.split(":")
    if parts[0] == "gemm":
        prec, form, shape = parts[1:4]
        N, K = (int(v) for v in shape.split("x"))
        if len(parts) > 4:  # gemm:PREC:FORM:NxK:ALGO -- x3.set_algo (auto / stream) around each call
            fn, algo = make(":".join(parts[:4]), M, g), parts[4]

            def run():
                prev = x3.set_algo(algo)
                fn()
                x3.set_algo(prev)
            return run
        a = torch.randn(M, K, device="cuda", generator=g)
        wf = torch.randn(N, K, device="cuda", generator=g) * 0.05
        bias = torch.randn(N, device="cuda", generator=g)
        out = torch.empty(M, N, device="cuda")
        mb = x3.mbits(M, "cuda")
        cs = x3.colsum_buf(M, N, "cuda")
        if form == "bwd":
            x3.gemm(a, x3.pack(wf, prec=prec), bias=bias, relu=True, mbits_out=mb, out=out)
            return lambda: x3.gemm(a, x3.pack(wf, prec=prec), mbits_in=mb, colsum=cs, out=out)
        if form == "fwd":
            return lambda: x3.gemm(a, x3.pack(wf, prec=prec), bias=bias, relu=True, mbits_out=mb, out=out)
        return lambda: x3.gemm(a, x3.pack(wf, prec=prec), bias=bias, out=out)
    if parts[0] == "wgrad":
        prec, shape = parts[1:]
        N, K = (int(v) for v in shape.split("x"))
        dy = torch.randn(M, N, device="cuda", generator=g)
        xx = torch.randn(M, K, device="cuda", generator=g)
        out = torch.empty(N, K, device="cuda")
        return lambda: x3.wgrad(dy, xx, prec=prec, out=out)
    if parts[0] == "front":
        from marlmaze.networks import Actor, _front_bwd_to, _front_fwd, front_params

        torch.manual_seed(0)
        actor = Actor([264, 264, 264]).cuda()
        params = front_params(actor.projection, actor.attention)
        x = torch.rand(M, 65, device="cuda", generator=g)
        dh = torch.randn(M, 460, device="cuda", generator=g) / M
        grads = [torch.empty_like(p) for p in params]
        if parts[1] == "fwd":
            return lambda: _front_fwd(x, True, params)
        ws, _ = _front_fwd(x, True, params)
        return lambda: _front_bwd_to(ws, x, True, dh, grads)
    raise ValueError(c)


def timed(fn, n=10):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


def main():
    libs = os.environ.get("LIBS", "tools/_var/base.so,marl-maze_amd/libmarlmaze.so").split(",")
    Ls = [load(os.path.join(REPO, p) if not os.path.isabs(p) else p) for p in libs]
    M = int(os.environ.get("M", 419430))
    reps = int(os.environ.get("REPS", 5))
    g = torch.Generator(device="cuda").manual_seed(0)
    for c in os.environ.get("CASES", DEFAULT).split(","):
        fns = []
        for L in Ls:
            _lib._LIB = L
            fns.append(make(c, M, g))
            fns[-1]()
        torch.cuda.synchronize()
        t = [[] for _ in Ls]
        for _ in range(reps):
            for k, L in enumerate(Ls):
                _lib._LIB = L
                t[k].append(timed(fns[k]))
        med = [sorted(v)[len(v) // 2] for v in t]
        print(f"{c:24s} M={M}: " + "  ".join(f"{os.path.basename(p)} {m:8.1f} us" for p, m in zip(libs, med)) +
              f"  ratio {med[-1] / med[0]:.3f}", flush=True)
        del fns
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
