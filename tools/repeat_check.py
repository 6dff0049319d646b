"""Run-to-run determinism check of single GEMM calls across library builds (in one process): each case is
run REPS times per library; prints the error against fp64 and whether every repeat was bitwise identical.

  LIBS=tools/_var/base.so,marl-maze_amd/libmarlmaze.so python tools/repeat_check.py
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "marl-maze_amd"))
import torch  # noqa: E402

from marlmaze import _lib, x3  # noqa: E402


def load(path):
    _lib.LIB_PATH = path
    _lib._LIB = None
    return _lib.lib()


def rel(a, ref, scale):
    return ((a.double() - ref).abs() / scale.clamp_min(1e-300)).max().item()


def cases():
    g = torch.Generator(device="cuda").manual_seed(40270)
    M, N, K = 40000, 6, 264
    dy = torch.randn(M, N, device="cuda", generator=g) / M
    x = torch.randn(M, K, device="cuda", generator=g)
    s = float(2 ** 15)
    ref = dy.double().t().mm(x.double())
    sc = dy.double().abs().t().mm(x.double().abs())
    yield "wgrad x2 40000x6x264", (lambda: x3.wgrad(dy, x, prec="x2", dscale=s)), ref, sc
    for prec, M, N, K in (("x2", 419430, 264, 264), ("x2", 209715, 64, 130), ("f16", 100000, 264, 264)):
        a = torch.randn(M, K, device="cuda", generator=g)
        w = torch.randn(N, K, device="cuda", generator=g) * 0.05
        b = torch.randn(N, device="cuda", generator=g)
        ref2 = (a.double() @ w.double().t() + b.double()).clamp_min(0)
        sc2 = a.double().abs() @ w.double().abs().t() + b.double().abs()
        yield (f"gemm {prec} fwd {M}x{N}x{K}",
               (lambda a=a, w=w, b=b, p=prec: x3.gemm(a, x3.pack(w, prec=p), bias=b, relu=True)), ref2, sc2)
    from marlmaze.networks import _heads_fwd
    h = torch.randn(419430, 264, device="cuda", generator=g).clamp_min(0)
    wh = torch.randn(6, 264, device="cuda", generator=g) * 0.01
    bh = torch.randn(6, device="cuda", generator=g)
    yield "heads_fwd 419430x264", (lambda: _heads_fwd(h, wh, bh)), h.double() @ wh.double().t() + bh.double(), \
        h.double().abs() @ wh.double().abs().t() + bh.double().abs()
    for prec in ("f16", "x2"):
        M, N, K = 40000, 460, 264
        a = torch.randn(M, K, device="cuda", generator=g)
        w = torch.randn(N, K, device="cuda", generator=g) * 0.05
        ref2 = a.double() @ w.double().t()
        sc2 = a.double().abs() @ w.double().abs().t()
        yield f"gemm {prec} plain 40000x460x264", (lambda a=a, w=w, p=prec: x3.gemm(a, x3.pack(w, prec=p))), ref2, sc2


def main():
    libs = os.environ.get("LIBS", "tools/_var/base.so,marl-maze_amd/libmarlmaze.so").split(",")
    reps = int(os.environ.get("REPS", 30))
    for path in libs:
        load(os.path.join(REPO, path) if not os.path.isabs(path) else path)
        for name, fn, ref, sc in cases():
            outs = [fn().clone() for _ in range(reps)]
            torch.cuda.synchronize()
            same = all(torch.equal(outs[0], o) for o in outs[1:])
            errs = [rel(o, ref, sc) for o in outs]
            print(f"{os.path.basename(path):16s} {name:28s} max err {max(errs):.3e} min err {min(errs):.3e} "
                  f"identical repeats {same}", flush=True)


if __name__ == "__main__":
    main()
