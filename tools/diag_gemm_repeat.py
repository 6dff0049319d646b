"""Repeat-launch determinism check of the forward / input-gradient GEMM kernels (k_bres, k_x3nt): the
kernels are deterministic, so every launch on the same inputs must give the first launch's output bit for
bit; a launch that differs is a corrupted one (the k_wgrad_rect failure mode, DESIGN.md section 4, showed
up this way in ~60% of its launches).  Prints the differing launches per case.

  python tools/diag_gemm_repeat.py            (REPS env, default 100; M env, default 419,430)
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "marl-maze_amd"))
import torch  # noqa: E402

from marlmaze import x3  # noqa: E402

reps = int(os.environ.get("REPS", 100))
M = int(os.environ.get("M", 419430))
shapes = [(264, 460), (264, 264), (6, 264), (64, 130), (460, 264)]
total_bad = 0
for prec in ("x2", "f16", "x3"):
    for algo in ("auto", "stream"):
        x3.set_algo(algo)
        for N, K in shapes:
            g = torch.Generator(device="cuda").manual_seed(N + K)
            a = torch.randn(M, K, device="cuda", generator=g)
            w = torch.randn(N, K, device="cuda", generator=g) * 0.1
            b = torch.randn(N, device="cuda", generator=g)
            bits = x3.mbits(M, "cuda") if N <= 272 else None
            wp = x3.pack(w, prec=prec)
            w2 = torch.randn(48, N, device="cuda", generator=g) * 0.1
            dy = torch.randn(M, 48, device="cuda", generator=g) / M
            ascale = 1.0 if prec == "x3" else float(2.0 ** int(torch.tensor(float(M)).log2().floor()))
            w2p = x3.pack(w2, trans=True, prec=prec)
            y0 = x3.gemm(a, wp, bias=b, relu=True, mbits_out=bits)
            dx0 = x3.gemm(dy, w2p, mbits_in=bits, ascale=ascale)
            bad_y = bad_dx = 0
            y = torch.empty_like(y0)
            dx = torch.empty_like(dx0)
            for r in range(reps):
                x3.gemm(a, wp, bias=b, relu=True, mbits_out=bits, out=y)
                x3.gemm(dy, w2p, mbits_in=bits, ascale=ascale, out=dx)
                by = int((y.view(torch.int32) != y0.view(torch.int32)).any().item())
                bd = int((dx.view(torch.int32) != dx0.view(torch.int32)).any().item())
                if by or bd:
                    print(f"  {prec} {algo} {N}x{K} launch {r}: forward differs {by}, input gradient differs {bd}",
                          flush=True)
                bad_y += by
                bad_dx += bd
            total_bad += bad_y + bad_dx
            print(f"{prec:4s} {algo:6s} M={M} N={N} K={K}: {reps} launches, forward differing {bad_y}, "
                  f"input gradient differing {bad_dx}", flush=True)
# the weight gradients (k_wgrad_rect for the update's shapes, the generic k_wgrad otherwise)
for prec in ("x2", "f16", "x3"):
    for N, K in shapes + [(48, 264), (264, 52)]:
        g = torch.Generator(device="cuda").manual_seed(7 * N + K)
        dy = torch.randn(M, N, device="cuda", generator=g) / M
        x = torch.randn(M, K, device="cuda", generator=g)
        s = 1.0 if prec == "x3" else float(2.0 ** int(torch.tensor(float(M)).log2().floor()))
        try:
            w0 = x3.wgrad(dy, x, prec=prec, dscale=s).clone()
        except Exception as e:  # a shape the weight gradient does not take (N > 272)
            print(f"{prec:4s} wgrad  M={M} N={N} K={K}: not run ({e})", flush=True)
            continue
        bad = 0
        for r in range(reps):
            w = x3.wgrad(dy, x, prec=prec, dscale=s)
            bad += int((w.view(torch.int32) != w0.view(torch.int32)).any().item())
        total_bad += bad
        print(f"{prec:4s} wgrad  M={M} N={N} K={K}: {reps} launches, differing {bad}", flush=True)
print(f"total differing launches: {total_bad}")
