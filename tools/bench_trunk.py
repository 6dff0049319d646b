"""Time the fused small-M trunk (mm_trunk3) against the three per-layer GEMMs it replaces, both captured
in a HIP graph (as the rollout runs them) and replayed back to back; HIP events around 200 replays.
MARLMAZE_TRUNK_D=1 times the form without weight prefetch beyond the next k-step.  Usage: python tools/bench_trunk.py [M ...] [--prec x2]"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "marl-maze_amd"))

import torch  # noqa: E402

from marlmaze import ops, x3  # noqa: E402


def graph_time(fn, reps=200):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(10):
            fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps // 10):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("M", nargs="*", type=int, default=[4096, 8192, 16384, 32768, 65536])
    ap.add_argument("--prec", default="x2")
    ap.add_argument("--heads", action="store_true", help="with the heads + action draws (mm_trunk3_head_sample "
                    "against the three GEMMs + ops.head_sample)")
    a = ap.parse_args()
    torch.manual_seed(0)
    ws = [torch.randn(264, 460, device="cuda") * 0.05, torch.randn(264, 264, device="cuda") * 0.06,
          torch.randn(264, 264, device="cuda") * 0.06]
    bs = [torch.randn(264, device="cuda") * 0.1 for _ in ws]
    packs = [x3.pack(w, prec=a.prec) for w in ws]
    res = []
    for M in a.M:
        h0 = torch.relu(torch.randn(M, 460, device="cuda"))
        out = torch.empty(M, 264, device="cuda")
        o1, o2, o3 = (torch.empty(M, 264, device="cuda") for _ in range(3))

        hw, hb = torch.randn(6, 264, device="cuda") * 0.2, torch.randn(6, device="cuda") * 0.1
        mk = (torch.rand(M, 6, device="cuda") < 0.6).to(torch.uint8)
        mk[:, 4] = 1
        act, lp, jl = (torch.empty((M, 2), dtype=torch.int8, device="cuda"), torch.empty(M, device="cuda"),
                       torch.empty((M + 1) // 2, device="cuda"))

        def fused():
            if a.heads:
                x3.trunk3_head_sample(h0, packs, bs, hw, hb, mk, 1, 0, act, lp, jl, h3=out)
            else:
                x3.trunk3(h0, packs, bs, out=out)

        def three():
            x3.gemm(h0, packs[0], bias=bs[0], relu=True, out=o1)
            x3.gemm(o1, packs[1], bias=bs[1], relu=True, out=o2)
            x3.gemm(o2, packs[2], bias=bs[2], relu=True, out=o3)
            if a.heads:
                ops.head_sample(o3, hw, hb, mk, 1, 0, actions=act, logp=lp, joint_logp=jl)

        tf, t3 = graph_time(fused), graph_time(three)
        fused()
        three()
        torch.cuda.synchronize()
        same = bool(torch.equal(out, o3))
        r = {"M": M, "prec": a.prec, "heads": a.heads, "depth": os.environ.get("MARLMAZE_TRUNK_D", "default"), "fused_us": round(tf, 2),
             "three_gemms_us": round(t3, 2), "speedup": round(t3 / tf, 3), "bit_identical": same}
        print(json.dumps(r), flush=True)
        res.append(r)


if __name__ == "__main__":
    main()
