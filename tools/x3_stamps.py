"""Phase clocks of k_x3nt from an X3_STAMPS diagnostic build (tools/x3_stamps.sh).

MARLMAZE_LIB=tools/_var/x3_STAMPS.so python tools/x3_stamps.py
One forward GEMM (bias + ReLU + bits, the bench's EM_FWD form) per shape, after
warm-up launches; per wave and unit: prologue (B stage 0 DMA + first A load +
barrier), main loop (all k-steps), epilogue (stores + barrier), in shader
cycles, and the clock from s_memtime / s_memrealtime (100 MHz).
SHAPES=264x264,... (N x K), M=... rows.
"""
import ctypes
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "marl-maze_amd"))
import torch  # noqa: E402

from marlmaze import _lib, x3  # noqa: E402

WAVES, SLOTS = 16, 8


def main():
    lib = _lib.lib()
    lib.mm_x3_stamps_read.argtypes = [ctypes.c_void_p, ctypes.c_long]
    M = int(os.environ.get("M", 419430))
    shapes = [(264, 264), (264, 460), (460, 264)]
    if os.environ.get("SHAPES"):
        shapes = [tuple(int(v) for v in t.split("x")) for t in os.environ["SHAPES"].split(",")]
    g = torch.Generator(device="cuda").manual_seed(0)
    for N, K in shapes:
        a = torch.randn(M, K, device="cuda", generator=g)
        w = x3.pack(torch.randn(N, K, device="cuda", generator=g) * 0.05)
        bias = torch.randn(N, device="cuda", generator=g)
        mb = x3.mbits(M, "cuda") if N <= 272 else None
        out = torch.empty(M, N, device="cuda")
        for _ in range(30):
            x3.gemm(a, w, bias=bias, relu=True, mbits_out=mb, out=out)
        torch.cuda.synchronize()
        lib.mm_x3_stamps_clear()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        x3.gemm(a, w, bias=bias, relu=True, mbits_out=mb, out=out)
        e1.record()
        torch.cuda.synchronize()
        n = 256 * 16 * WAVES * SLOTS
        buf = np.zeros(n, dtype=np.uint64)
        assert lib.mm_x3_stamps_read(buf.ctypes.data, n) == 0
        s = buf.reshape(256, 16, WAVES, SLOTS).astype(np.int64)
        ok = s[..., 0] != 0
        pro = (s[..., 1] - s[..., 0])[ok]
        loop = (s[..., 2] - s[..., 1])[ok]
        epi = (s[..., 3] - s[..., 2])[ok]
        unit = (s[..., 3] - s[..., 0])[ok]
        rt = (s[..., 5] - s[..., 4])[ok]
        clk = unit.sum() / (rt.sum() / 100e6) / 1e9
        # gaps between units of one wave (the persistent loop's own overhead)
        per_wg = ok[:, :, 0].sum(1)
        nks = (K + 31) // 32
        nt = 17 if N <= 272 else 15
        ideal = 6 * nt * nks * 16 * 4  # MFMA cycles per SIMD per unit (4 waves per SIMD, 16 cyc each)
        print(f"N={N} K={K} M={M}: {e0.elapsed_time(e1) * 1e3:.1f} us, units per WG {per_wg.min()}-{per_wg.max()}, "
              f"clock {clk:.2f} GHz")
        for name, v in (("prologue", pro), ("main loop", loop), ("epilogue", epi), ("unit", unit)):
            print(f"  {name:9s} mean {v.mean():8.0f} cyc  median {np.median(v):8.0f}  p10 {np.percentile(v, 10):8.0f}"
                  f"  p90 {np.percentile(v, 90):8.0f}")
        print(f"  main loop per k-step {loop.mean() / nks:.0f} cyc; MFMA-bound unit {ideal} cyc "
              f"({ideal / nks:.0f} per k-step)")
        del a, w, out, mb


if __name__ == "__main__":
    main()
