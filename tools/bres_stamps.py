"""Phase clocks of k_bres from an X3_STAMPS build (tools/x3_stamps.sh builds tools/_var/x3_STAMPS.so).

MARLMAZE_LIB=tools/_var/x3_STAMPS.so PREC=x3 SHAPE=264x264 python tools/bres_stamps.py
Per wave: the B-block load (start -> barrier), the unit loop, per-unit times; clock from
s_memtime / s_memrealtime.
"""
import ctypes
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "marl-maze_amd"))
import torch  # noqa: E402

from marlmaze import _lib, x3  # noqa: E402


def main():
    lib = _lib.lib()
    lib.mm_x3_stamps_read.argtypes = [ctypes.c_void_p, ctypes.c_long]
    N, K = (int(v) for v in os.environ.get("SHAPE", "264x264").split("x"))
    M = int(os.environ.get("M", 419430))
    prec = os.environ.get("PREC", "x3")
    g = torch.Generator(device="cuda").manual_seed(0)
    a = torch.randn(M, K, device="cuda", generator=g)
    w = x3.pack(torch.randn(N, K, device="cuda", generator=g) * 0.05, prec=prec)
    bias = torch.randn(N, device="cuda", generator=g)
    mb = x3.mbits(M, "cuda")
    out = torch.empty(M, N, device="cuda")
    for _ in range(20):
        x3.gemm(a, w, bias=bias, relu=True, mbits_out=mb, out=out)
    torch.cuda.synchronize()
    lib.mm_x3_stamps_clear()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    x3.gemm(a, w, bias=bias, relu=True, mbits_out=mb, out=out)
    e1.record()
    torch.cuda.synchronize()
    n = 256 * 16 * 16 * 8
    buf = np.zeros(n, dtype=np.uint64)
    assert lib.mm_x3_stamps_read(buf.ctypes.data, n) == 0
    s = buf.reshape(256, 16, 16, 8).astype(np.int64)
    st = s[:, 0, :, 0]
    ok = (st != 0) & (s[:, 0, :, 3] != 0)
    load = (s[:, 0, :, 1] - st)[ok]
    loop = (s[:, 0, :, 3] - s[:, 0, :, 1])[ok]
    clk = (s[:, 0, :, 3] - st)[ok].sum() / ((s[:, 0, :, 5] - s[:, 0, :, 4])[ok].sum() / 100e6) / 1e9
    t0 = st[ok].min()
    ends = s[:, 0, :, 3][ok] - t0
    starts = st[ok] - t0
    print(f"{prec} N={N} K={K} M={M}: {e0.elapsed_time(e1) * 1e3:.1f} us, clock {clk:.2f} GHz, "
          f"waves {ok.sum()}")
    print(f"  start spread  median {np.median(starts):8.0f}  max {starts.max():8.0f} cyc")
    print(f"  B load       mean {load.mean():8.0f}  median {np.median(load):8.0f}  p90 {np.percentile(load, 90):8.0f}")
    print(f"  unit loop    mean {loop.mean():8.0f}  median {np.median(loop):8.0f}  p90 {np.percentile(loop, 90):8.0f}")
    print(f"  wave end     median {np.median(ends):8.0f}  max {ends.max():8.0f}")
    units = []
    for b in range(256):
        for w in range(16):
            if not ok[b, w]:
                continue
            prev = s[b, 0, w, 1]
            for it in range(1, 16):
                e = s[b, it, w, 2]
                if e == 0:
                    break
                units.append(e - prev)
                prev = e
    units = np.array(units)
    print(f"  per unit     mean {units.mean():8.0f}  median {np.median(units):8.0f}  p10 {np.percentile(units, 10):8.0f}"
          f"  p90 {np.percentile(units, 90):8.0f}  (n={len(units)})")


if __name__ == "__main__":
    main()
