"""Phase clocks of the fused trunk kernel (k_trunk3) from the X3_STAMPS diagnostic build
(bash tools/x3_stamps.sh, then on the GPU box: MARLMAZE_LIB=tools/_var/x3_STAMPS.so python tools/trunk_stamps.py).
Per workgroup and wave (s_memtime cycles): staging, then per layer the k-loop and the epilogue + barrier;
the span of the launch from the s_memrealtime stamps (100 MHz)."""
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "marl-maze_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from marlmaze import _lib, x3  # noqa: E402

W = 8


def main():
    M = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
    prec = sys.argv[2] if len(sys.argv) > 2 else "x2"
    torch.manual_seed(0)
    ws = [torch.randn(264, 460, device="cuda") * 0.05, torch.randn(264, 264, device="cuda") * 0.06,
          torch.randn(264, 264, device="cuda") * 0.06]
    bs = [torch.randn(264, device="cuda") * 0.1 for _ in ws]
    packs = [x3.pack(w, prec=prec) for w in ws]
    h0 = torch.relu(torch.randn(M, 460, device="cuda"))
    for _ in range(20):
        y = x3.trunk3(h0, packs, bs)
    torch.cuda.synchronize()
    L = _lib.lib()
    L.mm_trunk_stamps_read.argtypes = [ctypes.c_void_p, ctypes.c_long]
    L.mm_x3_stamps_clear()
    y = x3.trunk3(h0, packs, bs)
    torch.cuda.synchronize()
    n = 1024 * W * 10
    buf = (ctypes.c_ulonglong * n)()
    assert L.mm_trunk_stamps_read(buf, n) == 0
    st = np.frombuffer(buf, dtype=np.uint64).reshape(1024, W, 10).astype(np.int64)
    nwg = (M + 31) // 32
    st = st[:nwg]
    names = ["staging", "L0 loop", "L0 epi+bar", "L1 loop", "L1 epi+bar", "L2 loop", "L2 epi"]
    d = np.diff(st[:, :, :8], axis=2)
    res = {"M": M, "prec": prec, "workgroups": nwg}
    for i, nm in enumerate(names):
        res[nm + " cycles (median wave)"] = float(np.median(d[:, :, i]))
        res[nm + " cycles (max wave, median wg)"] = float(np.median(d[:, :, i].max(axis=1)))
    res["total cycles (median wg)"] = float(np.median(st[:, :, 7].max(axis=1) - st[:, :, 0].min(axis=1)))
    rt = st[:, :, 8:10]
    res["span_us (first start to last end, memrealtime)"] = float((rt[:, :, 1].max() - rt[:, :, 0].min()) / 100.0)
    res["start spread us"] = float((rt[:, :, 0].max() - rt[:, :, 0].min()) / 100.0)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
