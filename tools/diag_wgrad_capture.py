"""Capture wrong weight-gradient partials for offline analysis (tools/diag_wgrad_fit.py): runs
mm_gemm_wgrad_partials REPS times on one seeded input (one process, one stream) and saves every row slice
whose partial differs from its fp64 truth by more than 1e-5 of the slice's max, together with that slice's
dY and X rows, into gpurun_out/r05/capture_<prec>_<M>x<N>x<K>.npz.

  python tools/diag_wgrad_capture.py PREC M N K   (REPS env, default 100; MARLMAZE_LIB picks a variant build)
"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "marl-maze_amd"))
import torch  # noqa: E402

from marlmaze import _lib, x3  # noqa: E402

prec = sys.argv[1] if len(sys.argv) > 1 else "x2"
M, N, K = (int(v) for v in sys.argv[2:5]) if len(sys.argv) > 4 else (40000, 6, 264)
reps = int(os.environ.get("REPS", 100))
L = _lib.lib()
g = torch.Generator(device="cuda").manual_seed(1)
dy = torch.randn(M, N, device="cuda", generator=g) / M
x = torch.randn(M, K, device="cuda", generator=g)
s = float(2 ** int(torch.tensor(float(M)).log2().floor())) if prec != "x3" else 1.0
S = L.mm_gemm_wgrad_slices(x3.PRECS[prec], M, N, K)
rows = ((M + S - 1) // S + 31) // 32 * 32
truth = torch.stack([dy[i * rows:(i + 1) * rows].double().t() @ x[i * rows:(i + 1) * rows].double()
                     for i in range(S)])
tmax = truth.abs().amax(dim=(1, 2)).clamp_min(1e-300)
bad_run, bad_slice, bad_part = [], [], []
first = None
for r in range(reps):
    ws = torch.full((S, N, K), float("nan"), device="cuda")
    _lib.check(L.mm_gemm_wgrad_partials(x3.PRECS[prec], _lib.ptr(dy), N, s, _lib.ptr(x), K, M, N, K, 1.0 / s,
                                        _lib.ptr(ws), _lib.stream_ptr()), "partials")
    torch.cuda.synchronize()
    rel = ((ws.double() - truth).abs().amax(dim=(1, 2)) / tmax)
    rel = torch.nan_to_num(rel, nan=1e30)
    if first is None:
        first = ws.clone()
    for sl in (rel > 1e-5).nonzero().flatten().tolist():
        bad_run.append(r)
        bad_slice.append(sl)
        bad_part.append(ws[sl].cpu().numpy())
        print(f"run {r} slice {sl}: rel err {rel[sl].item():.3e}", flush=True)
    if r % 20 == 19:
        print(f"{r + 1} runs, {len(bad_run)} bad slices so far", flush=True)
nbad = len(bad_run)
os.makedirs(os.path.join(REPO, "gpurun_out", "r05"), exist_ok=True)
out = os.path.join(REPO, "gpurun_out", "r05", f"capture_{prec}_{M}x{N}x{K}.npz")
sl_set = sorted(set(bad_slice))[:int(os.environ.get("KEEP", 30))]  # the rows of at most KEEP slices are saved
keep = [k for k, sl in enumerate(bad_slice) if sl in sl_set]
bad_run, bad_slice, bad_part = ([v[k] for k in keep] for v in (bad_run, bad_slice, bad_part))
np.savez_compressed(
    out, prec=prec, M=M, N=N, K=K, rows=rows, S=S, dscale=s, bad_run=np.array(bad_run, dtype=np.int64),
    bad_slice=np.array(bad_slice, dtype=np.int64),
    bad_part=np.array(bad_part, dtype=np.float32).reshape(-1, N, K),
    slices=np.array(sl_set, dtype=np.int64),
    dy_rows=np.array([dy[i * rows:(i + 1) * rows].cpu().numpy() for i in sl_set], dtype=np.float32).reshape(
        -1, rows, N),
    x_rows=np.array([x[i * rows:(i + 1) * rows].cpu().numpy() for i in sl_set], dtype=np.float32).reshape(
        -1, rows, K),
    good_part=np.array([first[i].cpu().numpy() for i in sl_set], dtype=np.float32).reshape(-1, N, K))
print(f"{reps} runs, {nbad} bad slices -> {out} ({len(keep)} kept)")
