"""Where two runs of the same weight-gradient partials differ (mm_gemm_wgrad_partials, one process): per
row slice and per output element, for a shape given as PREC M N K (default x2 40000 6 264)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "marl-maze_amd"))
import torch  # noqa: E402

from marlmaze import _lib, x3  # noqa: E402

prec = sys.argv[1] if len(sys.argv) > 1 else "x2"
M, N, K = (int(v) for v in sys.argv[2:5]) if len(sys.argv) > 4 else (40000, 6, 264)
L = _lib.lib()
g = torch.Generator(device="cuda").manual_seed(1)
dy = torch.randn(M, N, device="cuda", generator=g) / M
x = torch.randn(M, K, device="cuda", generator=g)
s = float(2 ** int(torch.tensor(float(M)).log2().floor())) if prec != "x3" else 1.0
S = L.mm_gemm_wgrad_slices(x3.PRECS[prec], M, N, K)
runs = []
for r in range(int(os.environ.get("REPS", 12))):
    ws = torch.full((S, N, K), float("nan"), device="cuda")
    _lib.check(L.mm_gemm_wgrad_partials(x3.PRECS[prec], _lib.ptr(dy), N, s, _lib.ptr(x), K, M, N, K, 1.0 / s,
                                        _lib.ptr(ws), _lib.stream_ptr()), "partials")
    torch.cuda.synchronize()
    runs.append(ws)
ref = runs[0]
for r, ws in enumerate(runs[1:], 1):
    d = (ws != ref) & ~(torch.isnan(ws) & torch.isnan(ref))
    nan = torch.isnan(ws).sum().item()
    if d.any() or nan:
        sl = d.any(dim=(1, 2)).nonzero().flatten().tolist()
        el = d.any(dim=0).nonzero().tolist()
        print(f"run {r}: {d.sum().item()} differing values, nan {nan}, slices {sl[:20]}, (n, k) {el[:24]}")
    else:
        print(f"run {r}: identical")
print("slices", S, "nan in run 0:", torch.isnan(ref).sum().item())

# the full call (partials + k_wg_reduce) through x3.wgrad, repeated: outputs compared bitwise
outs = [x3.wgrad(dy, x, prec=prec, dscale=s) for _ in range(int(os.environ.get("REPS", 12)))]
torch.cuda.synchronize()
ref_full = runs[0].sum(0)  # (fp32 torch sum of the partials: a different order, for scale only)
for r, o in enumerate(outs):
    print(f"full run {r}: identical to run 0: {torch.equal(o, outs[0])}, max |diff| vs torch partial sum "
          f"{(o - ref_full).abs().max().item():.3e}")
# the same with a fresh workspace filled with NaN each time (mm_gemm_wgrad directly)
L2 = L
n = L2.mm_gemm_wgrad_ws_len(M, N, K)
for r in range(4):
    ws = torch.full((n,), float("nan"), device="cuda")
    o = torch.full((N, K), float("nan"), device="cuda")
    _lib.check(L2.mm_gemm_wgrad(x3.PRECS[prec], _lib.ptr(dy), N, s, _lib.ptr(x), K, M, N, K, 1.0 / s, _lib.ptr(ws),
                                _lib.ptr(o), _lib.stream_ptr()), "wgrad")
    torch.cuda.synchronize()
    print(f"nan-ws run {r}: nan in out {torch.isnan(o).sum().item()}, identical to run 0 {torch.equal(o, outs[0])}")
