"""Mechanism of a wrong weight-gradient partial (tools/diag_wgrad_race.py finds them): for each slice that
differs from the fp64 truth, express its error in the per-32-row-step contributions of dY and X (least
squares over candidate explanations: a step's contribution missing / doubled, a step's dY paired with
another step's X, ...)."""
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
s = float(2 ** int(torch.tensor(float(M)).log2().floor()))
S = L.mm_gemm_wgrad_slices(x3.PRECS[prec], M, N, K)
rows = (M + S - 1) // S
rows = (rows + 31) // 32 * 32
dyd, xd = dy.double(), x.double()
found = 0
for r in range(int(os.environ.get("REPS", 80))):
    ws = torch.full((S, N, K), float("nan"), device="cuda")
    _lib.check(L.mm_gemm_wgrad_partials(x3.PRECS[prec], _lib.ptr(dy), N, s, _lib.ptr(x), K, M, N, K, 1.0 / s,
                                        _lib.ptr(ws), _lib.stream_ptr()), "partials")
    torch.cuda.synchronize()
    for sl in range(S):
        m0, m1 = sl * rows, min(M, (sl + 1) * rows)
        truth = dyd[m0:m1].t() @ xd[m0:m1]
        err = ws[sl].double() - truth
        rel = err.abs().max().item() / truth.abs().max().item()
        if rel < 1e-4:
            continue
        found += 1
        steps = [(a, min(m1, a + 32)) for a in range(m0, m1, 32)]
        contrib = [dyd[a:b].t() @ xd[a:b] for a, b in steps]
        print(f"run {r} slice {sl}: rel err {rel:.3e}")
        bad = err.abs() > 1e-4 * truth.abs().max().item()
        print("   wrong (n, k):", bad.sum().item(), "rows n:", bad.any(1).nonzero().flatten().tolist(),
              "k-tiles:", sorted(set((bad.any(0).nonzero().flatten() // 16).tolist())))
        # stale 8-row chunk candidates: the piece (step i, chunk c) of dY or of X read from step i - 2
        for i in range(2, (m1 - m0 + 31) // 32):
            for c in range(4):
                a = m0 + 32 * i + 8 * c
                b = m0 + 32 * (i - 2) + 8 * c
                candA = dyd[b:b + 8].t() @ xd[a:a + 8] - dyd[a:a + 8].t() @ xd[a:a + 8]
                candB = dyd[a:a + 8].t() @ xd[b:b + 8] - dyd[a:a + 8].t() @ xd[a:a + 8]
                for nm, cd in (("dY", candA), ("X", candB)):
                    res = ((err - cd) * bad).abs().max().item() / err.abs().max().item()
                    if res < 0.3:
                        print(f"   err ~ stale {nm} chunk: step {i} chunk {c} holds step {i - 2}'s (residual {res:.3f})")
        for i, c in enumerate(contrib):  # err = alpha * step i's contribution?
            alpha = (err * c).sum().item() / (c * c).sum().item()
            res = (err - alpha * c).abs().max().item() / err.abs().max().item()
            if res < 0.2:
                print(f"   err ~ {alpha:+.3f} x step {i} contribution (residual {res:.3f})")
        for i in range(len(steps)):  # err = dY_step_i^T X_step_j - dY_i^T X_i ?
            for j in range(len(steps)):
                if i == j:
                    continue
                a, b = steps[i]
                c2, d2 = steps[j]
                if b - a != d2 - c2:
                    continue
                cand = dyd[a:b].t() @ xd[c2:d2] - contrib[i]
                res = (err - cand).abs().max().item() / err.abs().max().item()
                cand2 = dyd[c2:d2].t() @ xd[a:b] - contrib[i]
                res2 = (err - cand2).abs().max().item() / err.abs().max().item()
                if res < 0.2:
                    print(f"   err ~ dY(step {i}) with X(step {j}) (residual {res:.3f})")
                if res2 < 0.2:
                    print(f"   err ~ dY(step {j}) with X(step {i}) (residual {res2:.3f})")
    if found >= 4:
        break
print("bad slices found:", found)
