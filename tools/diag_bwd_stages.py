"""Diagnostic: the actor MLP's explicit backward stage by stage (heads
backward, each input-gradient GEMM, each weight gradient and bias column sum)
against fp64 evaluated on the SAME saved activations and ReLU pattern, plus a
determinism check (the backward run twice)."""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "marl-maze_amd"))
from marlmaze import x3  # noqa: E402
from marlmaze.networks import Actor  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 6000
parity = (sys.argv[2] == "1") if len(sys.argv) > 2 else True


def rel(a, b):
    return ((a.double() - b).abs().max() / b.abs().max().clamp_min(1e-30)).item()


torch.manual_seed(0)
actor = Actor([264, 264, 264], parity_mode=parity).cuda()
x = torch.rand(B, 65, device="cuda") + 0.5 * torch.randn(B, 65, device="cuda")
dz = torch.randn(B, 6, device="cuda") / B
z, (xx, ws, hs, bits) = actor.train_forward(x)
torch.cuda.synchronize()
W = [lin.weight for lin in actor.layers]
wh, bh = actor.heads()
masks = [(h > 0) for h in hs[1:]]
# heads backward
dy, cs = x3.heads_bwd(dz, wh, bits[2])
ref = (dz.double() @ wh.double()) * masks[2]
print("heads dy", rel(dy, ref), "colsum", rel(x3.colsum(cs), ref.sum(0)))
dwh = x3.wgrad(dz, hs[3])
print("dWh", rel(dwh, dz.double().t() @ hs[3].double()))
dyr = ref
for l in (2, 1, 0):
    dw = x3.wgrad(dy, hs[l])
    print(f"L{l} dW", rel(dw, dy.double().t() @ hs[l].double()), "(vs chained fp64)", rel(dw, dyr.t() @ hs[l].double()))
    db = x3.colsum(cs)
    print(f"L{l} db", rel(db, dy.double().sum(0)))
    wt = x3.pack(W[l], trans=True)
    if l > 0:
        cs2 = x3.colsum_buf(B, W[l].shape[1], "cuda")
        dy2 = x3.gemm(dy, wt, mbits_in=bits[l - 1], colsum=cs2)
        r2 = (dy.double() @ W[l].double()) * masks[l - 1]
        print(f"L{l} dX(bits)", rel(dy2, r2), "colsum", rel(x3.colsum(cs2), r2.sum(0)))
        dyr = (dyr @ W[l].double()) * masks[l - 1]
        dy, cs = dy2, cs2
    else:
        dx = x3.gemm(dy, wt)
        print("L0 dX", rel(dx, dy.double() @ W[0].double()))
# determinism: the whole backward twice
g1, g2 = [], []
for out in (g1, g2):
    for p in actor.parameters():
        p.grad = torch.zeros_like(p)
    actor.train_backward((xx, ws, hs, bits), dz)
    torch.cuda.synchronize()
    out.extend(p.grad.clone() for p in actor.parameters())
print("deterministic:", all(torch.equal(a, b) for a, b in zip(g1, g2)))
