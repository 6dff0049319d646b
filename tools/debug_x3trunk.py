"""Per-tensor error of the actor trunk (x3 GEMMs vs library fp32) against an fp64 reference."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "marl-maze_amd"))
import torch  # noqa: E402

from marlmaze.networks import Actor  # noqa: E402

torch.manual_seed(1)
actor = Actor([264, 264, 264]).cuda()
M = int(os.environ.get("M", 40000))
x = torch.randn(M, 65, device="cuda")
dh = torch.randn(M, 264, device="cuda")
res = {}
for mode in ("auto", "lib"):
    os.environ["MARLMAZE_GEMM"] = mode
    actor.zero_grad(set_to_none=True)
    h0 = actor.trunk.__func__  # noqa
    from marlmaze.networks import _FusedFront, front_params, _X3Trunk, _linear
    hf = _FusedFront.apply(x, True, *front_params(actor.projection, actor.attention)).detach().requires_grad_(True)
    h = hf
    params = [t for lin in actor.layers for t in (lin.weight, lin.bias)]
    if mode == "auto":
        h = _X3Trunk.apply(hf, *params)
    else:
        for lin in actor.layers:
            h = _linear(h, lin.weight, lin.bias, relu=True)
    g = torch.autograd.grad(h, [hf] + params, dh)
    res[mode] = [h.detach()] + list(g)
# fp64 reference on the CPU
hf64 = hf.detach().double().cpu().requires_grad_(True)
p64 = [p.detach().double().cpu().requires_grad_(True) for p in params]
h = hf64
for i in range(3):
    h = torch.relu(h @ p64[2 * i].t() + p64[2 * i + 1])
g64 = torch.autograd.grad(h, [hf64] + p64, dh.double().cpu())
ref = [h.detach()] + list(g64)
names = ["h3", "dh0", "dW0", "db0", "dW1", "db1", "dW2", "db2"]
for n, a, b, r in zip(names, res["auto"], res["lib"], ref):
    sc = r.abs().max().item()
    ea = (a.double().cpu() - r).abs().max().item() / sc
    eb = (b.double().cpu() - r).abs().max().item() / sc
    print(f"{n}: max|ref| {sc:.3e}  x3 err {ea:.2e}  lib err {eb:.2e}", flush=True)
