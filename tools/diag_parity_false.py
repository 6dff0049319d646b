"""Diagnostic: stage-by-stage errors of the actor's explicit backward at a
given batch size and parity mode (the front-end forward h0, the MLP's dh0, the
front-end parameter gradients) against an fp64 evaluation of the same modules."""
import copy
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "marl-maze_amd"))
sys.path.insert(0, REPO)
from marlmaze.networks import Actor, front_params, _FusedFront  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 6000
parity = (sys.argv[2] == "1") if len(sys.argv) > 2 else False
torch.manual_seed(0)
actor = Actor([264, 264, 264], parity_mode=parity).cuda()
x = torch.rand(B, 65, device="cuda") + 0.5 * torch.randn(B, 65, device="cuda")
dz = torch.randn(B, 6, device="cuda") / B
z, saved = actor.train_forward(x)
for p in actor.parameters():
    p.grad = torch.zeros_like(p)
actor.train_backward(saved, dz)
a64 = copy.deepcopy(actor).double().cpu()
x64 = x.double().cpu().requires_grad_(False)
h0 = a64.attention(a64.projection(x64))
h0.retain_grad()
h = h0
for lin in a64.layers:
    h = torch.relu(lin(h))
w = torch.cat([a64.move_head.weight, a64.mark_head.weight])
b = torch.cat([a64.move_head.bias, a64.mark_head.bias])
z64 = h @ w.t() + b
z64.backward(dz.double().cpu())
print("z err", ((z.double().cpu() - z64).abs().max() / z64.abs().max()).item())
print("h0 err", ((saved[2][0].double().cpu() - h0).abs().max() / h0.abs().max()).item())
for (n, p), (_, q) in zip(actor.named_parameters(), a64.named_parameters()):
    e = ((p.grad.double().cpu() - q.grad).abs().max() / q.grad.abs().max().clamp_min(1e-30)).item()
    if e > 1e-6:
        print(f"{n}: {e:.2e}")
# the front-end alone with the fp64 dh0 as its upstream gradient
params = front_params(actor.projection, actor.attention)
hh = _FusedFront.apply(x, parity, *params)
g = torch.autograd.grad(hh, params, h0.grad.float().cuda())
p64 = front_params(a64.projection, a64.attention)
for i, (a, q) in enumerate(zip(g, p64)):
    e = ((a.double().cpu() - q.grad).abs().max() / q.grad.abs().max().clamp_min(1e-30)).item()
    if e > 1e-6:
        print(f"front-only param {i}: {e:.2e}")
