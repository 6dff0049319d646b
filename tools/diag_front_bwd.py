"""Front-end backward: per-parameter comparison of the two kernels (MFMA vs VALU) at a few batch sizes;
prints the max abs difference (and NaN counts) per parameter group."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "marl-maze_amd"))
import torch  # noqa: E402

from marlmaze import networks  # noqa: E402
from marlmaze.networks import Actor, _FusedFront, front_params  # noqa: E402

for B in [int(v) for v in (sys.argv[1:] or ["3000", "16", "8", "9"])]:
    torch.manual_seed(0)
    actor = Actor([264, 264, 264], parity_mode=True).cuda()
    with torch.no_grad():
        for p in actor.parameters():
            p.mul_(3.0)
    params = front_params(actor.projection, actor.attention)
    x = torch.randn(B, 65, device="cuda")
    dh = torch.randn(B, 460, device="cuda")
    res = {}
    for algo in ("valu", "mfma"):
        networks.FRONT_BWD_ALGO = algo
        h = _FusedFront.apply(x, True, *params)
        res[algo] = torch.autograd.grad(h, params, dh)
    names = [f"wp{i}" for i in range(23)] + [f"bp{i}" for i in range(23)] + ["wq", "wk", "wv"]
    bad = []
    for n, a, b in zip(names, res["valu"], res["mfma"]):
        d = (a - b).abs().max().item()
        nn_ = int(torch.isnan(b).sum().item())
        if nn_ or d > 1e-3 * a.abs().max().item():
            bad.append(f"{n}: diff {d:.3e} nan {nn_}/{b.numel()}")
    print(B, "OK" if not bad else bad[:12], flush=True)
