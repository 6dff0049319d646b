"""Diagnostic: forward error of the fused front-end (h0 = attention(projection(x)))
on the 4 distinct actor inputs of parity mode (facing one-hot), vs fp64, next to
torch-CPU fp32's error.  Prints max |err| in units of ulp(|h|) and relative."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "marl-maze_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from marlmaze.networks import _FusedFront, front_params, Actor  # noqa: E402
from oracle import ppo as oppo  # noqa: E402

n = np.load(os.path.join(REPO, "tests/golden/nets.npz"))
a = oppo.OActor()
a.load_state_dict({k[6:]: torch.as_tensor(n[k]) for k in n.files if k.startswith("actor/")})
x = torch.zeros(4, 65)
x[torch.arange(4), torch.arange(4)] = 1
a64 = oppo.OActor().double()
a64.load_state_dict(a.state_dict())
h64 = a64.attention(a64.projection(x.double())).detach()
h32 = a.attention(a.projection(x)).detach()
g = Actor([264, 264, 264]).cuda()
g.load_state_dict({k: v.cuda() for k, v in a.state_dict().items()})
hg = _FusedFront.apply(x.cuda(), True, *front_params(g.projection, g.attention)).detach().cpu()
ulp = torch.as_tensor(np.spacing(np.abs(h64.float().numpy())), dtype=torch.float64)
for nm, h in (("cpu32", h32), ("gpu", hg)):
    e = (h.double() - h64)
    print(f"{nm:6s} max err {(e.abs() / ulp).max().item():6.2f} ulp, rms {(e / ulp).pow(2).mean().sqrt().item():.3f} ulp,"
          f" mean signed {(e / ulp).mean().item():+.3f} ulp")
# the same through the MLP trunk (the library / x3 are irrelevant for 4 rows: library path)
