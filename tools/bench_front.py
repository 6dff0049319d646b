"""Times the fused actor front-end kernels (csrc/actor_front.hip) at the
update's row count (419,430 = 2 x 209,715) with HIP events."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "marl-maze_amd"))
import torch  # noqa: E402

from marlmaze.networks import Actor, _FusedFront, front_params  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 419430
PARITY = (sys.argv[2] != "0") if len(sys.argv) > 2 else True
torch.manual_seed(0)
actor = Actor([264, 264, 264]).cuda()
pr, at = actor.projection, actor.attention
x = torch.rand(B, 65, device="cuda")
dh = torch.randn(B, 460, device="cuda")
params = front_params(pr, at)


def fwd():
    return _FusedFront.apply(x, PARITY, *params)


def step():
    h = fwd()
    torch.autograd.backward(h, dh)


res = {}
for name, fn in (("fwd", fwd), ("fwd+bwd", step)):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        fn()
    e1.record()
    torch.cuda.synchronize()
    res[name + "_ms"] = e0.elapsed_time(e1) / 10
res["bwd_ms"] = res["fwd+bwd_ms"] - res["fwd_ms"]
res["rows"] = B
res["parity"] = PARITY
res["bwd_algo"] = os.environ.get("MARLMAZE_FRONT_BWD", "valu")
print(json.dumps(res))
