"""The two front-end forward kernels (k_front_fwd: 8 samples per workgroup, three per CU; k_front_fwd2: 16
samples, two per CU; bit-identical outputs) timed against each other per row count, in one process,
alternating, median of REPS rounds of 20 launches (HIP events; at small M the host's launch path dominates
these, so run it under rocprofv3 --kernel-trace --stats with SIZES=M for the kernels' own times)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "marl-maze_amd"))
import torch  # noqa: E402

from marlmaze import networks  # noqa: E402
from marlmaze.networks import Actor, _front_fwd, front_params  # noqa: E402


def timed(fn, n=20):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


torch.manual_seed(0)
actor = Actor([264, 264, 264]).cuda()
params = front_params(actor.projection, actor.attention)
reps = int(os.environ.get("REPS", 7))
sizes = os.environ.get("SIZES")
for M in (tuple(int(v) for v in sizes.split(",")) if sizes else (4096, 8192, 12288, 16384, 24576, 52428, 131072,
                                                                  419430)):
    x = torch.rand(M, 65, device="cuda")
    t = {"row1": [], "row2": []}
    for algo in t:
        networks.FRONT_FWD_ALGO = algo
        _front_fwd(x, True, params)
    torch.cuda.synchronize()
    for _ in range(reps):
        for algo in t:
            networks.FRONT_FWD_ALGO = algo
            t[algo].append(timed(lambda: _front_fwd(x, True, params)))
    med = {a: sorted(v)[len(v) // 2] for a, v in t.items()}
    print(f"M={M:7d}: row1 {med['row1']:8.1f} us  row2 {med['row2']:8.1f} us  ratio {med['row2'] / med['row1']:.3f}",
          flush=True)
