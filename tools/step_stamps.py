"""Phase clocks of the env-step kernel (k_step built with -DMM_STEP_STAMPS).

  python tools/step_stamps.py --build      # here: hipcc the instrumented library
  python tools/step_stamps.py              # on the GPU box

Each workgroup's thread 0 records s_memtime at: staging barrier passed (1),
compute done (2), rows staged in LDS (3), rows stored (4), relative to entry,
plus s_memrealtime (100 MHz) at entry and exit.
"""
import argparse
import glob
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "tools", "_var", "libmarlmaze_stamps.so")  # git-ignored; travels to the GPU box

ap = argparse.ArgumentParser()
ap.add_argument("--build", action="store_true")
ap.add_argument("--mazes", type=int, default=65536)
ap.add_argument("--size", type=int, default=10)
ap.add_argument("--steps", type=int, default=30)
a = ap.parse_args()

if a.build:
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    src = sorted(glob.glob(os.path.join(ROOT, "marl-maze_amd", "csrc", "*.hip")))
    subprocess.check_call(["hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-shared", "-std=c++17",
                           "-ffp-contract=off", "-DMM_STEP_STAMPS", "-I", os.path.join(ROOT, "include"),
                           "-I", os.path.join(ROOT, "marl-maze_amd", "csrc"), *src, "-o", OUT])
    print("built", OUT)
    sys.exit(0)

os.environ["MARLMAZE_LIB"] = OUT
sys.path.insert(0, os.path.join(ROOT, "marl-maze_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from marlmaze import ops  # noqa: E402
from marlmaze.vecmaze import VecMaze  # noqa: E402

n = a.mazes
env = VecMaze(n, default_size=(a.size, a.size), max_timestep=1200)
obs, masks = env.reset()
ml = torch.zeros((2 * n, 5), device="cuda")
kl = torch.zeros((2 * n,), device="cuda")
acts = torch.empty((2 * n, 2), dtype=torch.int8, device="cuda")
for i in range(a.steps):
    ops.sample(ml, kl, masks.view(2 * n, 6), seed=1, offset=i, actions=acts)
    env.step(acts.view(n, 2, 2), auto_reset=False, obs=obs, masks=masks)
    if i < a.steps - 1:
        env.reset(env.done, obs=obs, masks=masks)
torch.cuda.synchronize()
mpb = 16 if env.stride > 1024 else 32  # k_step's mazes per workgroup (kMPBig for layouts over 1 KB)
grid = (n + mpb - 1) // mpb
w = env.work[64:64 + 12 * grid].view(grid, 12).cpu().numpy().astype(np.int64)
ph = w[:, :4]
st5 = w[:, 6]
rt0 = w[:, 4] & 0xffffffff
rt1 = w[:, 5] & 0xffffffff
base = rt0.min()
start_us = (rt0 - base) / 100.0
end_us = (rt1 - base) / 100.0


def q(x):
    return {p: float(np.percentile(x, p)) for p in (5, 50, 95)}


print(json.dumps({
    "blocks": grid,
    "cycles_load": q(ph[:, 0]), "cycles_compute": q(ph[:, 1] - ph[:, 0]),
    "cycles_agent_step": q(st5 - ph[:, 0]), "cycles_summaries": q(w[:, 7]), "cycles_replays": q(w[:, 8]),
    "cycles_build_obs": q(ph[:, 1] - (st5 + w[:, 7] + w[:, 8])),
    "cycles_stage": q(ph[:, 2] - ph[:, 1]), "cycles_store": q(ph[:, 3] - ph[:, 2]),
    "cycles_total": q(ph[:, 3]),
    "block_us": q(end_us - start_us), "start_us": q(start_us), "end_us": q(end_us),
    "span_us": float(end_us.max()),
}, indent=1))
