"""Micro-benchmark of the env-step kernel alone (configs[2]: 65,536 10x10 mazes).

Random legal actions are produced on the device by the sampler kernel from
constant logits, so the loop is: sample -> step(auto_reset) per iteration.
Reports per-kernel times from HIP events on the stream the kernels run on.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "marl-maze_amd"))
import torch  # noqa: E402

from marlmaze import ops  # noqa: E402
from marlmaze.vecmaze import VecMaze  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--mazes", type=int, default=65536)
ap.add_argument("--size", type=int, default=10)
ap.add_argument("--steps", type=int, default=200)
ap.add_argument("--warmup", type=int, default=50)
ap.add_argument("--max-t", type=int, default=1200)
ap.add_argument("--no-pregen", action="store_true", help="generate every reset inline (no side stream)")
a = ap.parse_args()

n = a.mazes
env = VecMaze(n, default_size=(a.size, a.size), max_timestep=a.max_t, pregen=not a.no_pregen)
t0 = time.time()
obs, masks = env.reset()
torch.cuda.synchronize()
print("initial reset of", n, "mazes:", round(time.time() - t0, 3), "s", flush=True)
ml = torch.zeros((2 * n, 5), device="cuda")
kl = torch.zeros((2 * n,), device="cuda")
acts = torch.empty((2 * n, 2), dtype=torch.int8, device="cuda")
s = torch.cuda.current_stream()


def one(i, ev=None):
    ops.sample(ml, kl, masks.view(2 * n, 6), seed=1, offset=i, actions=acts)
    # the step kernel's duration from events stamped at its own start and end (mm_env_step_timed): stream
    # events around the launch would also hold the host's launch gaps of this Python loop
    env.step(acts.view(n, 2, 2), auto_reset=2, obs=obs, masks=masks,
             events=(ev[0], ev[1]) if ev else None)  # finished mazes queued (done list)
    env.reset_done(obs=obs, masks=masks)  # PPO.get_batch's reset (PPO.py:127-130); next mazes pre-generated
    if ev:
        ev[2].record(s)


for i in range(a.warmup):
    one(i)
torch.cuda.synchronize()
evs = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(a.steps)]
for e in evs:  # mm_env_step_timed takes events recorded once already
    e[0].record(s)
    e[1].record(s)
torch.cuda.synchronize()
t0 = time.time()
for i in range(a.steps):
    one(a.warmup + i, evs[i])
torch.cuda.synchronize()
wall = time.time() - t0
step_ms = sorted(e[0].elapsed_time(e[1]) for e in evs)
reset_ms = sorted(e[1].elapsed_time(e[2]) for e in evs)
info = env.maze_info()
H = 2 * a.size - 1
bytes_step = H * H + 703
med = step_ms[len(step_ms) // 2]
print(json.dumps({
    "mazes": n, "steps": a.steps, "wall_s": wall, "env_steps_per_s": n * a.steps / wall,
    "step_kernel_ms_median": med, "step_kernel_ms_min": step_ms[0],
    "reset_ms_median": reset_ms[len(reset_ms) // 2],
    "alg_bytes_per_env_step": bytes_step,
    "achieved_GBps": n * bytes_step / (med * 1e-3) / 1e9,
    "episodes": int(info["episodes"].sum()), "status_any": int(info["status"].any()),
}))
