#!/usr/bin/env python3
"""Headline benchmark: PPO training throughput over parallel 2-agent mazes.

BASELINE.json metric: "env-steps/sec (2-agent 10x10 maze) + PPO updates/sec at
1/2/4/8 MI355X".  One bench *step* = one full PPO iteration on every GPU:
rollout of ``horizon`` env-steps in each of ``mazes`` mazes (critic + actor
forward, sampler kernel, env-step kernel, auto-reset), the GAE scan, and the
update of PPO.py:46-85 (5 epochs x 5 minibatches, clipped surrogate + value
MSE, one flat-gradient all-reduce per minibatch under DP, Adam).

value = env-steps/s of the WHOLE job (all ranks, rollout + update time).
Default workload: 65,536 10x10 mazes per GPU (BASELINE configs[2] scale, the
north-star's 1M env-steps/s target) running configs[1]'s rollout+update loop.

Launch: python bench.py [--gpus 1 --steps K --warmup W]
        python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N
"""
import argparse
import glob
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "marl-maze_amd"))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from marlmaze.PPO import PPO  # noqa: E402
from marlmaze.dist import DP  # noqa: E402

HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for ln in f:
                if ln.startswith("model name"):
                    return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _cpu_epoch(threads, batch_size=15000, size=10, max_t=1200, lr=1.4e-4, max_steps=None, updates=5, full_batch=None):
    """One reference PPO.train() epoch (PPO.py:33-87) of the oracle's port: a
    single 10x10 maze, batch_size 15000 (whole episodes until more than that
    are stored, PPO.py:108-141), then 5 x 5 minibatch updates of 3,000.
    max_steps / updates < 5 bound the sample (the rollout's first max_steps
    env-steps and `updates` of the 5 update passes); the epoch's time is then
    extrapolated from the per-step and per-pass times, and the update runs on
    full_batch (a full epoch's batch, (env_steps, tensors), from another run)."""
    from oracle.env import OracleEnv
    from oracle.ppo import CpuPPOPort

    torch.set_num_threads(threads)
    env = OracleEnv(1, default_size=(size, size), max_timestep=max_t, seeds=[0])
    port = CpuPPOPort(env, batch_size=batch_size, lr=lr)
    t0 = time.time()
    steps, batch = port.get_batch(max_steps=max_steps)
    t_roll = time.time() - t0
    if max_steps is not None:  # the update runs on a full epoch's batch
        full, batch = full_batch
        t_roll *= full / steps
        steps = full
    t1 = time.time()
    hist = port.update(batch, updates=updates)
    t_upd = (time.time() - t1) * 5.0 / updates
    n_mb = len(hist) * 5 // updates
    return dict(threads=threads, env_steps=steps, epoch_s=t_roll + t_upd, rollout_s=t_roll, update_s=t_upd,
                env_steps_per_s=steps / (t_roll + t_upd), rollout_env_steps_per_s=steps / t_roll,
                ppo_updates_per_s=n_mb / t_upd, minibatch=batch_size // 5, minibatches=n_mb,
                sampled=("full epoch" if max_steps is None else
                         f"first {max_steps} rollout env-steps and {updates} of 5 update passes, extrapolated"),
                _batch=(steps, batch))


_BOUNDED_CHILD = r"""
import json, sys, time
t0 = time.time()
sys.path[:0] = [{repo!r}, {pkg!r}]
import torch
from oracle.env import OracleEnv
from oracle.ppo import CpuPPOPort
torch.set_num_threads({threads})
prog = open({prog!r}, "a")
def log(**k):
    prog.write(json.dumps(k) + "\n")
    prog.flush()
log(stage="start", s=time.time() - t0)
env = OracleEnv(1, default_size=(10, 10), max_timestep=1200, seeds=[0])
port = CpuPPOPort(env, batch_size=15000, lr=1.4e-4)
done, t_roll = 0, 0.0
while done < {max_steps}:  # the rollout in chunks of 10 env-steps, progress after each
    t = time.time()
    steps, _ = port.get_batch(max_steps=10)
    t_roll += time.time() - t
    done += steps
    log(stage="rollout", steps=done, s=t_roll)
fb = torch.load({fb!r}, weights_only=True)
t = time.time()
port.update(tuple(fb["batch"]), updates=1)
log(stage="update", passes=1, s=time.time() - t)
"""


def _cpu_epoch_bounded(threads, full_batch, max_steps=100, timeout=90):
    """The train() epoch at `threads` threads on a bounded sample, in a child
    process with a time limit (torch at os.cpu_count() threads inside the box's
    CPU share can be very slow on these tiny ops: a run past the limit is
    reported, not waited for).  The child logs its progress (the rollout in
    chunks of 10 env-steps, then one of the five update passes on a full epoch's
    batch), so a run cut by the limit still yields the rollout's rate.  The
    epoch is extrapolated: full_batch's env-steps at the rollout rate plus five
    update passes.  (1,500 steps in one piece never finished in 60 s at 256
    threads in a 16-CPU share, rounds 3-4.)"""
    import subprocess
    import tempfile

    with tempfile.TemporaryDirectory() as d:
        fb = os.path.join(d, "batch.pt")
        prog = os.path.join(d, "progress.jsonl")
        torch.save({"steps": full_batch[0], "batch": list(full_batch[1])}, fb)
        code = _BOUNDED_CHILD.format(repo=REPO, pkg=os.path.join(REPO, "marl-maze_amd"), threads=threads, prog=prog,
                                     max_steps=max_steps, fb=fb)
        timed_out, failed = False, None
        try:
            cp = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=timeout)
            if cp.returncode != 0:  # a crash (import error, OOM kill) is reported as one, not as slowness
                failed = dict(returncode=cp.returncode, stderr_tail=(cp.stderr or "")[-600:])
        except subprocess.TimeoutExpired:
            timed_out = True
        log = []
        if os.path.exists(prog):
            with open(prog) as f:
                log = [json.loads(line) for line in f if line.strip()]
    roll = [e for e in log if e["stage"] == "rollout"]
    upd = [e for e in log if e["stage"] == "update"]
    start = [e["s"] for e in log if e["stage"] == "start"]
    r = dict(threads=threads, timed_out_s=timeout if timed_out else None,
             startup_s=start[0] if start else None)
    if failed:
        r.update(error=failed)
    if not roll:
        if failed:
            r.update(env_steps_per_s=0.0, sampled=f"the child process failed (exit {failed['returncode']}) before "
                                                  "a rollout chunk of 10 env-steps finished")
            return r
        r.update(env_steps_per_s=0.0, sampled=f"no rollout chunk of 10 env-steps finished within {timeout} s")
        return r
    steps, t_roll = roll[-1]["steps"], roll[-1]["s"]
    r.update(rollout_env_steps_per_s=steps / t_roll)
    if upd:
        full = full_batch[0]
        epoch_s = full * t_roll / steps + 5.0 * upd[-1]["s"]
        r.update(env_steps=full, epoch_s=epoch_s, rollout_s=full * t_roll / steps, update_s=5.0 * upd[-1]["s"],
                 env_steps_per_s=full / epoch_s, minibatch=3000, minibatches=25,
                 sampled=f"first {steps} rollout env-steps and 1 of 5 update passes, extrapolated to the epoch")
    else:
        r.update(env_steps_per_s=0.0, sampled=f"{steps} rollout env-steps in {t_roll:.1f} s; the update pass did not "
                                              f"finish within {timeout} s (rollout rate only)")
    return r


def cpu_baseline():
    """BASELINE.md's CPU plan: one full train() epoch of
    the CPU port at the box's CPU share of threads and at 1 thread (and, with
    MARLMAZE_CPU_ALL_THREADS=1, a bounded sample at os.cpu_count() threads).  The port's environment is
    the C oracle (bit-exact to the reference's Python env, ~5x faster than it:
    SURVEY §6), its networks / sampling / update are torch-CPU fp32 like the
    reference's, so the figure OVERSTATES the reference's own train() speed."""
    n_cpu = os.cpu_count() or 1
    share = int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, n_cpu)
    runs = []
    for th in (share, 1):
        print(f"cpu baseline: one train() epoch at {th} thread(s)", file=sys.stderr, flush=True)
        runs.append(_cpu_epoch(th))
    # the os.cpu_count()-thread leg (256 threads in a 16-CPU share: ~0.4 env-steps/s, 90 s of every run in
    # round 5) is opt-in: MARLMAZE_CPU_ALL_THREADS=1
    if n_cpu > share and os.environ.get("MARLMAZE_CPU_ALL_THREADS") == "1":
        print(f"cpu baseline: bounded sample at os.cpu_count() = {n_cpu} threads", file=sys.stderr, flush=True)
        runs.append(_cpu_epoch_bounded(n_cpu, runs[1]["_batch"]))
    for r in runs:
        r.pop("_batch", None)
    best = max(runs, key=lambda r: r["env_steps_per_s"])  # the faster setting (1 thread usually: tiny per-step ops)
    return dict(value=best["env_steps_per_s"], unit="env-steps/s", cores=best["threads"], kind="port",
                sample=f"one full PPO.train() epoch (batch_size 15000, lr 1.4e-4, 1 maze 10x10, max_timestep 1200) "
                       f"of oracle.ppo.CpuPPOPort: C-oracle env (bit-exact, ~5x faster than the reference's Python "
                       f"env) + torch-CPU fp32 actor/critic/Adam; {best['env_steps']} env-steps + "
                       f"{best['minibatches']} minibatch updates of {best['minibatch']} in {best['epoch_s']:.1f} s "
                       f"at {best['threads']} thread(s) ({best['sampled']}; the fastest of "
                       f"{', '.join(str(r['threads']) for r in runs)} threads)",
                os_cpu_count=n_cpu, cpu_model=_cpu_model(), threads_used=[r["threads"] for r in runs],
                runs=runs)


def _workload_label(n, size, dtype):
    """The BASELINE.json config a run measures (the label names what actually ran)."""
    loop = "PPO rollout+GAE+update"
    if dtype == "f16":
        share = (" (configs[4]: 262,144 mazes over 8 GPUs, fp16 actor/critic)" if size == 10 and n * 8 == 262144
                 else " (fp16 actor/critic)")
        return f"{loop} over {n} parallel {size}x{size} 2-agent mazes per GPU, fp16 GEMMs{share}"
    if size == 10 and n == 65536:
        tag = "configs[2], the north-star workload: 65,536 parallel 10x10 mazes per GPU"
    elif size == 10 and n == 4096:
        tag = "configs[1]: 4,096 parallel 10x10 mazes"
    elif size == 20 and n * 8 == 65536:
        tag = "configs[3] per-GPU share: 65,536 20x20 mazes over 8 GPUs = 8,192 per GPU"
    else:
        tag = "not a BASELINE config"
    return f"{loop} over {n} parallel {size}x{size} 2-agent mazes per GPU ({tag})"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--mazes", type=int, default=None,
                    help="mazes per GPU (default 65,536; 32,768 = configs[4]'s 262,144 / 8 with --dtype f16)")
    ap.add_argument("--dtype", choices=("f32", "f16"), default="f32",
                    help="f32: the GEMMs at fp32-class accuracy (x2: fp16 hi + lo planes, three fp16 MFMAs per "
                         "product; a range guard redoes an update at bf16x3 when an operand leaves fp16's range; "
                         "the headline); f16: fp16 MFMA operands "
                         "with fp32 accumulation and fp32 master weights (BASELINE configs[4])")
    ap.add_argument("--size", type=int, default=10, help="default_size (cells); layout is 2*size-1")
    ap.add_argument("--horizon", type=int, default=16, help="env-steps per maze per iteration")
    ap.add_argument("--max-t", type=int, default=1200, help="max_timestep (main.py:20)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-parity", action="store_true",
                    help="parity_mode=False: every feature embedding reads its own observation slice (not the "
                         "reference's quirk Q1, under which the actor sees only obs[0:4])")
    ap.add_argument("--graph", choices=("auto", "on", "off"), default="auto",
                    help="replay the rollout as a captured HIP graph (auto: on below 16,384 mazes per GPU, where the "
                         "per-step launches are host-bound); the env-step kernel's duration for the roofline then "
                         "comes from one instrumented uncaptured rollout after the timed region")
    a = ap.parse_args()

    # MARLMAZE_DP_BACKEND=gloo rehearses N ranks on fewer GPUs (ranks share devices round-robin);
    # the default is nccl (= RCCL) with one rank per GPU
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local % max(1, torch.cuda.device_count()))  # bind the GPU before the process group
    dp = DP.from_env(backend=os.environ.get("MARLMAZE_DP_BACKEND"))  # (from_env binds it too, and passes device_id)
    world = dp.world
    if world != a.gpus and dp.rank == 0:
        print(f"warning: --gpus {a.gpus} but WORLD_SIZE {world}", file=sys.stderr)

    if a.mazes is None:
        a.mazes = 65536 if a.dtype == "f32" else 32768
    n, T = a.mazes, a.horizon
    samples_local = n * T
    batch_global = 5 * ((samples_local * world) // 5)
    graph = a.graph == "on" or (a.graph == "auto" and n < 16384)
    agent = PPO(2, epochs=1, batch_size=batch_global, lr=1.4e-4, n_envs=n, horizon=T, load=False, verbose=False,
                save=False, dp=dp, sample_seed=12345, dtype=a.dtype, graph_rollout=graph, parity_mode=not a.no_parity,
                env_config=dict(default_size=(a.size, a.size), max_timestep=a.max_t, seed_base=0))

    def iteration():
        b = agent.rollout()
        B = T * n
        agent.update(b["obs"][:T].reshape(B, 2, 65), b["act"].reshape(B, 2, 2), b["logp"].reshape(B),
                     b["masks"][:T].reshape(B, 2, 6), b["adv"].reshape(B), b["val"].reshape(B))
        agent._carry_over()

    for _ in range(a.warmup):
        iteration()
    torch.cuda.synchronize()
    dp.barrier()

    if not graph:
        agent.step_events = []  # instrumented env steps inside the timed region (uncaptured rollout)
    upd_ev, roll_ev = [], []
    t0 = time.time()
    for _ in range(a.steps):
        r0, r1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        r0.record()
        b = agent.rollout()
        r1.record()
        roll_ev.append((r0, r1))
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        B = T * n
        agent.update(b["obs"][:T].reshape(B, 2, 65), b["act"].reshape(B, 2, 2), b["logp"].reshape(B),
                     b["masks"][:T].reshape(B, 2, 6), b["adv"].reshape(B), b["val"].reshape(B))
        e1.record()
        upd_ev.append((e0, e1))
        agent._carry_over()
    torch.cuda.synchronize()
    dp.barrier()
    elapsed = time.time() - t0
    if dp.active:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    if graph:  # one instrumented uncaptured rollout after the timed region, for the env-step kernel's duration
        agent.step_events = []
        agent.rollout()
        agent._carry_over()
        torch.cuda.synchronize()
    step_ms = [s.elapsed_time(e) for s, e in agent.step_events]
    upd_ms = [s.elapsed_time(e) for s, e in upd_ev]
    roll_ms = [s.elapsed_time(e) for s, e in roll_ev]
    env_step_ms = float(np.mean(step_ms))
    H = 2 * a.size - 1
    alg_bytes = H * H + 703  # layout + marks + agents r/w + maze r/w + actions + obs + masks + reward + done
    achieved = n * alg_bytes / (env_step_ms * 1e-3) / 1e9
    n_updates = len(agent.history) or None
    minibatches_per_iter = agent.updates_per_batch * len(range(0, batch_global // world, (batch_global // world) // 5))
    total_steps = world * n * T * a.steps

    # HBM traffic of k_step from the latest round's PMC file for this workload (tools/pmc_bench.sh:
    # FETCH_SIZE and WRITE_SIZE in separate passes, gfx950 x2 FETCH correction), per launch
    traffic, traffic_src = None, None
    pmcs = sorted(glob.glob(os.path.join(REPO, "profiles", f"r[0-9][0-9]_pmc_env_step_{n}x{a.size}.json")))
    if pmcs:
        with open(pmcs[-1]) as f:
            traffic = json.load(f).get("hbm_bytes_per_launch")
        traffic_src = os.path.relpath(pmcs[-1], REPO)

    line = {
        "metric": "env-steps/sec (2-agent 10x10 maze) + PPO updates/sec",
        "value": total_steps / elapsed,
        "unit": "env-steps/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": elapsed / a.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": a.dtype,
        "data": "synthetic: procedurally generated mazes (CPython-MT seeds 0..N-1 per GPU), random-init "
                "actor/critic (torch.manual_seed(3234)), actions sampled by the policy",
        "config": {
            "workload": _workload_label(n, a.size, a.dtype),
            "mazes_per_gpu": n, "maze": f"{a.size}x{a.size} (layout {H}x{H})", "max_timestep": a.max_t,
            "horizon": T, "global_batch": batch_global, "minibatch": batch_global // 5,
            "minibatch_steps_per_iter": minibatches_per_iter, "parallelism": f"dp{world}",
            "rollout": "HIP graph replay" if graph else "stream launches",
            "gemm": agent.gemm_prec,
            "parity_mode": not a.no_parity,
        },
        "ppo_updates_per_sec": minibatches_per_iter * a.steps / elapsed,
        "update_ms_per_iter": float(np.mean(upd_ms)),
        "rollout_env_steps_per_sec": total_steps / (elapsed - sum(upd_ms) * 1e-3),
        "rollout_ms_per_iter": float(np.mean(roll_ms)),  # GPU time of rollout() + GAE (events around it)
        "rollout_us_per_step": float(np.mean(roll_ms)) * 1e3 / T,
        "roofline": {
            "kernel": "k_step (mm_env_step)", "bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBPS,
            "unit": "GB/s", "frac": achieved / HBM_PEAK_GBPS, "traffic": traffic, "traffic_source": traffic_src,
            "alg_bytes_per_env_step": alg_bytes, "launch_us": env_step_ms * 1e3,
            "launch_us_median": float(np.median(step_ms)) * 1e3, "launches": len(step_ms),
            "timed_in": "the timed region" if not graph else "one instrumented rollout after the timed region",
        },
    }
    del n_updates
    if dp.rank == 0:
        if world == 1 and not a.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline()
        print(json.dumps(line), flush=True)
    if dp.active:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
