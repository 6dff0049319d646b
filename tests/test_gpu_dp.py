"""Data parallelism on the GPU path: two ranks, one process
each, built through ``DP.from_env`` exactly as INTEGRATION.md tells a user
(torchrun environment, then ``PPO(..., dp=DP.from_env())``).  The box has one
GPU, so the rehearsal uses the gloo backend with both ranks on cuda:0; the
update then runs the real GPU path -- fused front-end, bf16x3 MLP trunk,
split-K weight gradients, fused policy loss, the flat gradient bucket whose
views become ``.grad``, fused Adam -- with the all-reduces between the ranks.

Workload: BASELINE configs[3]'s per-GPU share -- 8,192 parallel 20x20 mazes
per rank, T=32 (262,144 samples per rank, 52,428-sample minibatches).

Checks:
* each rank's rollout is the oracle's for the mazes it owns (seeds = global
  maze index; 32 columns per rank replayed, bit-exact);
* the per-epoch episode statistics are global (all-reduced);
* the 2-rank update equals ONE process updating on the union of the two
  shards (minibatch k = rank-0 slice k + rank-1 slice k): all 25 minibatches'
  losses and clipped-gradient norms at rtol 2e-5 (the two differ only in the
  summation order of the gradient all-reduce), parameters at the end equal on
  both ranks bit for bit.
"""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch

from oracle.env import OracleEnv

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
N_MAZES, T, SIZE, MAX_T = 8192, 32, 20, 12

_WORKER = r"""
import os, sys
sys.path.insert(0, {pkg!r}); sys.path.insert(0, {repo!r})
import torch
rank = int(sys.argv[1])
os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE="2", MASTER_ADDR="127.0.0.1",
                  MASTER_PORT=sys.argv[2])
from marlmaze.dist import DP
from marlmaze.PPO import PPO
import torch.distributed as dist
dp = DP.from_env(backend="gloo")
assert dp.rank == rank and dp.world == 2
assert torch.cuda.current_device() == rank % torch.cuda.device_count()
n, T = {n}, {T}
B = n * T
ag = PPO(2, epochs=1, batch_size=2 * (B - B % 5), lr=1.4e-4, n_envs=n, horizon=T, dp=dp, load=False,
         verbose=False, save=False, bootstrap=False, sample_seed=21,
         env_config=dict(default_size=({size}, {size}), max_timestep={max_t}, seed_base=0))
assert ag.device == torch.device("cuda", torch.cuda.current_device())
obs, act, lp, sp, ep_lens, masks, adv, val = ag.get_batch()
idx = torch.randperm(B, generator=torch.Generator().manual_seed(100 + rank))
hist = ag.update(obs, act, lp, masks, adv, val, index_list=idx)
stats = dp.episode_stats(ep_lens, sp)
torch.save(dict(obs=obs.cpu(), act=act.cpu(), logp=lp.cpu(), masks=masks.cpu(), adv=adv.cpu(), val=val.cpu(),
                idx=idx, hist=hist.cpu(), stats=torch.tensor(stats, dtype=torch.float64),
                local=torch.tensor([len(ep_lens), sum(ep_lens), sum(sp)], dtype=torch.float64),
                params={{k: v.cpu() for k, v in ag.actor.state_dict().items()}}),
           sys.argv[3] + "_%d.pt" % rank)
dist.destroy_process_group()
"""


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_two_rank_gpu_update_equals_union_update(tmp_path):
    from marlmaze.PPO import PPO

    script = tmp_path / "worker.py"
    script.write_text(_WORKER.format(pkg=os.path.join(REPO, "marl-maze_amd"), repo=REPO, n=N_MAZES, T=T, size=SIZE,
                                     max_t=MAX_T))
    out = str(tmp_path / "rank")
    port = str(_free_port())
    env = dict(os.environ)
    procs = [subprocess.Popen([sys.executable, "-u", str(script), str(r), port, out], env=env) for r in range(2)]
    rcs = [p.wait(timeout=240) for p in procs]
    assert rcs == [0, 0], rcs
    r = [torch.load(f"{out}_{k}.pt", weights_only=True) for k in range(2)]

    # each rank owns mazes [rank*n, (rank+1)*n): replay 32 of its columns in the oracle
    cols = np.arange(0, N_MAZES, N_MAZES // 32)
    for rank in range(2):
        o = r[rank]["obs"].numpy().reshape(T, N_MAZES, 2, 65)[:, cols]
        m = r[rank]["masks"].numpy().reshape(T, N_MAZES, 2, 6)[:, cols]
        a = r[rank]["act"].numpy().reshape(T, N_MAZES, 2, 2)[:, cols].astype(np.int8)
        ora = OracleEnv(len(cols), seeds=(cols + rank * N_MAZES).astype(np.uint64),
                        default_size=(SIZE, SIZE), max_timestep=MAX_T)
        oo, om = ora.reset_all()
        assert np.array_equal(o[0], oo) and np.array_equal(m[0], om), rank
        for s in range(T - 1):
            oo, om, _, _ = ora.step_all(a[s], auto_reset=True)
            assert np.array_equal(o[s + 1], oo) and np.array_equal(m[s + 1], om), (rank, s)

    # episode statistics: global on both ranks
    loc = r[0]["local"] + r[1]["local"]
    assert loc[0] > 0
    want = torch.tensor([loc[0], loc[1] / loc[0], loc[2] / loc[0]], dtype=torch.float64)
    for k in range(2):
        assert torch.allclose(r[k]["stats"], want, rtol=1e-12)

    # the union update in one process (same start parameters: seed 3234 on both sides)
    B = N_MAZES * T
    local_bs = B - B % 5
    mb_l = local_bs // 5
    glob = []
    for k in range(5):
        glob.append(r[0]["idx"][k * mb_l:(k + 1) * mb_l])
        glob.append(B + r[1]["idx"][k * mb_l:(k + 1) * mb_l])
    glob = torch.cat(glob)
    cat = {k: torch.cat([r[0][k], r[1][k]]).cuda() for k in ("obs", "act", "logp", "masks", "adv", "val")}
    ag = PPO(2, epochs=1, batch_size=2 * local_bs, lr=1.4e-4, n_envs=64, load=False, verbose=False, save=False)
    hist = ag.update(cat["obs"], cat["act"], cat["logp"], cat["masks"], cat["adv"], cat["val"],
                     index_list=glob).cpu().numpy()
    for k in range(2):
        # minibatch 0: the same parameters on both sides.  Its losses are per-row sums of the same values: the
        # 1e-5 bar.  Its unclipped gradient norms come from weight gradients summed in a different order (rank
        # halves, then the all-reduce, vs one reduction over the union); the critic's weight gradients cancel
        # ~100:1 over the rows, so the fp32 order alone moves their norm by up to ~4e-5: 1e-4.  Later
        # minibatches start from parameters that differ in their last bits (Adam steps on gradients rounded
        # differently), compounding over 24 further steps: 1e-4
        np.testing.assert_allclose(r[k]["hist"].numpy()[0, :2], hist[0, :2], rtol=1e-5, atol=1e-6)
        np.testing.assert_allclose(r[k]["hist"].numpy(), hist, rtol=1e-4, atol=1e-6)
    for name, v in r[0]["params"].items():
        assert torch.equal(v, r[1]["params"][name]), name
