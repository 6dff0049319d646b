"""Whole-episode batches: PPO(episode_batches=True).get_batch against the
reference's get_batch (PPO.py:89-152) replayed in the oracle.

The policy samples on the GPU (Philox, not torch's CPU generator), so the
actions are teacher-forced into the oracle environment.  Checked per batch:
the stop step (the reference's rule: the first episode end after more than
batch_size steps, summed over mazes), the batch composition (complete
episodes only, maze by maze, in time order), obs / masks / episode lengths
bit-exact, V within 1e-5 of the oracle critic, advantages bit-exact against
the reference GAE per whole episode on the same values, returns (adv + V)
within 1e-5 (atol 1e-5) of the oracle's own, and two batches in a row (each
batch starts from a fresh maze, PPO.py:104, so the RNG streams must agree).
"""
import time

import numpy as np
import pytest
import torch

from marlmaze.PPO import PPO
from oracle import ppo as oppo
from oracle.env import OracleEnv

pytestmark = pytest.mark.gpu


def _agent(**kw):
    kw.setdefault("load", False)
    kw.setdefault("verbose", False)
    kw.setdefault("save", False)
    return PPO(2, **kw)


def _segments(done_row, upto):
    """[start, end] of the episodes in done_row[:upto + 1] (each ends at a done)."""
    out, s = [], 0
    for t in range(upto + 1):
        if done_row[t]:
            out.append((s, t))
            s = t + 1
    return out


# (mazes, batch_size, side, max_timestep, episode_chunk); the last case is BASELINE configs[0] -- the reference's
# own run, main.py:17-20 at 10x10: PPO(agent_amount=2, batch_size=15000, lr=0.00014) on ONE maze, max_timestep
# 1200 -- through the drop-in: ~15,000 single-maze steps per batch, two batches in a row
CASES = [(1, 400, 6, 30, 8), (48, 1500, 6, 30, 8), (1, 15000, 10, 1200, 64)]


@pytest.mark.parametrize("n,bs,side,max_t,chunk", CASES, ids=["1maze", "48mazes", "configs0"])
def test_episode_batches_match_reference(n, bs, side, max_t, chunk):
    cfg = dict(default_size=(side, side), max_timestep=max_t)
    ag = _agent(n_envs=n, batch_size=bs, episode_batches=True, episode_chunk=chunk, sample_seed=11,
                env_config=dict(cfg, seed_base=70), lr=0.00014)
    ora = OracleEnv(n, seeds=np.arange(n, dtype=np.uint64) + np.uint64(70), **cfg)
    oc = oppo.OCritic()
    oc.load_state_dict({k: v.detach().cpu() for k, v in ag.critic.state_dict().items()})
    for batch in range(2):
        torch.cuda.synchronize()
        t_start = time.time()
        b_obs, b_act, b_lp, b_sp, ep_lens, b_masks, b_adv, b_val = ag.get_batch()
        torch.cuda.synchronize()
        print(f"get_batch {batch}: {time.time() - t_start:.2f} s for {ag._episode_info['t_stop'] + 1} steps x {n} "
              f"mazes ({b_obs.shape[0]} samples kept, {ag._episode_replayed} replayed after the rewind)")
        info = ag._episode_info
        A = info["act"].cpu().numpy()
        Ts = info["t_stop"] + 1
        assert A.shape[0] == Ts
        oo, om = ora.reset_all()  # PPO.py:104
        O, M, R, D = [], [], [], []
        for t in range(Ts):
            O.append(oo)
            M.append(om)
            oo, om, r, d = ora.step_all(A[t], auto_reset=True)  # PPO.py:120-130
            R.append(r)
            D.append(d)
        O, M, R, D = (np.stack(x, 1) for x in (O, M, R, D))  # [n, Ts, ...]
        assert np.array_equal(D.T, info["done"].cpu().numpy().astype(bool)), batch
        # the stop rule (PPO.py:126-141, summed over mazes)
        le, t_ref = np.full(n, -1), None
        for t in range(Ts):
            le = np.where(D[:, t], t, le)
            if (le + 1).sum() > bs:
                t_ref = t
                break
        assert t_ref == info["t_stop"], batch
        # composition: complete episodes, maze-major
        segs = [_segments(D[i], le[i]) for i in range(n)]
        rows = [(i, t) for i in range(n) for t in range(le[i] + 1)]
        ii, tt = np.array([r[0] for r in rows]), np.array([r[1] for r in rows])
        assert b_obs.shape[0] == len(rows) > bs
        assert np.array_equal(b_obs.cpu().numpy(), O[ii, tt])
        assert np.array_equal(b_masks.cpu().numpy(), M[ii, tt])
        assert np.array_equal(b_act.cpu().numpy(), A[tt, ii].astype(np.float32))
        assert ep_lens == [e - s + 1 for i in range(n) for (s, e) in segs[i]]
        assert len(b_sp) == len(ep_lens) and min(b_sp) > 0
        # values, advantages, returns
        with torch.no_grad():
            Vo = oc(torch.as_tensor(O[ii, tt])).squeeze(-1).numpy()
        Vg = b_val.cpu().numpy()
        np.testing.assert_allclose(Vg, Vo, rtol=1e-5, atol=1e-6)
        adv_g, adv_o, pos = [], [], 0
        for i in range(n):
            for (s, e) in segs[i]:
                L = e - s + 1
                rr = list(R[i, s:e + 1].astype(np.float64))
                dd = D[i, s:e + 1]
                adv_g.append(oppo.gae_fp32(rr, Vg[pos:pos + L], dd))
                adv_o.append(oppo.gae_fp32(rr, Vo[pos:pos + L], dd))
                pos += L
        assert np.array_equal(b_adv.cpu().numpy(), np.concatenate(adv_g)), batch
        rtg_o = np.concatenate(adv_o) + Vo
        np.testing.assert_allclose(info["rtg"].cpu().numpy(), rtg_o, rtol=1e-5, atol=1e-5)
        with torch.no_grad():
            lp = ag.policy_logp(b_obs.cuda(), b_act.cuda(), b_masks.cuda())
        np.testing.assert_allclose(lp.cpu().numpy(), b_lp.cpu().numpy(), rtol=1e-5, atol=2e-6)


def test_episode_batches_train_epoch():
    """train() in the reference's batch mode: whole episodes, then the update
    over batch_size samples of the longer batch (Q8)."""
    ag = _agent(n_envs=256, batch_size=4000, epochs=2, episode_batches=True, sample_seed=2,
                env_config=dict(default_size=(5, 5), max_timestep=40, seed_base=0))
    ag.train()
    assert len(ag.history) == 2
    for h in ag.history:
        assert h["episodes"] > 0 and np.isfinite([h["actor_loss"], h["critic_loss"]]).all()


def test_snapshot_restore_rewinds_every_stream():
    """VecMaze.snapshot / restore (the episode batch's rewind): the steps after a
    restore, with the same actions, repeat the first pass bit for bit, resets and
    MT19937 draws included, and the state after them is the same."""
    from marlmaze.vecmaze import VecMaze

    n, steps = 64, 60
    env = VecMaze(n, default_size=(5, 5), max_timestep=20, seeds=np.arange(n, dtype=np.uint64) + np.uint64(5))
    obs, masks = env.reset()
    rng = np.random.default_rng(1)
    for _ in range(7):  # somewhere mid-episode
        m = masks.cpu().numpy().astype(bool)
        mv = np.where(m[..., :5].any(-1), np.argmax(rng.random(m[..., :5].shape) * m[..., :5], -1), 4)
        obs, masks, _, _ = env.step(torch.as_tensor(np.stack([mv, np.zeros_like(mv)], -1).astype(np.int8)).cuda())
    snap = env.snapshot()
    acts, first = [], []
    for _ in range(steps):
        m = masks.cpu().numpy().astype(bool)
        mv = np.where(m[..., :5].any(-1), np.argmax(rng.random(m[..., :5].shape) * m[..., :5], -1), 4)
        mk = (rng.random((n, 2)) < 0.5) & m[..., 5]
        a = torch.as_tensor(np.stack([mv, mk], -1).astype(np.int8)).cuda()
        acts.append(a)
        obs, masks, r, d = env.step(a)
        first.append((obs.clone(), masks.clone(), r.clone(), d.clone()))
    assert sum(int(f[3].sum()) for f in first) > n  # many resets (and MT draws) in the window
    after = [t.clone() for t in env._state()]
    env.restore(snap)
    for t, s in zip(env._state(), snap):
        assert torch.equal(t, s)
    for a, (o1, m1, r1, d1) in zip(acts, first):
        obs, masks, r, d = env.step(a)
        assert torch.equal(obs, o1) and torch.equal(masks, m1) and torch.equal(r, r1) and torch.equal(d, d1)
    # layouts, agents, mazes, MT streams, and the done list's counters (the pre-generation buffers' progress
    # is asynchronous).  The list entries themselves are scratch: each step appends its finished mazes with
    # atomics from every workgroup, in an order the hardware does not fix (each entry is reset on its own,
    # so the order is not state), and a consumed list's stale entries keep that order.
    for t, s in zip(env._state()[:4], after[:4]):
        assert torch.equal(t, s)
    assert torch.equal(env.work[:64], after[4][:64])
