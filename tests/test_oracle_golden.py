"""The CPU oracle against the reference's golden vectors (tests/golden/*.npz).

These pin the oracle (oracle/maze_oracle.c, oracle/ppo.py) to the reference
itself; the GPU parity tests then compare the HIP path with the oracle and
with the same vectors.
"""
import random

import numpy as np
import pytest
import torch

from oracle.env import OracleEnv, mt_stream
from oracle import ppo as oppo


@pytest.mark.parametrize("seed", [0, 1, 7, 12345, 2**32 + 5, 2**63 + 11])
def test_mt19937_matches_cpython(seed):
    r = random.Random(seed)
    ref = np.array([r.getrandbits(32) for _ in range(3000)], np.uint32)
    assert np.array_equal(mt_stream(seed, 3000), ref)


def _gen_env(g, k, n=1):
    c = g["case_cfg"][g["case"][k]]
    return OracleEnv(n, default_size=(int(c[0]), int(c[1])), max_timestep=1200, difficulty=int(c[3]),
                     rand_start=bool(c[2]), rand_sizes=bool(c[4]), rand_range=(int(c[5]), int(c[6])),
                     seeds=[int(g["seed"][k])] * n)


def test_maze_generation_matches_reference(golden):
    g = golden("maze_gen")
    firsts = np.nonzero(g["reset"] == 0)[0]
    assert len(firsts) >= 40
    for k in firsts:
        e = _gen_env(g, k)
        for r in range(3):  # three consecutive resets continue one RNG stream
            kk = k + r
            obs, masks = e.reset(0)
            m = e.maze(0)
            assert (m["w"], m["h"]) == (g["w"][kk], g["h"][kk])
            assert m["start"] == tuple(g["start"][kk])
            assert m["end"] == tuple(g["end"][kk])
            assert m["key"] == tuple(g["key"][kk])
            assert m["path_len"] == g["path_len"][kk]
            assert np.array_equal(m["path"], g["path"][kk][:m["path_len"]])
            assert np.array_equal(m["layout"], g["layout"][kk][:m["h"], :m["w"]])
            assert np.array_equal(e.get_rng(0), g["mt"][kk])
            assert np.array_equal(obs, g["obs"][kk])
            assert np.array_equal(masks, g["masks"][kk])


def _traj_env(t, name):
    cfg = t[name + "/cfg"]
    return OracleEnv(1, default_size=(int(cfg[0]), int(cfg[1])), max_timestep=int(cfg[2]),
                     difficulty=int(cfg[3]), rand_start=bool(cfg[4]), rand_sizes=bool(cfg[5]),
                     rand_range=(int(cfg[6]), int(cfg[7])), seeds=[int(cfg[8])])


def test_env_trajectories_match_reference(golden):
    t = golden("env_traj")
    total = 0
    for name in t["names"]:
        e = _traj_env(t, name)
        obs, masks = e.reset(0)
        assert np.array_equal(obs, t[name + "/obs0"]) and np.array_equal(masks, t[name + "/masks0"])
        A = t[name + "/actions"]
        for s in range(len(A)):
            o, mk, r, d = e.step(0, A[s])
            st = np.stack([e.agent(0, a) for a in range(2)])
            if d:
                o, mk = e.reset(0)
            assert r == t[name + "/reward"][s] and d == t[name + "/done"][s], (name, s)
            assert np.array_equal(st, t[name + "/astate"][s]), (name, s)
            assert np.array_equal(o, t[name + "/obs"][s]), (name, s)
            assert np.array_equal(mk, t[name + "/masks"][s]), (name, s)
        total += len(A)
    assert total > 25000


def test_gae_matches_reference(golden):
    g = golden("gae")
    for i in range(int(g["n"])):
        a = oppo.gae_fp32(list(g[f"L{i}/rew"]), g[f"L{i}/val"], g[f"L{i}/done"])
        assert np.array_equal(a, g[f"L{i}/adv"].astype(np.float32))


def test_gae_bootstrap_restatement_on_reference_episodes(golden):
    """oracle.ppo.gae_bootstrap_fp32 (the bench's bootstrapped fragments; no
    reference counterpart) on a fragment made of the reference's recorded
    episodes back to back: every segment closed by its done flag, so the result
    is the reference's own per-episode advantages whatever V(s_T) is; with the
    last episode left open, its advantages move and the earlier ones do not."""
    g = golden("gae")
    eps = [(list(g[f"L{i}/rew"]), g[f"L{i}/val"], g[f"L{i}/done"].astype(bool)) for i in range(int(g["n"]))]
    assert all(d[-1] for _, _, d in eps)
    rew = sum((r for r, _, _ in eps), [])
    val = np.concatenate([v for _, v, _ in eps]).astype(np.float32)
    done = np.concatenate([d for _, _, d in eps])
    ref = np.concatenate([g[f"L{i}/adv"].astype(np.float32) for i in range(int(g["n"]))])
    for lv in (0.0, 3.5):
        assert np.array_equal(oppo.gae_bootstrap_fp32(rew, val, done, lv), ref)
    opened = done.copy()
    opened[-1] = False
    a = oppo.gae_bootstrap_fp32(rew, val, opened, 3.5)
    n_last = len(eps[-1][0])
    assert np.array_equal(a[:-n_last], ref[:-n_last]) and not np.array_equal(a[-n_last:], ref[-n_last:])


@pytest.fixture()
def four_threads():
    old = torch.get_num_threads()
    torch.set_num_threads(4)  # orthogonal_ init (LAPACK QR) depends on the thread count
    yield
    torch.set_num_threads(old)


def test_network_init_forward_update(golden, four_threads):
    n = golden("nets")
    actor, critic = oppo.make_nets()
    for k, v in actor.state_dict().items():
        assert np.array_equal(v.numpy(), n["actor/" + k]), k
    for k, v in critic.state_dict().items():
        assert np.array_equal(v.numpy(), n["critic/" + k]), k
    o, mk, ac = (torch.as_tensor(n[k]) for k in ("obs", "masks", "actions"))
    with torch.no_grad():
        mv, mr = actor(o.reshape(-1, 65))
        v = critic(o)
        lp0 = oppo.log_probs(actor, 0, o, ac, mk)
        lp1 = oppo.log_probs(actor, 1, o, ac, mk)
    assert np.array_equal(mv.numpy(), n["move_logits"]) and np.array_equal(mr.numpy(), n["mark_logits"])
    assert np.array_equal(v.numpy(), n["values"])
    assert np.array_equal(lp0.numpy(), n["logp0"]) and np.array_equal(lp1.numpy(), n["logp1"])
    aopt = torch.optim.Adam(actor.parameters(), lr=0.00014)
    copt = torch.optim.Adam(critic.parameters(), lr=0.00014)
    al, cl, ga, gc = oppo.minibatch_step(actor, critic, aopt, copt, o, ac, torch.as_tensor(n["old_logp"]),
                                         torch.as_tensor(n["advs"]), torch.as_tensor(n["rtgs"]), mk)
    assert np.float32(al) == n["actor_loss"] and np.float32(cl) == n["critic_loss"]
    assert np.float32(ga) == n["actor_gnorm"] and np.float32(gc) == n["critic_gnorm"]
    for k, p in actor.state_dict().items():
        assert np.array_equal(p.numpy(), n["actor_after/" + k]), k


def test_train_epoch_teacher_forced(golden, four_threads):
    t = golden("train_small")
    actor, critic = oppo.make_nets()
    aopt = torch.optim.Adam(actor.parameters(), lr=0.00014)
    copt = torch.optim.Adam(critic.parameters(), lr=0.00014)
    hist = oppo.update_epoch(actor, critic, aopt, copt, *(torch.as_tensor(t[k]) for k in
                             ("obs", "actions", "logp", "masks", "advs", "vals")), t["idx"], 600)
    assert np.array_equal(np.float32([h[0] for h in hist]), t["actor_loss"])
    assert np.array_equal(np.float32([h[1] for h in hist]), t["critic_loss"])
    assert np.array_equal(np.float32([[h[2], h[3]] for h in hist]).reshape(-1), t["gnorms"])
    for k, p in actor.state_dict().items():
        assert np.array_equal(p.numpy(), t["actor_after/" + k]), k
    assert aopt.param_groups[0]["lr"] == t["lr_final"]


def test_train_batch_advantages(golden):
    """b_advs of the recorded rollout = per-episode GAE of its rewards/values."""
    t = golden("train_small")
    rew, done, vals = t["rew"], t["done"], t["vals"]
    ends = np.nonzero(done)[0]
    start, out = 0, []
    for e in ends:
        out.append(oppo.gae_fp32(list(rew[start:e + 1]), vals[start:e + 1], done[start:e + 1]))
        start = e + 1
    assert np.array_equal(np.concatenate(out), t["advs"])


def load_ckpt(golden, actor, critic):
    c = golden("ckpt_logits")
    actor.load_state_dict({k[6:]: torch.as_tensor(c[k]) for k in c.files if k.startswith("actor/")})
    critic.load_state_dict({k[7:]: torch.as_tensor(c[k]) for k in c.files if k.startswith("critic/")})
    return c


def test_checkpoint_logits(golden):
    """The shipped PPO.pth weights (pinned as data) give the reference's logits."""
    actor, critic = oppo.make_nets()
    c = load_ckpt(golden, actor, critic)
    with torch.no_grad():
        mv, mr = actor(torch.as_tensor(c["obs"]).reshape(-1, 65))
        v = critic(torch.as_tensor(c["obs"]))
    assert np.array_equal(mv.numpy(), c["move_logits"]) and np.array_equal(mr.numpy(), c["mark_logits"])
    assert np.array_equal(v.numpy(), c["values"])
    assert c["adam_step"] == 2175  # 87 epochs x 25 minibatch steps


def test_oracle_under_asan_ubsan(tmp_path):
    """Host sanitizers over the C oracle: oracle/asan_driver.c (resets and
    random legal play, 10x10 / 20x20 / 4x4 / random-size / 6x6 mazes with
    auto-reset, ~200k env-steps) built with AddressSanitizer + UBSan, every
    finding fatal.  (GPU sanitizers are not available on this pool; the device
    code shares env_device.h's logic with no host build.)"""
    import os
    import shutil
    import subprocess

    if shutil.which("gcc") is None:
        pytest.skip("gcc not available")
    here = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle")
    exe = str(tmp_path / "asan_driver")
    cmd = ["gcc", "-O1", "-g", "-fno-omit-frame-pointer", "-std=c11", "-fsanitize=address,undefined",
           "-fno-sanitize-recover=all", "-o", exe, os.path.join(here, "maze_oracle.c"),
           os.path.join(here, "asan_driver.c"), "-lm"]
    b = subprocess.run(cmd, capture_output=True, text=True)
    if b.returncode != 0 and "asan" in b.stderr.lower():
        pytest.skip("sanitizer runtime not available: " + b.stderr[-200:])
    assert b.returncode == 0, b.stderr
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:halt_on_error=1:verify_asan_link_order=0",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    r = subprocess.run([exe], capture_output=True, text=True, env=env, timeout=120)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "asan_driver ok" in r.stdout
    assert "runtime error" not in r.stderr
