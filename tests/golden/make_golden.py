#!/usr/bin/env python3
"""Capture golden input/output vectors from the reference (rhuangr/MARL-Maze).

Run ONLY in the build container (the reference never travels to the GPU box):

    python tests/golden/make_golden.py            # writes tests/golden/*.npz

What it does
------------
* Injects a stub ``pygame`` module (the reference imports pygame at module top
  and uses ``pygame.Color`` at import time, ``maze.py:1,6-10``; pygame is not
  installed here) and puts ``/root/reference`` on ``sys.path``.
* Forces ``sys.pycache_prefix`` to a scratch directory so that the bytecode
  shipped in ``/root/reference/__pycache__`` is never loaded: the reference is
  imported from its ``.py`` sources only.
* Runs from a scratch CWD (``PPO.py:9`` makes ``PPO.pth`` CWD-relative), so a
  fresh ``PPO(...)`` never auto-loads the shipped checkpoint.  The shipped
  ``PPO.pth`` is read only with ``torch.load(..., weights_only=True)``.
* Writes small ``.npz`` fixtures (data only: inputs and expected outputs).

Fixtures
--------
maze_gen.npz   3 consecutive ``Maze.reset()`` per ``random.seed(s)`` for a grid
               of sizes / rand_start / difficulty / rand_sizes; layout, start,
               end, key, shortest path, and the CPython MT state after each
               reset (pins bit-exact generation + RNG continuation).
env_traj.npz   scripted legal random play (own ``random.Random(seed+1000)``)
               with auto-reset: actions -> obs/masks/reward/done + per-agent
               internal state per step.
env_ppo.npz    a trajectory whose actions are sampled by the reference
               ``PPO.get_action`` with the shipped ``PPO.pth`` weights.
gae.npz        random episodes -> ``PPO.get_GAEs``.
nets.npz       seeded Actor/Critic weights (``torch.manual_seed(3234)``, the
               import-time seed of ``PPO.py:7``), logits/values/log-probs on
               real observations, one clipped-surrogate minibatch update.
train_small.npz  one reference ``PPO.train()`` epoch at batch_size 600 with
               every sampled action, the numpy shuffle, per-minibatch losses,
               grad norms and final parameters (teacher-forced replay).
ckpt_logits.npz  Actor/Critic outputs of the shipped ``PPO.pth`` weights.
"""
import contextlib
import io
import os
import random
import sys
import types

import numpy as np

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))

# ----------------------------------------------------------------------------
# import the reference (stub pygame, private pycache, scratch cwd)
# ----------------------------------------------------------------------------
sys.pycache_prefix = "/tmp/_mm_ref_pycache"
sys.dont_write_bytecode = True
_pg = types.ModuleType("pygame")


class _Color:  # maze.py:6-10 / main.py:6-13 only construct colours
    def __init__(self, *a):
        self.a = a


_pg.Color = _Color
sys.modules["pygame"] = _pg
sys.path.insert(0, REF)
os.makedirs("/tmp/_mm_ref_cwd", exist_ok=True)
os.chdir("/tmp/_mm_ref_cwd")
if os.path.exists("PPO.pth"):
    os.remove("PPO.pth")

import torch  # noqa: E402

import maze as ref_maze  # noqa: E402
import maze_agent as ref_agent  # noqa: E402
import networks as ref_nets  # noqa: E402
import PPO as ref_ppo  # noqa: E402

torch.set_num_threads(4)


class _Brain:
    """Stand-in for the PPO brain when only the environment is exercised."""

    maze = None


def make_env(brain=None, **kw):
    brain = brain if brain is not None else _Brain()
    agents = (ref_agent.Agent("RED", brain, None, None, 2),
              ref_agent.Agent("BLUE", brain, None, None, 3))
    m = ref_maze.Maze(agents=agents, **kw)
    return m, agents


def pad_layout(layout, hmax, wmax):
    a = np.full((hmax, wmax), 255, np.uint8)
    h, w = len(layout), len(layout[0])
    a[:h, :w] = np.asarray(layout, np.uint8)
    return a


def mt_state():
    st = random.getstate()[1]  # 624 words + index
    return np.asarray(st, np.uint32)


def agent_state(a):
    """Compact per-agent internal state (for debugging parity failures)."""
    route = -1 if a.exit_route is None else len(a.exit_route)
    top = -1 if not a.exit_route else a.exit_route[-1]
    lm = (-1, -1) if a.last_mark_pos is None else a.last_mark_pos
    return [a.x, a.y, a.direction, int(a.has_key), int(a.team_has_key),
            int(a.knows_end), int(a.other_knows_end), a.exit_len,
            a.time_from_last_seen, route, top, lm[0], lm[1],
            a.min_x_visited, a.max_x_visited, a.min_y_visited,
            a.max_y_visited, a.other_last_seen[0], a.other_last_seen[1],
            int(a.sees_end), int(a.sees_key)] + [m for m in a.memory]


N_ASTATE = 25

# ----------------------------------------------------------------------------
# maze generation
# ----------------------------------------------------------------------------
GEN_CASES = []
for size in ([4, 4], [10, 10], [20, 20]):
    for rand_start in (False, True):
        for diff in (1, 3):
            GEN_CASES.append(dict(default_size=size, rand_start=rand_start,
                                  difficulty=diff, rand_sizes=False,
                                  rand_range=[6, 12]))
GEN_CASES.append(dict(default_size=[4, 4], rand_start=True, difficulty=1,
                      rand_sizes=True, rand_range=[12, 13]))  # main.py:20
GEN_CASES.append(dict(default_size=[8, 8], rand_start=False, difficulty=2,
                      rand_sizes=True, rand_range=[6, 12]))  # maze.py:22-23 defaults
GEN_CASES.append(dict(default_size=[7, 5], rand_start=True, difficulty=2,
                      rand_sizes=False, rand_range=[6, 12]))  # non-square
GEN_SEEDS = [0, 1, 7, 12345, 2**32 + 5]
N_RESETS = 3
HMAX = WMAX = 39
PMAX = HMAX * WMAX


def capture_maze_gen():
    rows = dict(case=[], seed=[], reset=[], w=[], h=[], start=[], end=[],
                key=[], path_len=[], path=[], layout=[], mt=[], obs=[],
                masks=[])
    for ci, case in enumerate(GEN_CASES):
        for seed in GEN_SEEDS:
            m, agents = make_env(max_timestep=1200, **case)
            random.seed(seed)
            for r in range(N_RESETS):
                obs, masks = m.reset()
                rows["case"].append(ci)
                rows["seed"].append(seed)
                rows["reset"].append(r)
                rows["w"].append(m.width)
                rows["h"].append(m.height)
                rows["start"].append(m.start)
                rows["end"].append(m.end)
                rows["key"].append(m.key)
                rows["path_len"].append(m.shortest_path_len)
                p = np.full((PMAX, 2), -1, np.int16)
                p[:len(m.shortest_path)] = np.asarray(m.shortest_path)
                rows["path"].append(p)
                rows["layout"].append(pad_layout(m.layout, HMAX, WMAX))
                rows["mt"].append(mt_state())
                rows["obs"].append(np.asarray(obs, np.float32))
                rows["masks"].append(np.asarray(masks, bool))
    cases = np.array([[c["default_size"][0], c["default_size"][1],
                       int(c["rand_start"]), c["difficulty"],
                       int(c["rand_sizes"]), c["rand_range"][0],
                       c["rand_range"][1]] for c in GEN_CASES], np.int32)
    out = {k: np.asarray(v) for k, v in rows.items()}
    out["case_cfg"] = cases
    out["seed"] = np.asarray(rows["seed"], np.uint64)
    np.savez_compressed(os.path.join(OUT, "maze_gen.npz"), **out)
    print("maze_gen:", len(rows["seed"]), "resets")


# ----------------------------------------------------------------------------
# environment trajectories (random legal play, auto-reset)
# ----------------------------------------------------------------------------
TRAJ_CASES = [
    # (name, maze kwargs, seed, steps)
    ("s4_t60", dict(default_size=[4, 4], max_timestep=60), 11, 6000),
    ("s4_rs_d3", dict(default_size=[4, 4], max_timestep=80, rand_start=True,
                      difficulty=3), 12, 6000),
    ("s6_t200", dict(default_size=[6, 6], max_timestep=200), 13, 5000),
    ("s10_t1200", dict(default_size=[10, 10], max_timestep=1200), 14, 3000),
    ("main_cfg", dict(default_size=[4, 4], max_timestep=1200, rand_sizes=True,
                      rand_range=[12, 13], rand_start=True, difficulty=1), 15,
     2500),
    ("s20_t300", dict(default_size=[20, 20], max_timestep=300), 16, 1500),
    ("rsz_5_7", dict(default_size=[4, 4], max_timestep=40, rand_sizes=True,
                     rand_range=[5, 7], rand_start=True), 17, 6000),
]


def legal_random_action(rng, mask):
    legal = [i for i in range(5) if mask[i]]
    if not legal:  # the reference's Categorical would be NaN here
        return None
    move = legal[rng.randrange(len(legal))]
    mark = 1 if (mask[5] and rng.random() < 0.5) else 0
    return [move, mark]


def capture_env_traj():
    out = {}
    stats = {}
    for name, kw, seed, steps in TRAJ_CASES:
        m, agents = make_env(**kw)
        random.seed(seed)
        rng = random.Random(seed + 1000)
        obs, masks = m.reset()
        A, O, M, R, D, S, RS, LAY, KEY, END = ([] for _ in range(10))
        O0, M0 = np.asarray(obs, np.float32), np.asarray(masks, bool)
        n_succ = n_key = n_nolegal = 0
        for t in range(steps):
            acts = [legal_random_action(rng, masks[i]) for i in range(2)]
            if any(a is None for a in acts):
                n_nolegal += 1
                acts = [a if a is not None else [4, 0] for a in acts]
            obs, masks, reward, done = m.step(acts)
            A.append(acts)
            R.append(float(reward))
            D.append(bool(done))
            S.append([agent_state(a) for a in agents])
            n_succ += reward == 1
            n_key += reward == 0.5
            reset_flag = False
            if done:
                obs, masks = m.reset()
                reset_flag = True
            RS.append(reset_flag)
            O.append(np.asarray(obs, np.float32))
            M.append(np.asarray(masks, bool))
            KEY.append(m.key if m.key != 0 else (-1, -1))
            END.append(m.end)
            LAY.append(np.frombuffer(bytes(
                pad_layout(m.layout, HMAX, WMAX).tobytes()), np.uint8).sum())
        out[name + "/obs0"] = O0
        out[name + "/masks0"] = M0
        out[name + "/actions"] = np.asarray(A, np.int8)
        out[name + "/obs"] = np.asarray(O, np.float32)
        out[name + "/masks"] = np.asarray(M, bool)
        out[name + "/reward"] = np.asarray(R, np.float32)
        out[name + "/done"] = np.asarray(D, bool)
        out[name + "/reset"] = np.asarray(RS, bool)
        out[name + "/astate"] = np.asarray(S, np.int32)
        out[name + "/key"] = np.asarray(KEY, np.int16)
        out[name + "/end"] = np.asarray(END, np.int16)
        out[name + "/layout_sum"] = np.asarray(LAY, np.int64)
        cfg = dict(default_size=[4, 4], max_timestep=3500, difficulty=1,
                   rand_start=False, rand_sizes=False, rand_range=[6, 12])
        cfg.update(kw)
        out[name + "/cfg"] = np.array(
            [cfg["default_size"][0], cfg["default_size"][1],
             cfg["max_timestep"], cfg["difficulty"], int(cfg["rand_start"]),
             int(cfg["rand_sizes"]), cfg["rand_range"][0],
             cfg["rand_range"][1], seed], np.int64)
        stats[name] = (n_succ, n_key, n_nolegal)
    out["names"] = np.array([c[0] for c in TRAJ_CASES])
    np.savez_compressed(os.path.join(OUT, "env_traj.npz"), **out)
    print("env_traj (succ, keys, no-legal):", stats)


# ----------------------------------------------------------------------------
# networks / PPO
# ----------------------------------------------------------------------------
def fresh_ppo(**kw):
    """A reference PPO built right after the import-time seed (PPO.py:7)."""
    torch.manual_seed(3234)
    with contextlib.redirect_stdout(io.StringIO()):
        brain = ref_ppo.PPO(agent_amount=2, **kw)
    return brain


def sd_to_np(prefix, sd, out):
    for k, v in sd.items():
        out[prefix + k] = v.detach().cpu().numpy().copy()


def capture_gae():
    brain = fresh_ppo()
    rng = np.random.default_rng(5)
    out = {}
    lens = [1, 2, 3, 7, 40, 200, 1200]
    for li, L in enumerate(lens):
        rew = [0.0] * L
        if L >= 3:
            rew[rng.integers(0, L - 1)] = 0.5
        if L >= 2 and li % 2 == 0:
            rew[-1] = 1  # success reward is a python int (maze.py:118)
        vals = [torch.tensor([[float(x)]], dtype=torch.float32)
                for x in rng.normal(0, 1, L).astype(np.float32)]
        dones = [False] * (L - 1) + [True]
        adv = brain.get_GAEs(rew, vals, dones)
        out[f"L{li}/rew"] = np.asarray(rew, np.float64)
        out[f"L{li}/val"] = np.asarray([v.item() for v in vals], np.float32)
        out[f"L{li}/done"] = np.asarray(dones, bool)
        out[f"L{li}/adv"] = np.asarray(adv, np.float64)
    out["n"] = np.array(len(lens))
    np.savez_compressed(os.path.join(OUT, "gae.npz"), **out)
    print("gae:", len(lens), "episodes")


def capture_nets():
    traj = np.load(os.path.join(OUT, "env_traj.npz"))
    obs = np.concatenate([traj["s4_t60/obs"][:96], traj["s10_t1200/obs"][:96],
                          traj["main_cfg/obs"][:64]])
    masks = np.concatenate([traj["s4_t60/masks"][:96],
                            traj["s10_t1200/masks"][:96],
                            traj["main_cfg/masks"][:64]])
    acts = np.concatenate([traj["s4_t60/actions"][1:97],
                           traj["s10_t1200/actions"][1:97],
                           traj["main_cfg/actions"][1:65]]).astype(np.float32)
    brain = fresh_ppo(batch_size=600, lr=0.00014)
    out = {}
    sd_to_np("actor/", brain.actor.state_dict(), out)
    sd_to_np("critic/", brain.critic.state_dict(), out)
    o = torch.as_tensor(obs)
    mk = torch.as_tensor(masks)
    ac = torch.as_tensor(acts)
    with torch.no_grad():
        mv, mr = brain.actor(o.reshape(-1, 65))
        v = brain.critic(o)
    out["obs"] = obs
    out["masks"] = masks
    out["actions"] = acts
    out["move_logits"] = mv.numpy()
    out["mark_logits"] = mr.numpy()
    out["values"] = v.numpy()

    class _M:
        agents = (0, 1)

    brain.maze = _M()
    with torch.no_grad():
        lp = [brain.get_log_probs(i, o, ac, mk).numpy() for i in range(2)]
    out["logp0"], out["logp1"] = lp
    # one clipped-surrogate minibatch update (PPO.py:58-85) on this batch
    g = np.random.default_rng(9)
    old_lp = (lp[0] + lp[1] + g.normal(0, 0.1, len(obs))).astype(np.float32)
    advs = g.normal(0, 1, len(obs)).astype(np.float32)
    rtgs = g.normal(0, 1, len(obs)).astype(np.float32)
    out["old_logp"], out["advs"], out["rtgs"] = old_lp, advs, rtgs
    m_old = torch.as_tensor(old_lp)
    m_adv = torch.as_tensor(advs)
    m_rtg = torch.as_tensor(rtgs)
    V = brain.get_state_values(o)
    cur = 0
    for i in range(2):
        cur += brain.get_log_probs(i, o, ac, mk)
    ratio = torch.exp(cur - m_old)
    s1 = ratio * m_adv
    s2 = torch.clamp(ratio, 1 - brain.clip, 1 + brain.clip) * m_adv
    actor_loss = -torch.mean(torch.min(s1, s2))
    brain.actor_optim.zero_grad()
    actor_loss.backward()
    an = torch.nn.utils.clip_grad_norm_(brain.actor.parameters(), brain.max_grad)
    brain.actor_optim.step()
    critic_loss = torch.nn.MSELoss()(V, m_rtg)
    brain.critic_optim.zero_grad()
    critic_loss.backward()
    cn = torch.nn.utils.clip_grad_norm_(brain.critic.parameters(), brain.max_grad)
    brain.critic_optim.step()
    out["actor_loss"] = np.float32(actor_loss.item())
    out["critic_loss"] = np.float32(critic_loss.item())
    out["actor_gnorm"] = np.float32(an.item())
    out["critic_gnorm"] = np.float32(cn.item())
    sd_to_np("actor_after/", brain.actor.state_dict(), out)
    sd_to_np("critic_after/", brain.critic.state_dict(), out)
    np.savez_compressed(os.path.join(OUT, "nets.npz"), **out)
    print("nets: actor_loss", actor_loss.item(), "critic_loss",
          critic_loss.item())


def capture_ckpt_logits():
    sd = torch.load(os.path.join(REF, "PPO.pth"), weights_only=True,
                    map_location="cpu")
    brain = fresh_ppo()
    brain.actor.load_state_dict(sd["actor"])
    brain.critic.load_state_dict(sd["critic"])
    traj = np.load(os.path.join(OUT, "env_traj.npz"))
    obs = traj["s10_t1200/obs"][:128]
    with torch.no_grad():
        mv, mr = brain.actor(torch.as_tensor(obs).reshape(-1, 65))
        v = brain.critic(torch.as_tensor(obs))
    w = {}
    sd_to_np("actor/", sd["actor"], w)
    sd_to_np("critic/", sd["critic"], w)
    w["adam_step"] = np.float32(sd["actor_optim"]["state"][0]["step"])
    w["adam_lr"] = np.float64(sd["actor_optim"]["param_groups"][0]["lr"])
    np.savez_compressed(os.path.join(OUT, "ckpt_logits.npz"), obs=obs,
                        move_logits=mv.numpy(), mark_logits=mr.numpy(),
                        values=v.numpy(), **w)
    print("ckpt_logits: move logit mean", mv.mean(0).numpy())


def capture_env_ppo():
    """Trajectory driven by the reference policy (PPO.pth weights)."""
    sd = torch.load(os.path.join(REF, "PPO.pth"), weights_only=True,
                    map_location="cpu")
    brain = fresh_ppo()
    brain.actor.load_state_dict(sd["actor"])
    brain.critic.load_state_dict(sd["critic"])
    m, agents = make_env(brain=brain, default_size=[6, 6], max_timestep=150)
    random.seed(21)
    torch.manual_seed(22)
    obs, masks = m.reset()
    O0, M0 = np.asarray(obs, np.float32), np.asarray(masks, bool)
    A, LP, O, M, R, D = ([] for _ in range(6))
    with contextlib.redirect_stdout(io.StringIO()):
        for t in range(600):
            acts, lps = [], []
            for i in range(2):
                a, lp = brain.get_action(obs[i], masks[i])
                acts.append([int(a[0]), int(a[1])])
                lps.append(float(lp.reshape(-1)[0]))
            obs, masks, reward, done = m.step(acts)
            if done:
                obs, masks = m.reset()
            A.append(acts)
            LP.append(lps)
            O.append(np.asarray(obs, np.float32))
            M.append(np.asarray(masks, bool))
            R.append(float(reward))
            D.append(bool(done))
    np.savez_compressed(os.path.join(OUT, "env_ppo.npz"), obs0=O0, masks0=M0,
                        actions=np.asarray(A, np.int8),
                        logp=np.asarray(LP, np.float32),
                        obs=np.asarray(O, np.float32),
                        masks=np.asarray(M, bool),
                        reward=np.asarray(R, np.float32),
                        done=np.asarray(D, bool),
                        cfg=np.array([6, 6, 150, 1, 0, 0, 6, 12, 21]))
    print("env_ppo: dones", int(np.sum(D)))


def capture_train_small():
    """One reference PPO.train() epoch, recording everything stochastic."""
    brain = fresh_ppo(epochs=1, batch_size=600, lr=0.00014)
    m, agents = make_env(brain=brain, default_size=[4, 4], max_timestep=120)
    rec = dict(rew=[], done=[], gn=[], loss=[], idx=None)
    real_step = m.step

    def step(action):
        o, k, r, d = real_step(action)
        rec["rew"].append(float(r))
        rec["done"].append(bool(d))
        return o, k, r, d

    m.step = step
    real_clip = torch.nn.utils.clip_grad_norm_

    def clip(params, max_norm, *a, **k):
        n = real_clip(params, max_norm, *a, **k)
        rec["gn"].append(float(n))
        return n

    torch.nn.utils.clip_grad_norm_ = clip
    real_shuffle = np.random.shuffle

    def shuffle(x):
        real_shuffle(x)
        rec["idx"] = np.array(x, copy=True)

    np.random.shuffle = shuffle
    real_mse = torch.nn.MSELoss.forward

    def mse(self, a, b):
        r = real_mse(self, a, b)
        rec["loss"].append(("critic", float(r)))
        return r

    torch.nn.MSELoss.forward = mse
    real_mean = torch.mean

    def tmean(x, *a, **k):
        r = real_mean(x, *a, **k)
        if x.requires_grad and x.dim() == 1:
            rec["loss"].append(("actor", -float(r)))
        return r

    batch = {}
    real_gb = brain.get_batch

    def gb():
        res = real_gb()
        batch["res"] = res
        return res

    brain.get_batch = gb
    random.seed(31)
    np.random.seed(32)
    torch.manual_seed(33)
    torch.mean = tmean
    try:
        with contextlib.redirect_stdout(io.StringIO()):
            brain.train()
    finally:
        torch.mean = real_mean
        torch.nn.utils.clip_grad_norm_ = real_clip
        np.random.shuffle = real_shuffle
        torch.nn.MSELoss.forward = real_mse
    (b_obs, b_act, b_lp, b_sp, ep_lens, b_masks, b_advs, b_vals) = batch["res"]
    out = dict(obs=b_obs.numpy(), actions=b_act.numpy(), logp=b_lp.numpy(),
               masks=b_masks.numpy(), advs=b_advs.numpy(),
               vals=b_vals.numpy(), ep_lens=np.asarray(ep_lens, np.int32),
               shortest=np.asarray(b_sp, np.int32),
               rew=np.asarray(rec["rew"], np.float64),
               done=np.asarray(rec["done"], bool), idx=rec["idx"],
               gnorms=np.asarray(rec["gn"], np.float32),
               actor_loss=np.asarray([v for k, v in rec["loss"]
                                      if k == "actor"], np.float32),
               critic_loss=np.asarray([v for k, v in rec["loss"]
                                       if k == "critic"], np.float32),
               lr_final=np.float64(brain.actor_optim.param_groups[0]["lr"]))
    # initial weights are those of fresh_ppo(); final weights after the epoch
    sd_to_np("actor_after/", brain.actor.state_dict(), out)
    sd_to_np("critic_after/", brain.critic.state_dict(), out)
    np.savez_compressed(os.path.join(OUT, "train_small.npz"), **out)
    if os.path.exists("PPO.pth"):  # train() saves into the scratch cwd
        os.remove("PPO.pth")
    print("train_small: B", len(out["obs"]), "episodes", len(ep_lens),
          "actor losses", len(out["actor_loss"]))


if __name__ == "__main__":
    which = sys.argv[1:] or ["maze_gen", "env_traj", "gae", "nets",
                             "ckpt_logits", "env_ppo", "train_small"]
    for w in which:
        globals()["capture_" + w]()
