"""GPU parity of the HIP environment (libmarlmaze.so via VecMaze) -- bit-exact.

Checks the HIP path against (a) the reference's own golden vectors and (b) the
C oracle on large batches of independent mazes driven by random legal play,
at the BASELINE configurations' maze sizes (10x10 and 20x20, 65,536 mazes).
"""
import numpy as np
import pytest
import torch

from marlmaze.vecmaze import VecMaze
from oracle.env import OracleEnv

pytestmark = pytest.mark.gpu


def _cfg_kwargs(c):
    return dict(default_size=(int(c[0]), int(c[1])), difficulty=int(c[3]), rand_start=bool(c[2]),
                rand_sizes=bool(c[4]), rand_range=(int(c[5]), int(c[6])))


def test_generation_matches_reference(golden):
    g = golden("maze_gen")
    for ci, c in enumerate(g["case_cfg"]):
        ks = np.nonzero((g["case"] == ci) & (g["reset"] == 0))[0]
        seeds = [int(g["seed"][k]) for k in ks]
        env = VecMaze(len(ks), max_timestep=1200, seeds=seeds, **_cfg_kwargs(c))
        for r in range(3):
            obs, masks = env.reset()
            obs, masks = obs.cpu().numpy(), masks.cpu().numpy().astype(bool)
            info = env.maze_info()
            lays = env.layouts()
            assert not info["status"].any()
            for j, k in enumerate(ks):
                kk = k + r
                assert (info["w"][j], info["h"][j]) == (g["w"][kk], g["h"][kk])
                assert (info["sx"][j], info["sy"][j]) == tuple(g["start"][kk])
                assert (info["ex"][j], info["ey"][j]) == tuple(g["end"][kk])
                assert (info["kx"][j], info["ky"][j]) == tuple(g["key"][kk])
                assert info["path_len"][j] == g["path_len"][kk]
                assert np.array_equal(np.asarray(env.shortest_path(j)), g["path"][kk][:g["path_len"][kk]])
                assert np.array_equal(lays[j], g["layout"][kk][:info["h"][j], :info["w"][j]])
                assert np.array_equal(env.get_rng(j), g["mt"][kk])
                assert np.array_equal(obs[j], g["obs"][kk]), (ci, j, r)
                assert np.array_equal(masks[j], g["masks"][kk]), (ci, j, r)


@pytest.mark.parametrize("auto_reset", [False, True])
def test_trajectories_match_reference(golden, auto_reset):
    t = golden("env_traj")
    for name in t["names"]:
        cfg = t[name + "/cfg"]
        env = VecMaze(1, default_size=(int(cfg[0]), int(cfg[1])), max_timestep=int(cfg[2]),
                      difficulty=int(cfg[3]), rand_start=bool(cfg[4]), rand_sizes=bool(cfg[5]),
                      rand_range=(int(cfg[6]), int(cfg[7])), seeds=[int(cfg[8])])
        obs, masks = env.reset()
        assert np.array_equal(obs.cpu().numpy()[0], t[name + "/obs0"])
        assert np.array_equal(masks.cpu().numpy()[0].astype(bool), t[name + "/masks0"])
        A = torch.as_tensor(t[name + "/actions"]).cuda()
        for s in range(len(A)):
            obs, masks, r, d = env.step(A[s:s + 1], auto_reset=auto_reset)
            if not auto_reset:
                st = env.agent_state(0)
                assert np.array_equal(st, t[name + "/astate"][s]), (name, s, st, t[name + "/astate"][s])
                if bool(d[0]):
                    env.reset(d)
            assert float(r[0]) == t[name + "/reward"][s] and bool(d[0]) == t[name + "/done"][s], (name, s)
            assert np.array_equal(obs.cpu().numpy()[0], t[name + "/obs"][s]), (name, s)
            assert np.array_equal(masks.cpu().numpy()[0].astype(bool), t[name + "/masks"][s]), (name, s)
        assert not env.status().any()


def test_policy_trajectory_matches_reference(golden):
    """Trajectory whose actions the reference PPO.pth policy sampled."""
    t = golden("env_ppo")
    env = VecMaze(1, default_size=(6, 6), max_timestep=150, seeds=[21])
    obs, masks = env.reset()
    assert np.array_equal(obs.cpu().numpy()[0], t["obs0"])
    A = torch.as_tensor(t["actions"]).cuda()
    for s in range(len(A)):
        obs, masks, r, d = env.step(A[s:s + 1], auto_reset=True)
        assert np.array_equal(obs.cpu().numpy()[0], t["obs"][s]), s
        assert np.array_equal(masks.cpu().numpy()[0].astype(bool), t["masks"][s]), s
        assert float(r[0]) == t["reward"][s] and bool(d[0]) == t["done"][s]


def random_legal(rng, masks):
    """masks [n,2,6] bool -> actions [n,2,2] int8: uniform legal move, mark ~ B(0.5) if allowed."""
    mv = masks[..., :5]
    u = rng.random(mv.shape) * mv
    move = np.argmax(u, axis=-1)
    move = np.where(mv.any(-1), move, 4)
    mark = (rng.random(masks.shape[:2]) < 0.5) & masks[..., 5]
    return np.stack([move, mark], -1).astype(np.int8)


CONFIGS = {
    "10x10": dict(default_size=(10, 10), max_timestep=150),
    "20x20": dict(default_size=(20, 20), max_timestep=120),
    "4x4_t30": dict(default_size=(4, 4), max_timestep=30),
    "main_cfg": dict(default_size=(4, 4), max_timestep=60, rand_sizes=True, rand_range=(12, 13),
                     rand_start=True),
    "d3_rs": dict(default_size=(7, 5), max_timestep=40, rand_start=True, difficulty=3),
    # edge cases: the largest supported side (41x41 layout), the smallest maze
    # with an episode end every step (and key/end give-ups), the full size range
    "21x21_max": dict(default_size=(21, 21), max_timestep=100),
    "2x2_t1": dict(default_size=(2, 2), max_timestep=1),
    "rs_2_21": dict(default_size=(5, 5), max_timestep=25, rand_sizes=True, rand_range=(2, 21), rand_start=True,
                    difficulty=2),
}


@pytest.mark.parametrize("name", list(CONFIGS))
def test_random_play_matches_oracle(name):
    cfg = CONFIGS[name]
    big = max(cfg["default_size"]) >= 20 or cfg.get("rand_sizes", False)
    n, steps = (512 if big else 2048), 260  # the C oracle steps large mazes slowly
    if name == "2x2_t1":  # every step regenerates, and half the 2x2 mazes hit the 65,536-draw give-up
        n, steps = 256, 24
    seeds = np.arange(n, dtype=np.uint64) * np.uint64(7919) + np.uint64(3)
    env = VecMaze(n, seeds=seeds, **cfg)
    ora = OracleEnv(n, seeds=seeds, **cfg)
    go, gm = env.reset()
    oo, om = ora.reset_all()
    assert np.array_equal(go.cpu().numpy(), oo) and np.array_equal(gm.cpu().numpy().astype(bool), om)
    rng = np.random.default_rng(1)
    masks = om
    n_done = 0
    for s in range(steps):
        act = random_legal(rng, masks)
        go, gm, gr, gd = env.step(torch.as_tensor(act).cuda(), auto_reset=True)
        oo, om, orw, od = ora.step_all(act, auto_reset=True)
        gd = gd.cpu().numpy().astype(bool)
        assert np.array_equal(gd, od), s
        assert np.array_equal(gr.cpu().numpy(), orw), s
        assert np.array_equal(go.cpu().numpy(), oo), s
        gmn = gm.cpu().numpy().astype(bool)
        assert np.array_equal(gmn, om), s
        masks = om
        n_done += int(od.sum())
    assert n_done > 0
    # generation give-ups (the reference would hang) must coincide exactly
    assert np.array_equal(env.status() & 1, ora.errors() & 1)
    assert not (env.status() & 2).any()
    for i in range(0, n, 97):
        assert np.array_equal(env.agent_state(i), np.stack([ora.agent(i, a) for a in range(2)])), i
        lay = ora.maze(i)["layout"]
        assert np.array_equal(env.layouts()[i], lay), i


@pytest.mark.parametrize("n", [1, 33, 100])
def test_ragged_batch_sizes_match_oracle(n):
    """Batches that do not fill the 32-maze step tiles (last tile partial)."""
    cfg = dict(default_size=(10, 10), max_timestep=40)
    seeds = np.arange(n, dtype=np.uint64) + np.uint64(11)
    env = VecMaze(n, seeds=seeds, **cfg)
    ora = OracleEnv(n, seeds=seeds, **cfg)
    go, gm = env.reset()
    oo, om = ora.reset_all()
    assert np.array_equal(go.cpu().numpy(), oo)
    rng = np.random.default_rng(n)
    masks = om
    for s in range(90):
        act = random_legal(rng, masks)
        go, gm, gr, gd = env.step(torch.as_tensor(act).cuda(), auto_reset=True)
        oo, om, orw, od = ora.step_all(act, auto_reset=True)
        assert np.array_equal(go.cpu().numpy(), oo), s
        assert np.array_equal(gm.cpu().numpy().astype(bool), om), s
        assert np.array_equal(gr.cpu().numpy(), orw) and np.array_equal(gd.cpu().numpy().astype(bool), od), s
        masks = om


def test_65536_mazes_10x10_match_oracle():
    """configs[2] scale: 65,536 parallel 10x10 mazes, bit-exact vs the oracle."""
    n, steps = 65536, 24
    cfg = dict(default_size=(10, 10), max_timestep=1200)
    env = VecMaze(n, **cfg)
    ora = OracleEnv(n, **cfg)
    go, gm = env.reset()
    oo, om = ora.reset_all()
    assert np.array_equal(go.cpu().numpy(), oo)
    rng = np.random.default_rng(2)
    masks = om
    for s in range(steps):
        act = random_legal(rng, masks)
        go, gm, gr, gd = env.step(torch.as_tensor(act).cuda(), auto_reset=True)
        oo, om, orw, od = ora.step_all(act, auto_reset=True)
        assert np.array_equal(go.cpu().numpy(), oo), s
        assert np.array_equal(gm.cpu().numpy().astype(bool), om), s
        assert np.array_equal(gr.cpu().numpy(), orw) and np.array_equal(gd.cpu().numpy().astype(bool), od)
        masks = om


def test_big_layouts_many_workgroup_rounds_match_oracle():
    """Large layouts (16 mazes per workgroup) step in the latency form (every lane replays both agents; each
    lane's two directions split over the half-wavefronts) at every batch size; layouts up to 1 KB switch to
    the throughput form (replays handed between the wavefronts) above 2 workgroups per CU, which the
    65,536-maze 10x10 test runs.  Here 20x20 mazes above 2 x 256 CUs x 16 mazes per workgroup (several
    workgroup rounds per CU), with resets."""
    n, steps = 9000, 40
    cfg = dict(default_size=(20, 20), max_timestep=30)
    seeds = np.arange(n, dtype=np.uint64) * np.uint64(31) + np.uint64(5)
    env = VecMaze(n, seeds=seeds, **cfg)
    ora = OracleEnv(n, seeds=seeds, **cfg)
    go, gm = env.reset()
    oo, om = ora.reset_all()
    assert np.array_equal(go.cpu().numpy(), oo)
    rng = np.random.default_rng(9)
    masks = om
    for s in range(steps):
        act = random_legal(rng, masks)
        go, gm, gr, gd = env.step(torch.as_tensor(act).cuda(), auto_reset=True)
        oo, om, orw, od = ora.step_all(act, auto_reset=True)
        assert np.array_equal(go.cpu().numpy(), oo), s
        assert np.array_equal(gm.cpu().numpy().astype(bool), om), s
        assert np.array_equal(gr.cpu().numpy(), orw) and np.array_equal(gd.cpu().numpy().astype(bool), od), s
        masks = om
    for i in range(0, n, 997):
        assert np.array_equal(env.agent_state(i), np.stack([ora.agent(i, a) for a in range(2)])), i


def test_reset_mask_and_independence():
    """Resetting a subset leaves the other mazes untouched; per-maze streams are
    independent of the batch they live in (seed i behaves the same alone)."""
    cfg = dict(default_size=(6, 6), max_timestep=50)
    seeds = np.array([5, 17, 99, 1234], np.uint64)
    big = VecMaze(4, seeds=seeds, **cfg)
    big.reset()
    lay0 = [l.copy() for l in big.layouts()]
    mask = torch.tensor([0, 1, 0, 1], dtype=torch.uint8, device="cuda")
    big.reset(mask)
    lay1 = big.layouts()
    assert np.array_equal(lay0[0], lay1[0]) and np.array_equal(lay0[2], lay1[2])
    for j in (1, 3):
        single = VecMaze(1, seeds=[int(seeds[j])], **cfg)
        single.reset()
        single.reset()
        assert np.array_equal(single.layouts()[0], lay1[j])
        assert np.array_equal(single.get_rng(0), big.get_rng(j))


@pytest.mark.parametrize("cfg", [dict(default_size=(10, 10), max_timestep=3),
                                 dict(default_size=(2, 2), max_timestep=1),
                                 dict(default_size=(20, 20), max_timestep=5)])
def test_pregeneration_is_invisible(cfg):
    """mm_env_pregen (next mazes generated ahead on a side stream, resets copy
    them in) gives bit-identical layouts, MT states, observations and episode
    records to inline generation -- also when many resets are queued with no
    host synchronisation, so that resets find their next maze pending (and
    generate it inline) or in flight (and wait for it)."""
    n, steps = 4096, 40
    seeds = np.arange(n, dtype=np.uint64) * np.uint64(31) + np.uint64(5)
    envs = [VecMaze(n, seeds=seeds, pregen=p, **cfg) for p in (False, True)]
    acts = torch.randint(0, 2, (steps, n, 2, 2), generator=torch.Generator().manual_seed(0)).to(torch.int8).cuda()
    outs = []
    for env in envs:
        env.reset()
        rec = []
        for s in range(steps):  # stay (move 4) or 0..1 moves: legality does not matter for this comparison
            a = acts[s].clone()
            a[..., 0] = torch.where(a[..., 0] == 0, 4, 0).to(torch.int8)
            if s % 2:
                env.step(a, auto_reset=2)
                env.reset_done()
            else:
                env.step(a, auto_reset=True)
            rec.append(env.obs.clone())
        torch.cuda.synchronize()
        outs.append((torch.stack(rec).cpu(), env.layout.cpu(), env.rng.cpu(), env.mazes.cpu(), env.agents.cpu()))
    for a, b in zip(*outs):
        assert torch.equal(a, b)
    torch.cuda.synchronize()
    st = envs[1].gen_state.cpu()
    assert ((st == 0) | (st == 1)).all()
    envs[1]._kick_pregen()
    torch.cuda.synchronize()
    assert (envs[1].gen_state.cpu() == 0).all()  # every maze's next maze is ready after one idle pass


def test_illegal_move_is_refused_and_flagged():
    """A move the action mask forbids (into a wall, or an out-of-range move
    code) is refused and flagged with MM_ST_BAD_MOVE in the maze's status word;
    the agent stays on its cell.  The reference walks into the wall after
    printing (maze.py:140-145), i.e. its state is undefined from there on; only
    a caller that ignores the masks reaches this.  Mazes given legal actions in
    the same launch are unaffected: bit-exact with the oracle."""
    from marlmaze import _lib

    n = 512
    cfg = dict(default_size=(10, 10), max_timestep=1200)
    env = VecMaze(n, seeds=list(range(n)), **cfg)
    obs, masks = env.reset()
    m = masks.cpu().numpy().astype(bool)
    ora = OracleEnv(n, seeds=np.arange(n, dtype=np.uint64), **cfg)
    oo, om = ora.reset_all()
    assert np.array_equal(obs.cpu().numpy(), oo) and np.array_equal(m, om)
    before = env.agent_info()
    act = np.zeros((n, 2, 2), np.int8)
    act[:, :, 0] = 4  # stay
    bad = np.zeros(n, bool)
    for i in range(0, n, 2):
        walls = np.nonzero(~m[i, 0, :4])[0]
        if i % 4 == 0 and len(walls):
            act[i, 0, 0] = walls[0]  # into a wall
            bad[i] = True
        elif i % 4 == 2:
            act[i, 0, 0] = 7  # not a move code
            bad[i] = True
    assert bad.sum() > n // 8
    env.step(torch.as_tensor(act).cuda(), auto_reset=False)
    st = env.status()
    assert np.array_equal((st & _lib.ST_BAD_MOVE) != 0, bad)
    assert not (st & ~np.uint16(_lib.ST_BAD_MOVE)).any()
    after = env.agent_info()
    assert np.array_equal(after["x"][bad, 0], before["x"][bad, 0])
    assert np.array_equal(after["y"][bad, 0], before["y"][bad, 0])
    ok = ~bad
    act_ok = act.copy()
    act_ok[bad, 0, 0] = 4  # the oracle follows the reference (walks into walls): give it legal actions there
    o2, m2, r2, d2 = ora.step_all(act_ok, auto_reset=False)
    assert np.array_equal(env.obs.cpu().numpy()[ok], o2[ok])
    assert np.array_equal(env.masks.cpu().numpy().astype(bool)[ok], m2[ok])
    assert np.array_equal(env.reward.cpu().numpy()[ok], r2[ok])
