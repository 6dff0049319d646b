"""The reference's single-maze API (Maze / Agent) over the HIP kernels: same
mazes from the same global ``random`` seeding, the same continuation of the
global MT19937 stream, and the same step results as the reference."""
import random
import types

import numpy as np
import pytest

from marlmaze.maze import Maze
from marlmaze.maze_agent import Agent

pytestmark = pytest.mark.gpu


def _agents():
    brain = types.SimpleNamespace(maze=None)
    return (Agent("RED", brain, None, None, 2), Agent("BLUE", brain, None, None, 3)), brain


def _case_kwargs(c):
    return dict(default_size=[int(c[0]), int(c[1])], rand_start=bool(c[2]), difficulty=int(c[3]),
                rand_sizes=bool(c[4]), rand_range=[int(c[5]), int(c[6])])


def test_maze_facade_generation_and_global_random(golden):
    g = golden("maze_gen")
    for ci, c in enumerate(g["case_cfg"]):
        k0 = int(np.nonzero(g["case"] == ci)[0][0])  # first seed of the case, resets 0..2
        agents, brain = _agents()
        m = Maze(agents, max_timestep=1200, **_case_kwargs(c))
        assert brain.maze is m and all(a.maze is m for a in agents)
        random.seed(int(g["seed"][k0]))
        for r in range(3):
            k = k0 + r
            obs, masks = m.reset()
            assert (m.width, m.height) == (g["w"][k], g["h"][k])
            assert m.start == tuple(g["start"][k]) and m.end == tuple(g["end"][k])
            assert m.key == tuple(g["key"][k])
            assert m.shortest_path_len == g["path_len"][k]
            assert np.array_equal(np.asarray(m.shortest_path), g["path"][k][:g["path_len"][k]])
            assert np.array_equal(np.asarray(m.layout), g["layout"][k][:m.height, :m.width])
            # the global stream continues exactly as after the reference's reset
            assert np.array_equal(np.asarray(random.getstate()[1], np.uint32), g["mt"][k]), (ci, r)
            assert np.array_equal(np.asarray(obs, np.float32), g["obs"][k])
            assert np.array_equal(np.asarray(masks, bool), g["masks"][k])
            # agents stand on shortest_path[0] and [1] (maze.py:64-68)
            assert [(a.x, a.y) for a in agents] == [tuple(p) for p in m.shortest_path[:2]]
            assert all(a.direction == 2 and a.exit_len == -1 and not a.has_key for a in agents)


def test_maze_facade_trajectories(golden):
    t = golden("env_traj")
    for name in t["names"]:
        cfg = t[name + "/cfg"]
        agents, _ = _agents()
        m = Maze(agents, max_timestep=int(cfg[2]), difficulty=int(cfg[3]), rand_start=bool(cfg[4]),
                 rand_sizes=bool(cfg[5]), rand_range=[int(cfg[6]), int(cfg[7])],
                 default_size=[int(cfg[0]), int(cfg[1])])
        random.seed(int(cfg[8]))
        obs, masks = m.reset()
        assert np.array_equal(np.asarray(obs, np.float32), t[name + "/obs0"])
        A = t[name + "/actions"]
        for s in range(len(A)):
            obs, masks, r, d = m.step(A[s].tolist())
            st = t[name + "/astate"][s]
            for i, a in enumerate(agents):  # astate fields 0-8 (make_golden.agent_state order)
                assert [a.x, a.y, a.direction, int(a.has_key), int(a.team_has_key), int(a.knows_end),
                        int(a.other_knows_end), a.exit_len, a.time_from_last_seen] == list(st[i][:9]), (name, s)
                assert list(a.memory) == list(st[i][21:25])
            assert r == t[name + "/reward"][s] and d == bool(t[name + "/done"][s]), (name, s)
            if d:
                obs, masks = m.reset()
            assert np.array_equal(np.asarray(obs, np.float32), t[name + "/obs"][s]), (name, s)
            assert np.array_equal(np.asarray(masks, bool), t[name + "/masks"][s]), (name, s)
            o_i, m_i = agents[1].get_observations()
            assert np.array_equal(np.asarray(o_i, np.float32), t[name + "/obs"][s][1])


def test_main_py_wiring_trains():
    """main.py's construction order: PPO brain, two Agents, a Maze that wires
    itself into the brain; PPO.train() then rolls out that maze configuration
    over many parallel mazes."""
    from marlmaze.PPO import PPO

    brain = PPO(agent_amount=2, batch_size=2000, lr=0.00014, epochs=1, n_envs=256, load=False, verbose=False,
                save=False, sample_seed=4)
    agents = (Agent("RED", brain, None, None, 2), Agent("BLUE", brain, None, None, 3))
    maze = Maze(agents=agents, max_timestep=60, rand_sizes=True, rand_range=[12, 13], rand_start=True,
                difficulty=1, default_size=[4, 4])
    assert brain.maze is maze
    random.seed(0)
    brain.train()
    env = brain.venv
    info = env.maze_info()
    assert env.max_timestep == 60 and env.rand_sizes and env.rand_start
    assert set(np.unique(info["w"]).tolist()) <= {23, 25} and not info["status"].any()
    assert len(brain.history) == 1 and np.isfinite(brain.history[0]["actor_loss"])


def test_integration_snippet_runs():
    """INTEGRATION.md section 2's ctypes block, executed as written from the
    repository root (its asserts: every call returns 0, pre-generation off), and
    its reset observations equal the package's own VecMaze for the same seeds."""
    import os
    import re

    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    md = open(os.path.join(repo, "INTEGRATION.md")).read()
    block = re.search(r"```python\n(import ctypes, torch.*?)```", md, re.S).group(1)
    cwd = os.getcwd()
    os.chdir(repo)
    try:
        ns = {}
        exec(compile(block, "INTEGRATION.md", "exec"), ns)
    finally:
        os.chdir(cwd)
    import torch

    from marlmaze.vecmaze import VecMaze

    N = ns["N"]
    env = VecMaze(N, default_size=(10, 10), max_timestep=1200, seeds=list(range(N)), pregen=False)
    env.reset()
    # the snippet stepped once with "stay": the same step through the package
    act = torch.zeros(N, 2, 2, dtype=torch.int8, device="cuda")
    act[..., 0] = 4
    o1, m1, r1, _ = env.step(act, auto_reset=True)
    assert torch.equal(o1, ns["obs"]) and torch.equal(m1.to(torch.uint8), ns["masks"])
    assert torch.equal(r1, ns["reward"])


def test_display_policy_headless(tmp_path):
    """main.py:17-23 end to end, headless: PPO brain, two Agents with main.py's colours, the Maze, then
    display_policy -- a reset and policy steps through the HIP env, one frame per state, written as a
    GIF; every frame shows the current layout (walls black, marks in the agents' mark colours) and
    the fogged agent view shows the agent's own cell."""
    from PIL import Image

    from marlmaze import viewer
    from marlmaze.PPO import PPO

    brain = PPO(agent_amount=2, batch_size=2000, lr=0.00014, n_envs=16, load=False, verbose=False, save=False,
                sample_seed=6)
    agents = (Agent("RED", brain, "red", "palevioletred1", 2), Agent("BLUE", brain, "royalblue1", "darkslategray1", 3))
    maze = Maze(agents=agents, max_timestep=1200, rand_sizes=True, rand_range=[12, 13], rand_start=True,
                difficulty=1, default_size=[4, 4])
    random.seed(5)
    path = tmp_path / "policy.gif"
    frames = maze.display_policy(steps=6, path=str(path))
    assert len(frames) >= 7 and path.exists()
    assert Image.open(path).n_frames == len(frames)
    img = np.asarray(frames[-1])
    C = viewer.CELL_SIZE
    assert img.shape == (maze.height * C, maze.width * C, 3)
    lay = np.asarray(maze.layout)
    occupied = set(maze.agent_positions) | {maze.start, maze.end} | set(map(tuple, maze.shortest_path or []))
    if maze.key != 0:
        occupied.add(maze.key)
    mark_rgb = {2: viewer.rgb("palevioletred1"), 3: viewer.rgb("darkslategray1")}
    for y in range(maze.height):
        for x in range(maze.width):
            px = tuple(img[y * C + 2, x * C + 2])  # a cell corner: no agent / flag / key / dot drawn there
            if lay[y, x] == 1:
                assert px == viewer.WALL_COLOR, (x, y)
            elif lay[y, x] in mark_rgb and (x, y) not in occupied:
                assert px == mark_rgb[lay[y, x]], (x, y)
    ax, ay = agents[0].x, agents[0].y
    fog = np.asarray(maze.draw_maze(id=2))
    assert tuple(fog[ay * C + C // 2, ax * C + C // 2]) == viewer.rgb("red")  # the agent's body
    assert tuple(fog[ay * C + 1, ax * C + 1]) == viewer.PATH_COLOR  # its own cell is drawn
    far = [(x, y) for y in range(maze.height) for x in range(maze.width) if abs(x - ax) + abs(y - ay) > 12]
    if far:
        x, y = far[0]
        assert tuple(fog[y * C + 2, x * C + 2]) == viewer.FOG_COLOR  # beyond any ray: fog
