"""``Maze`` -- the reference's single-environment API (maze.py:21-163) on the GPU.

Drop-in for ``maze.Maze``: same constructor, ``reset() -> (obs, masks)`` and
``step(action) -> (obs, masks, reward, done)`` with Python lists, and the
public attributes the reference's callers read (``agents``, ``layout``,
``start``, ``end``, ``key``, ``shortest_path``, ``shortest_path_len``,
``current_t``, ``agent_positions``, ``width``, ``height``).  It also wires
``agent.maze`` and ``agent.brain.maze`` (maze.py:39-42), so that
``PPO.train()`` picks up this maze's configuration for its vectorised rollout.

Underneath is a ``VecMaze`` of ONE maze: generation, stepping and observation
run in the same HIP kernels as the batched path.  Like the reference
(maze.py:170-259 draws from the module-level ``random``), ``reset()`` consumes
Python's global ``random`` stream: the MT19937 state is handed to the device
before generation and handed back afterwards, so a program that seeds
``random`` sees exactly the reference's mazes and the same continuation of
``random`` afterwards.

Observation values are the float32 values the reference's lists become inside
``PPO`` (PPO.py:144, ``torch.tensor(obs, dtype=torch.float)``).  The
reference's pygame viewer (maze.py:276-522) is drawn headless by
``marlmaze.viewer`` (``draw_maze`` / ``display_policy`` return PIL images and
write an animated GIF instead of opening a window).
"""
import random

import numpy as np
import torch

from .vecmaze import VecMaze

DELTAS = [(0, -1), (1, 0), (0, 1), (-1, 0)]  # maze.py:19


class Maze:
    def __init__(self, agents, max_timestep=3500, difficulty=1, rand_start=False, rand_sizes=False,
                 rand_range=[6, 12], default_size=[8, 8], device=None):
        self.width = default_size[0] * 2 - 1
        self.height = default_size[1] * 2 - 1
        self.start = None
        self.end = None
        self.key = None
        self.shortest_path = None
        self.shortest_path_len = None
        self.exit_found = False
        self.current_t = 0
        self.agents = agents
        for agent in self.agents:
            agent.maze = self
            if getattr(agent, "brain", None) is not None:
                agent.brain.maze = self
        self.agent_positions = {}
        self.max_timestep = max_timestep
        self.rand_sizes = rand_sizes
        self.rand_range = rand_range
        self.rand_start = rand_start
        self.difficulty = difficulty
        self.default_size = default_size
        self._device = device
        self._env = None
        self._agent_rec = None
        self._obs = None
        self._masks = None

    # ------------------------------------------------------------------
    def _venv(self):
        if self._env is None:
            self._env = VecMaze(1, default_size=tuple(self.default_size), max_timestep=self.max_timestep,
                                difficulty=self.difficulty, rand_start=self.rand_start, rand_sizes=self.rand_sizes,
                                rand_range=tuple(self.rand_range), seeds=np.zeros(1, np.uint64),
                                device=self._device, pregen=False)  # Python's global random feeds each reset
        return self._env

    def _sync(self, obs, masks):
        """Pull the device state of the maze back into the reference's attributes."""
        env = self._env
        mz = env.maze_info()[0]
        self._agent_rec = env.agent_info()[0]
        self.current_t = int(mz["t"])
        self.width, self.height = int(mz["w"]), int(mz["h"])
        self.start = (int(mz["sx"]), int(mz["sy"]))
        self.end = (int(mz["ex"]), int(mz["ey"]))
        self.key = 0 if int(mz["kx"]) < 0 else (int(mz["kx"]), int(mz["ky"]))  # maze.py:157-158
        self.agent_positions = {}
        for agent, rec in zip(self.agents, self._agent_rec):
            self.agent_positions.setdefault((int(rec["x"]), int(rec["y"])), []).append(agent)
        self._obs = obs[0].cpu().tolist()
        self._masks = masks[0].cpu().bool().tolist()

    @property
    def layout(self):
        """Cell values as the reference's list of rows (0 path, 1 wall, 2/3 marks)."""
        if self._env is None:
            return None
        return self._env.layouts()[0].astype(int).tolist()

    def _agent_index(self, agent):
        for i, a in enumerate(self.agents):
            if a is agent:
                return i
        raise ValueError("agent is not in this maze")

    # ------------------------------------------------------------------
    def reset(self):
        """maze.py:55-72.  Draws the new maze from Python's global ``random``."""
        env = self._venv()
        version, words, gauss = random.getstate()
        env.set_rng(0, np.asarray(words, np.uint32))
        obs, masks = env.reset()
        random.setstate((version, tuple(int(w) for w in env.get_rng(0)), gauss))
        self.exit_found = False
        self.shortest_path = env.shortest_path(0)
        self.shortest_path_len = len(self.shortest_path)
        self._sync(obs, masks)
        return [list(o) for o in self._obs], [list(m) for m in self._masks]

    def step(self, action):
        """maze.py:74-122: action = [[move, mark], [move, mark]]."""
        env = self._venv()
        a = torch.as_tensor(np.asarray(action, np.int8).reshape(1, 2, 2), device=env.device)
        obs, masks, reward, done = env.step(a, auto_reset=False)
        self._sync(obs, masks)
        solved = bool(done[0]) and float(reward[0]) == 1.0
        r = 1 if solved else float(reward[0])  # maze.py:115-119: int 1 on success, else key_found * 0.5
        return [list(o) for o in self._obs], [list(m) for m in self._masks], r, bool(done[0])

    def is_valid_cell(self, x, y):  # maze.py:165-167
        return 0 <= x < self.width and 0 <= y < self.height

    def get_shortest_path(self, start, end):
        """maze.py:261-273 (the path through the tree; start/end must be this maze's)."""
        if tuple(start) != self.start or tuple(end) != self.end:
            raise NotImplementedError("only the start -> end path of the current maze is kept on the device")
        return list(self.shortest_path)

    # ---- the viewer (maze.py:276-522), headless: marlmaze.viewer ----
    def draw_maze(self, id=-1):
        """maze.py:277-361: the full maze (id -1) or agent `id`'s fogged view, as a PIL image."""
        from . import viewer

        return viewer.draw_maze(self, id)

    def print_maze(self):  # maze.py:456-458
        for row in self.layout:
            print(row)

    def display_policy(self, id=-1, steps=200, path=None):
        """maze.py:466-522 without the window: `steps` policy steps from a reset, one frame per state
        (returned; an animated GIF at `path` when given)."""
        from . import viewer

        return viewer.display_policy(self, id=id, steps=steps, path=path)
