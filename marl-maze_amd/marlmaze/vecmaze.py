"""VecMaze: N independent reference mazes stepped together on one MI355X.

Each maze is one reference ``Maze`` with its two ``Agent`` s (maze.py:21-273,
maze_agent.py:15-358) and its own CPython-compatible MT19937 stream
(``random.seed(seed_i)`` semantics, continued across resets).  All state lives
in HBM as structure-of-arrays tensors; stepping, observation gather, masks,
rewards, auto-reset and maze generation run in the HIP kernels of
``libmarlmaze.so`` (``csrc/env_kernels.hip``).  No host synchronisation happens
inside ``step``/``reset``.

Memory per maze (10x10 reference maze, 19x19 layout): 361 B layout + 64 B agents
+ 32 B scalars + 2.5 KB RNG state (touched only at reset).
"""
import ctypes
import os

import numpy as np
import torch

from . import _lib

AGENT_DTYPE = np.dtype([
    ("x", "i1"), ("y", "i1"), ("dir", "i1"), ("flags", "u1"),
    ("lmx", "i1"), ("lmy", "i1"), ("olsx", "i1"), ("olsy", "i1"),
    ("minx", "i1"), ("maxx", "i1"), ("miny", "i1"), ("maxy", "i1"),
    ("mem", "i1", (4,)), ("exit_len", "<i4"), ("tfls", "<i4"), ("reserved", "<i4", (2,)),
])
MAZE_DTYPE = np.dtype([
    ("t", "<i4"), ("w", "i1"), ("h", "i1"), ("ex", "i1"), ("ey", "i1"),
    ("kx", "i1"), ("ky", "i1"), ("sx", "i1"), ("sy", "i1"),
    ("path_len", "<i2"), ("status", "<u2"), ("episodes", "<i4"), ("last_len", "<i4"),
    ("last_path", "<i4"), ("spawn1", "<i4"),
])
assert AGENT_DTYPE.itemsize == 32 and MAZE_DTYPE.itemsize == 32

DELTAS = [(0, -1), (1, 0), (0, 1), (-1, 0)]  # maze.py:19


class VecMaze:
    """``n`` mazes with the reference ``Maze`` configuration (maze.py:22-23).

    Buffers (device tensors, owned here):
      layout [n, stride] u8, agents [n, 2, 32] u8, mazes [n, 32] u8,
      rng [n, 625] i32, work [n + 64] i32,
      obs [n, 2, 65] f32, masks [n, 2, 6] u8, reward [n] f32, done [n] u8.
    """

    def __init__(self, n, default_size=(8, 8), max_timestep=3500, difficulty=1,
                 rand_start=False, rand_sizes=False, rand_range=(6, 12), seeds=None,
                 seed_base=0, device=None, pregen=True):
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device())
        self.device = torch.device(device)
        if self.device.type != "cuda":
            raise _lib.MMError("VecMaze runs on the GPU only (no CPU fallback)")
        L = _lib.lib()
        self.n = int(n)
        self.default_size = (int(default_size[0]), int(default_size[1]))
        self.max_timestep = int(max_timestep)
        self.difficulty = int(difficulty)
        self.rand_start = bool(rand_start)
        self.rand_sizes = bool(rand_sizes)
        self.rand_range = (int(rand_range[0]), int(rand_range[1]))
        stride = L.mm_layout_stride(self.default_size[0], self.default_size[1], int(self.rand_sizes),
                                    self.rand_range[0], self.rand_range[1])
        if stride < 0:
            raise _lib.MMError(f"maze size exceeds the {_lib.MAX_SIDE}x{_lib.MAX_SIDE} layout limit")
        self.stride = stride
        d = self.device
        self.layout = torch.ones((self.n, stride), dtype=torch.uint8, device=d)
        self.agents = torch.zeros((self.n, 2, 32), dtype=torch.uint8, device=d)
        self.mazes = torch.zeros((self.n, 32), dtype=torch.uint8, device=d)
        self.rng = torch.zeros((self.n, _lib.RNG_WORDS), dtype=torch.int32, device=d)
        self.work = torch.zeros(self.n + 64, dtype=torch.int32, device=d)
        self.obs = torch.zeros((self.n, 2, _lib.OBS_DIM), dtype=torch.float32, device=d)
        self.masks = torch.zeros((self.n, 2, _lib.MASK_DIM), dtype=torch.uint8, device=d)
        self.reward = torch.zeros(self.n, dtype=torch.float32, device=d)
        self.done = torch.zeros(self.n, dtype=torch.uint8, device=d)
        # pre-generation (mm_env_pregen): each maze's next maze is generated ahead on a side stream,
        # so a reset is a copy (the serial backtracker leaves the step's critical path)
        self.pregen = bool(pregen) and os.environ.get("MARLMAZE_PREGEN", "1") != "0"
        # True while a HIP graph captures steps: the side-stream pre-generation is then kicked by the
        # caller after each replay instead (a captured fork must rejoin its origin stream)
        self.capturing = False
        # True while a rollout runs its steps: the kicks only mark the side-stream generation pending and
        # flush_pregen() queues one after the last step, so the generation (a ~1 ms latency-bound kernel)
        # overlaps what follows the rollout instead of sharing the CUs with every step's kernels.  A maze
        # that finishes twice inside one rollout generates its second maze in its reset (same maze).
        self.defer_pregen = False
        self._pregen_pending = False
        if self.pregen:
            self.next_layout = torch.ones((self.n, stride), dtype=torch.uint8, device=d)
            self.next_mazes = torch.zeros((self.n, 32), dtype=torch.uint8, device=d)
            self.next_rng = torch.zeros((self.n, _lib.RNG_WORDS), dtype=torch.int32, device=d)
            self.gen_state = torch.ones(self.n, dtype=torch.int32, device=d)
            self._gen_stream = torch.cuda.Stream(device=d)
            # the side stream reads/writes these: the caching allocator must not hand their memory to
            # another tensor before the side stream's queued work is done
            for t in (self.rng, self.next_layout, self.next_mazes, self.next_rng, self.gen_state):
                t.record_stream(self._gen_stream)
            pg = (self.next_layout.data_ptr(), self.next_mazes.data_ptr(), self.next_rng.data_ptr(),
                  self.gen_state.data_ptr())
        else:
            pg = (None, None, None, None)
        self._desc = _lib.EnvDesc(
            self.n, self.default_size[0], self.default_size[1], self.max_timestep, self.difficulty,
            int(self.rand_start), int(self.rand_sizes), self.rand_range[0], self.rand_range[1], stride,
            self.layout.data_ptr(), self.agents.data_ptr(), self.mazes.data_ptr(), self.rng.data_ptr(),
            self.work.data_ptr(), *pg)
        self.seed(seeds if seeds is not None else np.arange(self.n, dtype=np.uint64) + np.uint64(seed_base))

    # ------------------------------------------------------------------
    # hot path
    # ------------------------------------------------------------------
    def _kick_pregen(self):
        """Queue mm_env_pregen on the side stream, after everything queued so far
        on the current stream (the resets that left mazes pending).  The current
        stream never waits for it: a reset whose next maze is not ready yet
        generates it itself, or waits for the one in flight (gen_state)."""
        if not self.pregen or self.capturing:
            return
        if self.defer_pregen:
            self._pregen_pending = True
            return
        cur = torch.cuda.current_stream(self.device)
        self._gen_stream.wait_stream(cur)
        with torch.cuda.stream(self._gen_stream):
            _lib.check(_lib.lib().mm_env_pregen(ctypes.byref(self._desc), _lib.stream_ptr()), "mm_env_pregen")

    def flush_pregen(self):
        """Queue the generation the deferred kicks left pending (defer_pregen)."""
        if self._pregen_pending:
            self._pregen_pending = False
            self._kick_pregen()

    def _quiesce_pregen(self):
        """The current stream waits for the side stream (before the MT rows are rewritten)."""
        if self.pregen:
            torch.cuda.current_stream(self.device).wait_stream(self._gen_stream)

    def seed(self, seeds):
        """random.seed(seeds[i]) for every maze; agents as Agent.__init__."""
        self._quiesce_pregen()
        s = np.ascontiguousarray(np.asarray(seeds, dtype=np.uint64).reshape(self.n))
        st = torch.from_numpy(s.view(np.int64)).to(self.device)
        _lib.check(_lib.lib().mm_env_seed(ctypes.byref(self._desc), _lib.ptr(st), _lib.stream_ptr()),
                   "mm_env_seed")
        self._seed_keep = st  # keep alive until the kernel ran

    def reset(self, mask=None, obs=None, masks=None):
        """Maze.reset() (maze.py:55-72) for all mazes or those with mask != 0."""
        obs = self.obs if obs is None else obs
        masks = self.masks if masks is None else masks
        m = None
        if mask is not None:
            m = mask.to(device=self.device, dtype=torch.uint8).contiguous()
        _lib.check(_lib.lib().mm_env_reset(ctypes.byref(self._desc), _lib.ptr(m), _lib.ptr(obs),
                                           _lib.ptr(masks), _lib.stream_ptr()), "mm_env_reset")
        self._reset_mask_keep = m  # read by the kernel after this call returns
        self._kick_pregen()
        return obs, masks

    def step(self, actions, auto_reset=True, obs=None, masks=None, reward=None, done=None, ep_stats=None,
             events=None):
        """Maze.step(actions) for all mazes (maze.py:74-122).

        actions: [n, 2, 2] int8 (move 0..4, mark 0/1) on the device.  With
        ``auto_reset`` (=1/True) finished mazes are regenerated and their rows
        hold the reset observation, as ``PPO.get_batch`` does (PPO.py:127-130);
        ``auto_reset=2`` only queues them for ``reset_done()``.
        ep_stats: optional [n, 2] int32 receiving (episode length, shortest
        path length) for the mazes that finished this step.
        events: optional (start, end) ``torch.cuda.Event`` pair (timing
        enabled, already recorded once) stamped at the step kernel's own start
        and end (mm_env_step_timed).
        """
        obs = self.obs if obs is None else obs
        masks = self.masks if masks is None else masks
        reward = self.reward if reward is None else reward
        done = self.done if done is None else done
        if actions.dtype != torch.int8 or not actions.is_contiguous():
            actions = actions.to(torch.int8).contiguous()
        if events is None:
            _lib.check(_lib.lib().mm_env_step(ctypes.byref(self._desc), _lib.ptr(actions), _lib.ptr(obs),
                                              _lib.ptr(masks), _lib.ptr(reward), _lib.ptr(done), _lib.ptr(ep_stats),
                                              int(auto_reset), _lib.stream_ptr()), "mm_env_step")
        else:
            e0, e1 = (ctypes.c_void_p(e.cuda_event) if e is not None else None for e in events)
            _lib.check(_lib.lib().mm_env_step_timed(ctypes.byref(self._desc), _lib.ptr(actions), _lib.ptr(obs),
                                                    _lib.ptr(masks), _lib.ptr(reward), _lib.ptr(done),
                                                    _lib.ptr(ep_stats), int(auto_reset), _lib.stream_ptr(), e0, e1),
                       "mm_env_step_timed")
        if int(auto_reset) == 1:
            self._kick_pregen()
        return obs, masks, reward, done

    def reset_done(self, obs=None, masks=None):
        """Reset the mazes queued by the last step(auto_reset=2)."""
        obs = self.obs if obs is None else obs
        masks = self.masks if masks is None else masks
        _lib.check(_lib.lib().mm_env_reset_done(ctypes.byref(self._desc), _lib.ptr(obs), _lib.ptr(masks),
                                                _lib.stream_ptr()), "mm_env_reset_done")
        self._kick_pregen()
        return obs, masks

    def _state(self):
        ts = [self.layout, self.agents, self.mazes, self.rng, self.work]
        if self.pregen:
            ts += [self.next_layout, self.next_mazes, self.next_rng, self.gen_state]
        return ts

    def snapshot(self):
        """Device copies of every state buffer (the mazes, agents, MT19937 streams, the pre-generated next
        mazes): restore() rewinds the environment to this point, stream-ordered, no host sync."""
        self._quiesce_pregen()  # no generation in flight: the copies are one consistent state
        return [t.clone() for t in self._state()]

    def restore(self, snap):
        """Rewind to a snapshot() (the steps since then, their resets and RNG draws are undone)."""
        self._quiesce_pregen()  # generation queued since the snapshot must not land after the rewind
        for t, s in zip(self._state(), snap):
            t.copy_(s)
        self._kick_pregen()  # mazes whose next maze was pending at the snapshot

    # ------------------------------------------------------------------
    # host-side introspection (tests, facades, stats) -- synchronising
    # ------------------------------------------------------------------
    def maze_info(self):
        return self.mazes.cpu().numpy().view(MAZE_DTYPE).reshape(self.n)

    def agent_info(self):
        return self.agents.cpu().numpy().view(AGENT_DTYPE).reshape(self.n, 2)

    def layouts(self):
        """List of [h, w] uint8 arrays with the reference's cell values."""
        info = self.maze_info()
        lay = self.layout.cpu().numpy()
        out = []
        for i in range(self.n):
            w, h = int(info["w"][i]), int(info["h"][i])
            out.append((lay[i, :w * h] & 3).reshape(h, w))
        return out

    def exit_dirs(self, i):
        info = self.maze_info()[i]
        w, h = int(info["w"]), int(info["h"])
        return (self.layout[i, :w * h].cpu().numpy() >> 2 & 7).reshape(h, w)

    def get_rng(self, i):
        return self.rng[i].cpu().numpy().view(np.uint32).copy()

    def set_rng(self, i, state625):
        self._quiesce_pregen()
        st = np.ascontiguousarray(np.asarray(state625, np.uint32)).view(np.int32)
        self.rng[i].copy_(torch.from_numpy(st))
        if self.pregen:
            self.gen_state[i] = 1  # the pre-generated next maze came from the old state

    def shortest_path(self, i):
        """Reconstruct Maze.shortest_path (start -> end) from the exit table."""
        info = self.maze_info()[i]
        dirs = self.exit_dirs(i)
        x, y = int(info["sx"]), int(info["sy"])
        path = [(x, y)]
        while dirs[y, x] != 4 and len(path) <= dirs.size:
            dx, dy = DELTAS[int(dirs[y, x])]
            x, y = x + dx, y + dy
            path.append((x, y))
        return path

    def agent_state(self, i):
        """Per-agent state vectors in tests/golden/make_golden.py agent_state() order."""
        mz = self.maze_info()[i]
        ag = self.agent_info()[i]
        dirs = self.exit_dirs(i)
        out = []
        for a in ag:
            f = int(a["flags"])
            knows = bool(f & _lib.AF_KNOWS_END)
            x, y = int(a["x"]), int(a["y"])
            if knows:
                # route length = tree-path length from the agent's cell
                n, cx, cy = 0, x, y
                while dirs[cy, cx] != 4 and n <= dirs.size:
                    dx, dy = DELTAS[int(dirs[cy, cx])]
                    cx, cy = cx + dx, cy + dy
                    n += 1
                route_len = n
                top = int(dirs[y, x]) if n > 0 else -1
            else:
                route_len, top = -1, -1
            has_mark = bool(f & _lib.AF_HAS_MARK)
            out.append([x, y, int(a["dir"]), int(bool(f & _lib.AF_HAS_KEY)),
                        int(bool(f & _lib.AF_TEAM_KEY)), int(knows),
                        int(bool(f & _lib.AF_OTHER_KNOWS)), int(a["exit_len"]), int(a["tfls"]),
                        route_len, top,
                        int(a["lmx"]) if has_mark else -1, int(a["lmy"]) if has_mark else -1,
                        int(a["minx"]), int(a["maxx"]), int(a["miny"]), int(a["maxy"]),
                        int(a["olsx"]), int(a["olsy"]), int(bool(f & _lib.AF_SEES_END)),
                        int(bool(f & _lib.AF_SEES_KEY))] + [int(v) for v in a["mem"]])
        del mz
        return np.asarray(out, np.int32)

    def status(self):
        return self.maze_info()["status"]
