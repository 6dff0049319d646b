"""ctypes front-end of ``oracle/maze_oracle.c`` (TEST ORACLE ONLY; see oracle/__init__.py).

``OracleEnv`` mirrors a batch of independent reference mazes
(``maze.py:21-273`` + ``maze_agent.py``), each with its own CPython-compatible
MT19937 stream seeded like ``random.seed(seed)``.
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None

OBS_DIM = 65
MASK_DIM = 6
N_ASTATE = 25


def build():
    """Compile liboracle.so with the committed Makefile (gcc only)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "liboracle.so")
        if not os.path.exists(path):
            build()
        L = ctypes.CDLL(path)
        P = ctypes.c_void_p
        i32 = ctypes.c_int
        L.oenv_new.restype = P
        L.oenv_new.argtypes = [i32] * 9
        L.oenv_free.argtypes = [P]
        L.oenv_seed.argtypes = [P, i32, ctypes.c_uint64]
        L.oenv_set_rng.argtypes = [P, i32, P]
        L.oenv_get_rng.argtypes = [P, i32, P]
        L.oenv_reset.argtypes = [P, i32, P, P]
        L.oenv_reset.restype = i32
        L.oenv_step.argtypes = [P, i32, P, P, P, P, P]
        L.oenv_step_all.argtypes = [P, P, P, P, P, P, i32]
        L.oenv_step_all.restype = i32
        L.oenv_reset_all.argtypes = [P, P, P]
        L.oenv_reset_all.restype = i32
        L.oenv_get_maze.argtypes = [P, i32, P, P, P]
        L.oenv_get_agent.argtypes = [P, i32, i32, P]
        L.orng_seed_stream.argtypes = [ctypes.c_uint64, i32, P]
        L.orng_first_random.argtypes = [ctypes.c_uint64]
        L.orng_first_random.restype = ctypes.c_double
        _LIB = L
    return _LIB


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


class OracleEnv:
    """A batch of ``n`` reference mazes (2 agents, tags 2 and 3)."""

    def __init__(self, n, default_size=(8, 8), max_timestep=3500, difficulty=1,
                 rand_start=False, rand_sizes=False, rand_range=(6, 12),
                 seeds=None):
        self.n = n
        self.max_timestep = max_timestep
        L = lib()
        self._h = L.oenv_new(n, default_size[0], default_size[1], max_timestep,
                             difficulty, int(rand_start), int(rand_sizes),
                             rand_range[0], rand_range[1])
        if seeds is None:
            seeds = range(n)
        for i, s in enumerate(seeds):
            L.oenv_seed(self._h, i, int(s))

    def __del__(self):
        if getattr(self, "_h", None):
            lib().oenv_free(self._h)
            self._h = None

    # -- RNG state (CPython random.getstate()[1] layout: 624 words + index)
    def set_rng(self, i, state625):
        st = np.ascontiguousarray(state625, np.uint32)
        lib().oenv_set_rng(self._h, i, _p(st))

    def get_rng(self, i):
        st = np.zeros(625, np.uint32)
        lib().oenv_get_rng(self._h, i, _p(st))
        return st

    # -- Maze.reset / Maze.step
    def reset_all(self):
        obs = np.zeros((self.n, 2, OBS_DIM), np.float32)
        masks = np.zeros((self.n, 2, MASK_DIM), np.uint8)
        lib().oenv_reset_all(self._h, _p(obs), _p(masks))  # failures: maze(i)["error"] & 1
        return obs, masks.astype(bool)

    def reset(self, i):
        obs = np.zeros((2, OBS_DIM), np.float32)
        masks = np.zeros((2, MASK_DIM), np.uint8)
        lib().oenv_reset(self._h, i, _p(obs), _p(masks))  # failures: maze(i)["error"] & 1
        return obs, masks.astype(bool)

    def step(self, i, action):
        act = np.ascontiguousarray(action, np.int8).reshape(2, 2)
        obs = np.zeros((2, OBS_DIM), np.float32)
        masks = np.zeros((2, MASK_DIM), np.uint8)
        r = np.zeros(1, np.float32)
        d = np.zeros(1, np.uint8)
        lib().oenv_step(self._h, i, _p(act), _p(obs), _p(masks), _p(r), _p(d))
        return obs, masks.astype(bool), float(r[0]), bool(d[0])

    def step_all(self, actions, auto_reset=True):
        act = np.ascontiguousarray(actions, np.int8).reshape(self.n, 2, 2)
        obs = np.zeros((self.n, 2, OBS_DIM), np.float32)
        masks = np.zeros((self.n, 2, MASK_DIM), np.uint8)
        r = np.zeros(self.n, np.float32)
        d = np.zeros(self.n, np.uint8)
        lib().oenv_step_all(self._h, _p(act), _p(obs), _p(masks), _p(r), _p(d), int(auto_reset))
        return obs, masks.astype(bool), r, d.astype(bool)

    # -- introspection
    def maze(self, i):
        info = np.zeros(12, np.int32)
        layout = np.zeros(41 * 41, np.uint8)
        path = np.zeros((41 * 41, 2), np.int16)
        lib().oenv_get_maze(self._h, i, _p(info), _p(layout), _p(path))
        w, h = int(info[0]), int(info[1])
        return dict(w=w, h=h, start=(int(info[2]), int(info[3])),
                    end=(int(info[4]), int(info[5])),
                    key=(int(info[7]), int(info[8])) if info[6] else 0,
                    path_len=int(info[9]), t=int(info[10]),
                    error=int(info[11]),
                    layout=layout[:w * h].reshape(h, w).copy(),
                    path=path[:int(info[9])].copy())

    def errors(self):
        return np.array([self.maze(i)["error"] for i in range(self.n)], np.int32)

    def agent(self, i, a):
        out = np.zeros(N_ASTATE, np.int32)
        lib().oenv_get_agent(self._h, i, a, _p(out))
        return out


def mt_stream(seed, n):
    out = np.zeros(n, np.uint32)
    lib().orng_seed_stream(int(seed), n, _p(out))
    return out
