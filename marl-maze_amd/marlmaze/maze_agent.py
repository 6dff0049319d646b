"""``Agent`` -- the reference's agent API (maze_agent.py:16-83) over device state.

Drop-in for ``maze_agent.Agent``: same constructor, ``get_action(obs, mask)``
(-> ``(action, exp(log_prob))`` through the brain, maze_agent.py:81-83),
``get_observations()`` and the state attributes the reference exposes
(``x``, ``y``, ``direction``, ``has_key``, ``knows_end``, ``exit_len``,
``memory`` ...).  The state itself lives in the maze's device buffers and is
advanced by the HIP step kernel; the attributes read the copy that
``Maze.reset()`` / ``Maze.step()`` pull back after every call.  The tags must
be 2 and 3, as in the reference (``id[2 - tag]``, maze_agent.py:129).
"""
from collections import deque

from . import _lib
from .maze import DELTAS

ACTIONS = ['forward', 'right', 'backward', 'left']  # maze_agent.py:5-6
DIRECTIONS = ['north', 'east', 'south', 'west']
FEATURE_DIMS = [4, 4, 4, 4, 4, 4, 4, 4, 4, 4, 4, 4, 2, 2, 1, 4, 1, 1, 1, 1, 1, 1, 2]  # maze_agent.py:13


class Agent:
    def __init__(self, name, brain, color, mark_color, tag, vision_range=4):
        if tag not in (2, 3):
            raise ValueError("agent tags must be 2 and 3 (maze_agent.py:129)")
        self.maze = None
        self.name = name
        self.vision_range = vision_range
        self.brain = brain
        self.color = color
        self.mark_color = mark_color
        self.tag = tag

    # ------------------------------------------------------------------
    def get_action(self, obs, mask):
        """maze_agent.py:81-83."""
        from math import exp

        action, prob = self.brain.get_action(obs, mask)
        return action, exp(float(prob))

    def get_observations(self):
        """The observation / action mask of this agent computed by the last
        ``Maze.reset()`` or ``Maze.step()`` (the kernel computes them there)."""
        i = self.maze._agent_index(self)
        return list(self.maze._obs[i]), list(self.maze._masks[i])

    # ------------------------------------------------------------------
    def _rec(self):
        if self.maze is None or self.maze._agent_rec is None:
            return None
        return self.maze._agent_rec[self.maze._agent_index(self)]

    def _flag(self, bit):
        r = self._rec()
        return bool(int(r["flags"]) & bit) if r is not None else False

    @property
    def x(self):
        r = self._rec()
        return int(r["x"]) if r is not None else 0

    @property
    def y(self):
        r = self._rec()
        return int(r["y"]) if r is not None else 0

    @property
    def direction(self):
        r = self._rec()
        return int(r["dir"]) if r is not None else 2

    @property
    def has_key(self):
        return self._flag(_lib.AF_HAS_KEY)

    @property
    def team_has_key(self):
        return self._flag(_lib.AF_TEAM_KEY)

    @property
    def knows_end(self):
        return self._flag(_lib.AF_KNOWS_END)

    @property
    def other_knows_end(self):
        return self._flag(_lib.AF_OTHER_KNOWS)

    @property
    def sees_end(self):
        return self._flag(_lib.AF_SEES_END)

    @property
    def sees_key(self):
        return self._flag(_lib.AF_SEES_KEY)

    @property
    def exit_len(self):
        r = self._rec()
        return int(r["exit_len"]) if r is not None else -1

    @property
    def time_from_last_seen(self):
        r = self._rec()
        return int(r["tfls"]) if r is not None else 0

    @property
    def last_mark_pos(self):
        r = self._rec()
        if r is None or not (int(r["flags"]) & _lib.AF_HAS_MARK):
            return None
        return (int(r["lmx"]), int(r["lmy"]))

    @property
    def other_last_seen(self):
        r = self._rec()
        return (int(r["olsx"]), int(r["olsy"])) if r is not None else None

    @property
    def min_x_visited(self):
        r = self._rec()
        return int(r["minx"]) if r is not None else 0

    @property
    def max_x_visited(self):
        r = self._rec()
        return int(r["maxx"]) if r is not None else 0

    @property
    def min_y_visited(self):
        r = self._rec()
        return int(r["miny"]) if r is not None else 0

    @property
    def max_y_visited(self):
        r = self._rec()
        return int(r["maxy"]) if r is not None else 0

    @property
    def width_estimate(self):  # update_maze_dims (maze_agent.py:330-336)
        return max(1, self.max_x_visited - self.min_x_visited)

    @property
    def height_estimate(self):
        return max(1, self.max_y_visited - self.min_y_visited)

    @property
    def memory(self):
        """deque(maxlen=4) of the last relative moves, -1 = empty (maze_agent.py:54)."""
        r = self._rec()
        vals = [int(v) for v in r["mem"]] if r is not None else [-1, -1, -1, -1]
        return deque(vals, maxlen=4)

    @property
    def exit_route(self):
        """The reference's route stack (maze.py:148-154): directions back from
        the exit, top = next move.  It always equals the tree path to the exit."""
        if not self.knows_end:
            return None
        env = self.maze._env
        dirs = env.exit_dirs(0)
        x, y, route = self.x, self.y, []
        while dirs[y, x] != 4 and len(route) <= dirs.size:
            d = int(dirs[y, x])
            route.append(d)
            x, y = x + DELTAS[d][0], y + DELTAS[d][1]
        return list(reversed(route))

    @property
    def next_move_to_exit(self):
        """One-hot of the relative next move toward the exit (maze_agent.py:113-118)."""
        route = self.exit_route
        if not route:  # unknown or empty route
            return [1, 1, 1, 1]
        out = [0, 0, 0, 0]
        out[(route[-1] - self.direction) % 4] = 1
        return out
