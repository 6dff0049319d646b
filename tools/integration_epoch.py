"""INTEGRATION.md section 1 run as written (the reference's main.py with the
imports swapped), for one training epoch: PPO(agent_amount=2,
batch_size=15000, lr=0.00014) with main.py's Maze configuration (12-13-cell
random sizes, random starts).  Used under rocprofv3 to show that every kernel
of the drop-in's epoch is hand-written (no library GEMM).  The agents' colours
are plain tuples here (pygame is not needed by the GPU path)."""
import os
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "marl-maze_amd"))
os.chdir(tempfile.mkdtemp())  # PPO.pth is CWD-relative (PPO.py:9): start without one

from marlmaze.maze import Maze  # noqa: E402
from marlmaze.maze_agent import Agent  # noqa: E402
from marlmaze.PPO import PPO  # noqa: E402

RED, PALE_RED, BLUE, PALE_BLUE = (255, 0, 0), (219, 112, 147), (72, 118, 255), (151, 255, 255)
brain = PPO(agent_amount=2, batch_size=15000, lr=0.00014)
agents = (Agent('RED', brain, RED, PALE_RED, 2),
          Agent('BLUE', brain, BLUE, PALE_BLUE, 3))
maze = Maze(agents=agents, max_timestep=1200, rand_sizes=True, rand_range=[12, 13], rand_start=True, difficulty=1,
            default_size=[4, 4])
brain.epochs = 1
brain.train()
print("epoch done:", brain.history[-1])
