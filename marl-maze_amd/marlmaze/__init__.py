"""marlmaze -- MI355X-native hot path of rhuangr/MARL-Maze.

Reference-compatible API (drop-in for training):
  from marlmaze.maze import Maze            # maze.py:21
  from marlmaze.maze_agent import Agent     # maze_agent.py:15
  from marlmaze.PPO import PPO              # PPO.py:11
  from marlmaze.networks import Actor, Critic   # networks.py:13,84
Batched GPU environment:
  from marlmaze.vecmaze import VecMaze
"""
__version__ = "0.1.0"
