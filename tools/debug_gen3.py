import sys, os, shutil
sys.path.insert(0, "marl-maze_amd")
shutil.copy("marl-maze_amd/libmarlmaze_dbg.so", "marl-maze_amd/libmarlmaze.so")
import numpy as np, torch
from marlmaze.vecmaze import VecMaze
env = VecMaze(5, default_size=(4,4), max_timestep=1200, seeds=[0,1,7,12345,2**32+5])
env.reset()
r = env.maze_info()["reserved"]
for x in r: print("nb", x & 15, "w", (x>>4)&63, "h", (x>>10)&63, "cell", (x>>16)&255, "open", (x>>24)&1, "inb", (x>>25)&1)
