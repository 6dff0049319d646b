import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "marl-maze_amd"))
import numpy as np, torch
from marlmaze.vecmaze import VecMaze
g = np.load('tests/golden/maze_gen.npz')
ks = np.nonzero((g['case']==0)&(g['reset']==0))[0]
env = VecMaze(len(ks), default_size=(4,4), max_timestep=1200, seeds=[int(g['seed'][k]) for k in ks])
obs, masks = env.reset()
obs = obs.cpu().numpy(); masks = masks.cpu().numpy()
for j,k in enumerate(ks):
    d = np.nonzero(obs[j] != g['obs'][k])
    print(j, 'obs diff idx', list(zip(*d)), 'gpu', obs[j][d], 'ref', g['obs'][k][d], 'mask gpu', masks[j].astype(int).tolist(), 'ref', g['masks'][k].astype(int).tolist())
    print('  layout raw', env.layout[j, :49].cpu().numpy().reshape(7,7).tolist())
    print('  agents', env.agent_state(j).tolist())
