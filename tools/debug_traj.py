import sys; sys.path.insert(0, "marl-maze_amd")
import numpy as np, torch
from marlmaze.vecmaze import VecMaze
t = np.load("tests/golden/env_traj.npz")
name = sys.argv[1] if len(sys.argv) > 1 else "s4_t60"
auto = int(sys.argv[2]) if len(sys.argv) > 2 else 0
cfg = t[name + "/cfg"]
env = VecMaze(1, default_size=(int(cfg[0]), int(cfg[1])), max_timestep=int(cfg[2]), difficulty=int(cfg[3]),
              rand_start=bool(cfg[4]), rand_sizes=bool(cfg[5]), rand_range=(int(cfg[6]), int(cfg[7])), seeds=[int(cfg[8])])
env.reset()
A = torch.as_tensor(t[name + "/actions"]).cuda()
for s in range(len(A)):
    prev_state = env.agent_state(0)
    obs, masks, r, d = env.step(A[s:s + 1], auto_reset=auto)
    if not auto and bool(d[0]):
        env.reset(d)
    o = obs.cpu().numpy()[0]
    if not np.array_equal(o, t[name + "/obs"][s]):
        idx = np.nonzero(o != t[name + "/obs"][s])
        print("step", s, "diff idx", list(zip(*idx)), "gpu", o[idx], "ref", t[name + "/obs"][s][idx])
        print("prev state", prev_state.tolist()); print("state", env.agent_state(0).tolist()); print("ref state", t[name + "/astate"][s].tolist())
        print("act", A[s].tolist(), "done", bool(d[0]), "ref done", t[name + "/done"][s])
        print("layout", env.layouts()[0].tolist())
        break
else:
    print("all ok")
