import sys, os
sys.path.insert(0, "marl-maze_amd"); sys.path.insert(0, ".")
import numpy as np, torch
from marlmaze.PPO import PPO
ag = PPO(2, n_envs=512, horizon=40, batch_size=20480, bootstrap=False, sample_seed=5, load=False, verbose=False, save=False,
         env_config=dict(default_size=(6, 6), max_timestep=30, seed_base=100))
b = ag.rollout()
T, n = 40, 512
obs = b["obs"][:T].reshape(-1, 65); masks = b["masks"][:T].reshape(-1, 6).bool(); act = b["act"].reshape(-1, 2)
with torch.no_grad():
    ml, kl = ag.actor(obs)
mlm = ml.masked_fill(~masks[:, :5], float("-inf"))
lpm = torch.log_softmax(mlm, -1).gather(1, act[:, 0:1].long()).squeeze(1)
p = torch.sigmoid(kl.squeeze(1).masked_fill(~masks[:, 5], float("-inf")))
lpk = torch.log(torch.where(act[:, 1] != 0, p, 1 - p))
row = b["rowlogp"].reshape(-1)
ref = lpm + lpk
bad = (row - ref).abs() > 1e-4
print("rows", row.numel(), "bad", int(bad.sum()))
idx = torch.nonzero(bad).view(-1)[:8]
for i in idx.tolist():
    print(i, "row", row[i].item(), "ref", ref[i].item(), "move lp", lpm[i].item(), "mark lp", lpk[i].item(), "act", act[i].tolist(), "mask", masks[i].int().tolist(), "ml", [round(x, 4) for x in ml[i].tolist()], "kl", kl[i].item())
# also: recompute the rollout-time logits for step 0 with the same batch size
with torch.no_grad():
    ml0, kl0 = ag.actor(b["obs"][0].reshape(-1, 65))
print("logit diff batch-size", (ml0 - ml[:2 * n]).abs().max().item())
