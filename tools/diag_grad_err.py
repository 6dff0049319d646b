"""Diagnostic: per-tensor gradient error (relative to the tensor's max) of the
GPU update path vs an fp64 evaluation of the oracle, split by stage:
  cpu32  -- the fp32 oracle on the CPU
  gpu    -- PPO.minibatch_grads (x3 trunk for >= 16,384 actor rows)
  front  -- the fused front-end backward alone, fed the fp64 dh (rounded to fp32)
Usage: python tools/diag_grad_err.py [S]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "marl-maze_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from marlmaze.PPO import PPO  # noqa: E402
from marlmaze.networks import _FusedFront, front_params  # noqa: E402
from oracle import ppo as oppo  # noqa: E402

S = int(sys.argv[1]) if len(sys.argv) > 1 else 32768
n = np.load(os.path.join(REPO, "tests/golden/nets.npz"))


def nets(dt):
    a, c = oppo.OActor(), oppo.OCritic()
    a.load_state_dict({k[6:]: torch.as_tensor(n[k]) for k in n.files if k.startswith("actor/")})
    c.load_state_dict({k[7:]: torch.as_tensor(n[k]) for k in n.files if k.startswith("critic/")})
    return a.to(dt), c.to(dt)


g = torch.Generator().manual_seed(S)
idx = torch.arange(S) % 256
batch = (torch.as_tensor(n["obs"])[idx], torch.as_tensor(n["actions"])[idx],
         torch.as_tensor(n["old_logp"])[idx] + 0.3 * torch.randn(S, generator=g), torch.randn(S, generator=g),
         torch.randn(S, generator=g), torch.as_tensor(n["masks"])[idx])
if len(sys.argv) > 2 and sys.argv[2] == "random":  # independent rows: random obs in the fixture's value range
    o = batch[0].clone()
    o[..., :4] = torch.rand(S, 2, 4, generator=g).round()
    batch = (o,) + batch[1:]
if len(sys.argv) > 2 and sys.argv[2] == "facing":  # rollout-like: obs[0:4] = facing one-hot (4 distinct actor inputs)
    o = batch[0].clone()
    o[..., :4] = torch.nn.functional.one_hot(torch.randint(0, 4, (S, 2), generator=g), 4).float()
    batch = (o,) + batch[1:]
r64 = oppo.minibatch_grads(*nets(torch.float64), *batch)
r32 = oppo.minibatch_grads(*nets(torch.float32), *batch)
ag = PPO(2, n_envs=64, load=False, verbose=False, save=False)
a32, c32 = nets(torch.float32)
ag.actor.load_state_dict({k: v.cuda() for k, v in a32.state_dict().items()})
ag.critic.load_state_dict({k: v.cuda() for k, v in c32.state_dict().items()})
ag.minibatch_grads(*(t.cuda() for t in batch))
gpu = ({k: p.grad.cpu() for k, p in ag.actor.named_parameters()},
       {k: p.grad.cpu() for k, p in ag.critic.named_parameters()})

# front-end alone with the fp64 dh
a64, _ = nets(torch.float64)
x = batch[0].reshape(-1, 65).double()
h = a64.attention(a64.projection(x)).detach().requires_grad_(True)
hh = h
for lin in a64.layers:
    hh = torch.relu(lin(hh))
# dh of the actor loss: rebuild the loss from h
ml, kl = a64.move_head(hh), a64.mark_head(hh)
# reuse log_probs through a wrapper actor that starts at h
from oracle.ppo import log_probs  # noqa: E402


class FromH(torch.nn.Module):
    def forward(self, _):
        return [ml, kl]


cur = 0
mk, act = batch[5], batch[1]
M = S
mlr, klr = ml.view(M, 2, 5), kl.view(M, 2, 1)
for i in range(2):
    m_i = mlr[:, i].masked_fill(~mk[:, i, 0:5], float("-inf"))
    lpm = torch.distributions.Categorical(logits=m_i).log_prob(act[:, i, 0])
    k_i = klr[:, i].squeeze().masked_fill(~mk[:, i, 5], float("-inf"))
    p = torch.sigmoid(k_i)
    p = torch.where(act[:, i, 1].to(torch.bool), p, 1 - p)
    cur = cur + lpm + torch.log(p)
ratio = torch.exp(cur - batch[2].double())
adv = batch[3].double()
aloss = -torch.mean(torch.min(ratio * adv, torch.clamp(ratio, 0.8, 1.2) * adv))
dh, = torch.autograd.grad(aloss, h)
params = front_params(ag.actor.projection, ag.actor.attention)
xg = x.float().cuda()
hf = _FusedFront.apply(xg, True, *params)
fg = torch.autograd.grad(hf, params, dh.float().cuda())
names = ([f"projection.layers.{i}.weight" for i in range(23)] + [f"projection.layers.{i}.bias" for i in range(23)] +
         ["attention.querys.weight", "attention.keys.weight", "attention.values.weight"])
front = dict(zip(names, [t.cpu() for t in fg]))

print(f"S={S}  per-tensor max|err| / max|g64|")
print(f"{'tensor':36s} {'max|g|':>10s} {'cpu32':>9s} {'gpu':>9s} {'front':>9s}")
for d64, d32, dg, tag in ((r64[2], r32[2], gpu[0], "actor"), (r64[3], r32[3], gpu[1], "critic")):
    for k in d64:
        s = d64[k].abs().max().item()
        e32 = (d32[k].double() - d64[k]).abs().max().item() / s
        eg = (dg[k].double() - d64[k]).abs().max().item() / s
        ef = (front[k].double() - d64[k]).abs().max().item() / s if k in front else float("nan")
        flag = " <" if max(eg, 0 if ef != ef else ef) > 1e-5 else ""
        print(f"{tag + '.' + k:36s} {s:10.3e} {e32:9.2e} {eg:9.2e} {ef:9.2e}{flag}")

# actor backward on the GPU fed the fp64 d loss / d head logits (isolates the loss kernels)
ml64, kl64 = a64(x)
z = torch.cat([ml64, kl64], 1).detach().requires_grad_(True)
mlz, klz = z[:, :5].view(M, 2, 5), z[:, 5:6].view(M, 2, 1)
cur = 0
for i in range(2):
    m_i = mlz[:, i].masked_fill(~mk[:, i, 0:5], float("-inf"))
    lpm = torch.distributions.Categorical(logits=m_i).log_prob(act[:, i, 0])
    k_i = klz[:, i].squeeze().masked_fill(~mk[:, i, 5], float("-inf"))
    p = torch.sigmoid(k_i)
    p = torch.where(act[:, i, 1].to(torch.bool), p, 1 - p)
    cur = cur + lpm + torch.log(p)
ratio = torch.exp(cur - batch[2].double())
aloss = -torch.mean(torch.min(ratio * adv, torch.clamp(ratio, 0.8, 1.2) * adv))
dz, = torch.autograd.grad(aloss, z)
for p_ in ag.actor.parameters():
    p_.grad = None
zg = ag.actor.logits(xg)
zg.backward(dz.float().cuda())
print("actor backward fed the fp64 dz (max|err| / max|g64|)")
for k, p_ in ag.actor.named_parameters():
    s = r64[2][k].abs().max().item()
    e = (p_.grad.cpu().double() - r64[2][k]).abs().max().item() / s
    if e > 1e-6:
        print(f"  {k:34s} {e:9.2e}")
