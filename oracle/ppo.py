"""CPU restatement of the reference PPO path (TEST ORACLE ONLY; see oracle/__init__.py).

Restates, on the CPU in fp32:

* ``gae_fp32``            -- ``PPO.get_GAEs`` (PPO.py:193-203), numpy fp32;
  ``gae_bootstrap_fp32`` the same recursion with a bootstrapped open segment.
* ``OActor`` / ``OCritic`` -- ``networks.py:13-106`` with the reference's
  module/parameter names, init order and the Projection quirk (Q1: every
  feature embedding reads ``x[:, 0:d_i]``, networks.py:59-63).
* ``log_probs``           -- ``PPO.get_log_probs`` (PPO.py:154-168).
* ``update_epoch``        -- the update body of ``PPO.train`` (PPO.py:46-85,
  216-220), teacher-forced on a recorded batch and shuffle.
* ``CpuPPOPort``          -- a single-maze ``PPO.train()`` port (rollout with
  one actor call per agent per step, PPO.py:89-152, then the update), used by
  ``bench.py`` as the timed CPU baseline.  Its environment is the C oracle.

Pinned by tests/golden/{gae,nets,train_small,ckpt_logits}.npz.
"""
import math

import numpy as np
import torch
import torch.nn as nn

FEATURE_DIMS = [4, 4, 4, 4, 4, 4, 4, 4, 4, 4, 4, 4, 2, 2, 1, 4, 1, 1, 1, 1, 1, 1, 2]  # networks.py:8
OBS = 65
EMB = 20


# ----------------------------------------------------------------------------
# GAE (PPO.py:193-203) -- fp32 arithmetic exactly as torch performs it
# ----------------------------------------------------------------------------
def gae_fp32(rew, val, done, gamma=0.99, lam=0.95):
    """rew: python floats; val: f32; done: bool.  Returns f32 advantages.

    delta = (r + f32(gamma)*V[t+1]*(1-d[t+1])) - V[t]   (t < L-1)
    delta = r - V[t]                                     (t = L-1)
    A     = delta + f32(gamma*lam)*(1-d[t])*A[t+1]
    """
    f = np.float32
    g = f(gamma)
    gl = f(gamma * lam)  # python float product, cast once (PPO.py:201)
    L = len(rew)
    out = np.zeros(L, np.float32)
    adv = f(0.0)
    for t in range(L - 1, -1, -1):
        v = f(val[t])
        if t + 1 == L:
            delta = f(f(rew[t]) - v)
        else:
            boot = f(g * f(val[t + 1]))
            if done[t + 1]:
                boot = f(boot * f(0.0))
            delta = f(f(f(rew[t]) + boot) - v)
        scale = f(0.0) if done[t] else gl
        adv = f(delta + f(scale * adv))
        out[t] = adv
    return out


def gae_bootstrap_fp32(rew, val, done, last_val, gamma=0.99, lam=0.95):
    """One env's fixed-horizon fragment [T] whose last segment may end mid-episode:
    the recursion of ``gae_fp32`` (PPO.py:193-203) run backwards over the whole
    fragment, an episode end (done[t]) cutting it as the reference's per-episode
    call does, and the open last segment bootstrapped with V(s_T) = last_val
    (delta = r + gamma V(s_T) - V(s_{T-1})).  Inside an episode the next value
    is zeroed when the next step is the episode's last (the reference's
    (1 - d[t+1]) factor, PPO.py:200).  No reference counterpart: the reference
    only ever cuts at episode ends (its last fragment is treated as terminal).
    Same fp32 operation order as ``gae_fp32`` step for step."""
    f = np.float32
    g = f(gamma)
    gl = f(gamma * lam)
    L = len(rew)
    out = np.zeros(L, np.float32)
    adv = f(0.0)
    for t in range(L - 1, -1, -1):
        v = f(val[t])
        if done[t]:
            delta = f(f(rew[t]) - v)
        else:
            boot = f(g * f(last_val)) if t + 1 == L else f(g * f(val[t + 1]))
            if t + 1 < L and done[t + 1]:
                boot = f(boot * f(0.0))
            delta = f(f(f(rew[t]) + boot) - v)
        scale = f(0.0) if done[t] else gl
        adv = f(delta + f(scale * adv))
        out[t] = adv
    return out


# ----------------------------------------------------------------------------
# networks (networks.py)
# ----------------------------------------------------------------------------
class OProjection(nn.Module):
    def __init__(self, parity=True):
        super().__init__()
        self.layers = nn.ModuleList([nn.Linear(d, EMB) for d in FEATURE_DIMS])
        self.parity = parity

    def forward(self, x):
        # networks.py:58-65 -- the slice start never advances (Q1).  parity=False is NOT the
        # reference: each feature reads its own slice x[:, s_i:s_i + d_i], s_i = sum of the earlier
        # widths -- what the code evidently intended (the product's parity_mode=False); it has no
        # reference counterpart to pin it, so tests use it only against the product.
        starts = [0] * len(FEATURE_DIMS) if self.parity else list(np.cumsum([0] + FEATURE_DIMS[:-1]))
        outs = [lin(x[:, s:s + d]) for lin, d, s in zip(self.layers, FEATURE_DIMS, starts)]
        return torch.cat(outs, dim=1).reshape(-1, len(FEATURE_DIMS), EMB)


class OAttention(nn.Module):
    def __init__(self, kq=10):
        super().__init__()
        self.kq_dim = kq
        self.keys = nn.Linear(EMB, kq, bias=False)
        self.querys = nn.Linear(EMB, kq, bias=False)
        self.values = nn.Linear(EMB, EMB, bias=False)

    def forward(self, h):  # networks.py:75-82
        k, q, v = self.keys(h), self.querys(h), self.values(h)
        logits = torch.einsum("bij,bkj->bik", q, k) / np.sqrt(self.kq_dim)
        w = torch.softmax(logits, dim=-1)
        ctx = torch.einsum("bij,bjk->bik", w, v)
        return (h + ctx).reshape(-1, len(FEATURE_DIMS) * EMB)


class OActor(nn.Module):
    def __init__(self, hidden=(264, 264, 264), parity=True):
        super().__init__()
        self.projection = OProjection(parity)
        self.attention = OAttention()
        sizes = [len(FEATURE_DIMS) * EMB] + list(hidden)
        self.layers = nn.ModuleList([nn.Linear(a, b) for a, b in zip(sizes[:-1], sizes[1:])])
        self.move_head = nn.Linear(hidden[-1], 5)
        self.mark_head = nn.Linear(hidden[-1], 1)
        for lin in self.layers:  # networks.py:43-48
            nn.init.orthogonal_(lin.weight)
        with torch.no_grad():
            self.move_head.weight *= 0.01
            self.mark_head.weight *= 0.01

    def forward(self, x, relu_masks=None):  # networks.py:31-41
        """relu_masks (tests only, no reference counterpart): per hidden layer a bool
        [rows, width] pattern replacing ReLU by the linear map on that pattern --
        the network linearised at another evaluation's ReLU pattern (a ReLU whose
        input is within rounding of 0 may fall on either side under a different
        summation order)."""
        x = torch.as_tensor(x, dtype=self.move_head.weight.dtype).reshape(-1, OBS)
        x = self.attention(self.projection(x))
        for l, lin in enumerate(self.layers):
            x = torch.relu(lin(x)) if relu_masks is None else lin(x) * relu_masks[l].to(x.dtype)
        return [self.move_head(x), self.mark_head(x)]


class OCritic(nn.Module):
    def __init__(self, agents=2, hidden=(64, 64)):
        super().__init__()
        self.agent_amount = agents
        sizes = [agents * OBS] + list(hidden) + [1]
        self.layers = nn.ModuleList([nn.Linear(a, b) for a, b in zip(sizes[:-1], sizes[1:])])
        for lin in self.layers:  # networks.py:104-106
            nn.init.orthogonal_(lin.weight)

    def forward(self, x, relu_masks=None):  # networks.py:96-102 (relu_masks: as OActor.forward)
        x = torch.as_tensor(x, dtype=self.layers[0].weight.dtype).reshape(-1, self.agent_amount * OBS)
        for l, lin in enumerate(self.layers[:-1]):
            x = torch.relu(lin(x)) if relu_masks is None else lin(x) * relu_masks[l].to(x.dtype)
        return self.layers[-1](x)


def make_nets(seed=3234):
    """Actor + Critic initialised as right after ``PPO.py:7`` (seed 3234)."""
    torch.manual_seed(seed)
    return OActor(), OCritic()


# ----------------------------------------------------------------------------
# PPO pieces
# ----------------------------------------------------------------------------
def log_probs(actor, i, obs, act, masks, relu_masks=None):
    """PPO.get_log_probs (PPO.py:154-168).  relu_masks: the actor's patterns over
    the interleaved [2M] agent rows (row 2m + i), see OActor.forward."""
    moves, marks = act[:, i, 0], act[:, i, 1]
    ml, kl = actor(obs[:, i, :]) if relu_masks is None else actor(obs[:, i, :], [m[i::2] for m in relu_masks])
    ml = ml.masked_fill(~masks[:, i, 0:5], float("-inf"))
    lp_move = torch.distributions.Categorical(logits=ml).log_prob(moves)
    kl = kl.squeeze().masked_fill(~masks[:, i, 5], float("-inf"))
    p = torch.sigmoid(kl)
    p = torch.where(marks.to(torch.bool), p, 1 - p)
    return lp_move + torch.log(p)


def minibatch_grads(actor, critic, obs, act, old_lp, adv, rtg, masks, clip=0.2, patterns=None):
    """The two losses of PPO.py:62-80 and their gradients (before clip_grad_norm_
    and Adam).  Returns (actor_loss, critic_loss, {name: actor grad},
    {name: critic grad}); works for fp32 or fp64 modules (inputs are cast).
    patterns: optional (actor relu masks, critic relu masks), see OActor.forward."""
    dt = next(actor.parameters()).dtype
    obs, adv, rtg, old_lp = (t.to(dt) for t in (obs, adv, rtg, old_lp))
    pa, pc = patterns if patterns is not None else (None, None)
    V = critic(obs, pc).squeeze()
    cur = 0
    for i in range(2):
        cur = cur + log_probs(actor, i, obs, act, masks, pa)
    ratio = torch.exp(cur - old_lp)
    aloss = -torch.mean(torch.min(ratio * adv, torch.clamp(ratio, 1 - clip, 1 + clip) * adv))
    closs = torch.nn.MSELoss()(V, rtg)
    ga = torch.autograd.grad(aloss, list(actor.parameters()))
    gc = torch.autograd.grad(closs, list(critic.parameters()))
    return (float(aloss.detach()), float(closs.detach()), {k: g for (k, _), g in zip(actor.named_parameters(), ga)},
            {k: g for (k, _), g in zip(critic.named_parameters(), gc)})


def minibatch_step(actor, critic, aopt, copt, obs, act, old_lp, adv, rtg, masks,
                   clip=0.2, max_grad=0.5, patterns=None):
    """One iteration of PPO.py:58-85.  Returns (actor_loss, critic_loss, gn_a, gn_c).
    patterns: as minibatch_grads."""
    pa, pc = patterns if patterns is not None else (None, None)
    V = critic(obs, pc).squeeze()
    cur = 0
    for i in range(2):
        cur = cur + log_probs(actor, i, obs, act, masks, pa)
    ratio = torch.exp(cur - old_lp)
    s1 = ratio * adv
    s2 = torch.clamp(ratio, 1 - clip, 1 + clip) * adv
    aloss = -torch.mean(torch.min(s1, s2))
    aopt.zero_grad()
    aloss.backward()
    gna = torch.nn.utils.clip_grad_norm_(actor.parameters(), max_grad)
    aopt.step()
    closs = torch.nn.MSELoss()(V, rtg)
    copt.zero_grad()
    closs.backward()
    gnc = torch.nn.utils.clip_grad_norm_(critic.parameters(), max_grad)
    copt.step()
    return float(aloss.detach()), float(closs.detach()), float(gna), float(gnc)


def update_epoch(actor, critic, aopt, copt, b_obs, b_act, b_lp, b_masks, b_advs, b_vals,
                 index_list, batch_size, updates=5, clip=0.2, max_grad=0.5):
    """Update body of PPO.train (PPO.py:46-85) given the shuffle ``index_list``."""
    b_rtgs = b_advs + b_vals
    b_advs = (b_advs - torch.mean(b_advs)) / (torch.std(b_advs) + 1e-10)
    mb = batch_size // 5
    hist = []
    for _ in range(updates):
        for opt in (aopt, copt):  # decay_lr PPO.py:216-220
            for g in opt.param_groups:
                g["lr"] *= 0.997
        for start in range(0, batch_size, mb):
            idx = index_list[start:start + mb]
            hist.append(minibatch_step(actor, critic, aopt, copt, b_obs[idx], b_act[idx], b_lp[idx],
                                       b_advs[idx], b_rtgs[idx], b_masks[idx], clip, max_grad))
    return hist


# ----------------------------------------------------------------------------
# single-maze train() port (CPU baseline)
# ----------------------------------------------------------------------------
class CpuPPOPort:
    """PPO.train() on one maze, one step at a time, as the reference runs it.

    Rollout: per step one critic call on both observations and one actor call
    per agent (PPO.py:108-141); masked-Categorical + Bernoulli sampling
    (PPO.py:170-186; the per-step print of PPO.py:185 is not restated).
    The environment is the C oracle (``oracle.env.OracleEnv``).
    """

    def __init__(self, env, batch_size=15000, lr=1.4e-4, seed=3234):
        self.env = env
        self.batch_size = batch_size
        self.actor, self.critic = make_nets(seed)
        self.aopt = torch.optim.Adam(self.actor.parameters(), lr=lr)
        self.copt = torch.optim.Adam(self.critic.parameters(), lr=lr)

    def _act(self, obs, mask):
        ml, kl = self.actor(obs)
        ml = torch.where(torch.as_tensor(mask[0:5]), ml, torch.tensor(-math.inf))
        dist = torch.distributions.Categorical(logits=ml)
        move = dist.sample()
        p = torch.sigmoid(kl) if mask[5] else torch.zeros((1, 1))
        mark = torch.bernoulli(p)
        p = p if mark == 1 else 1 - p
        return [int(move.item()), int(mark.item())], dist.log_prob(move) + torch.log(p)

    def get_batch(self, max_steps=None):
        """Returns (steps, batch) where batch mirrors PPO.get_batch's tensors."""
        obs, masks = self.env.reset(0)
        B_obs, B_act, B_lp, B_mask, B_adv, B_val = [], [], [], [], [], []
        ep_r, ep_v, ep_d = [], [], []
        total = 0
        with torch.no_grad():
            while True:
                B_obs.append(obs)
                B_mask.append(masks)
                ep_v.append(float(self.critic(obs)))
                acts, lp = [], 0
                for i in range(2):
                    a, l = self._act(obs[i], masks[i])
                    acts.append(a)
                    lp = lp + l
                obs, masks, r, d = self.env.step(0, acts)
                B_act.append(acts)
                B_lp.append(float(lp.sum()))
                ep_r.append(r)
                ep_d.append(d)
                total += 1
                stop = max_steps is not None and total >= max_steps
                if d or stop:
                    if d:
                        obs, masks = self.env.reset(0)
                    B_val.extend(ep_v)
                    B_adv.extend(gae_fp32(ep_r, np.asarray(ep_v, np.float32), ep_d))
                    ep_r, ep_v, ep_d = [], [], []
                    if total > self.batch_size or stop:
                        break
        batch = (torch.as_tensor(np.asarray(B_obs), dtype=torch.float32),
                 torch.as_tensor(np.asarray(B_act), dtype=torch.float32),
                 torch.as_tensor(B_lp, dtype=torch.float32),
                 torch.as_tensor(np.asarray(B_mask), dtype=torch.bool),
                 torch.as_tensor(np.asarray(B_adv), dtype=torch.float32),
                 torch.as_tensor(B_val, dtype=torch.float32))
        return total, batch

    def update(self, batch, updates=5):
        b_obs, b_act, b_lp, b_mask, b_adv, b_val = batch
        idx = np.arange(len(b_obs))
        np.random.shuffle(idx)
        bs = min(self.batch_size, len(b_obs))
        hist = update_epoch(self.actor, self.critic, self.aopt, self.copt, b_obs, b_act, b_lp,
                            b_mask, b_adv, b_val, idx, bs, updates=updates)
        return hist
