"""GPU parity of the PPO update against the pinned oracle (oracle/ppo.py,
bit-exact to the reference's own update on tests/golden/nets.npz and
train_small.npz at 4 threads -- see test_oracle_golden.py).

The bar (BASELINE north star): 1e-5 relative.  Stated per quantity:

* losses and clipped-gradient norms vs the fp32 oracle:
  |got - ref| <= 1e-5 |ref| + 1e-6 (the actor loss of a normalised advantage
  batch is ~0, hence the absolute floor);
* gradients, per parameter tensor, before clipping / all-reduce / Adam:
  max|g - g_ref| <= 1e-5 max|g_ref|, where g_ref is the oracle evaluated in
  fp64.  The fp32 oracle (= the reference's own arithmetic) is NOT within that
  bar of the exact gradient for the attention weights: their per-sample terms
  cancel ~100:1 over the minibatch, and torch-CPU fp32 lands 1.2e-5..2.8e-5
  of max|g| away from fp64 there (tools/diag_grad_err.py).  On such a tensor
  the bound is twice the reference's own fp32 error instead.
  BASELINE configs[1]'s rollout minibatch is held to the same 1e-5.  There the
  actor sees only the 4 facing one-hots (Q1), every gradient sum over the
  26,214 rows collapses onto 4 activation vectors, and rounding that is
  coherent across rows does not average out: in round 3 one tensor,
  projection.layers.0.bias, landed at 1.27e-5 of max|g| (its gradient f_0 +
  Wqkv^T e_0 cancels).  The front-end's partial sums are now reduced and
  combined in fp64 (k_front_sum / k_front_combine), and the trunk runs on the
  x2 arithmetic: no tensor is above 1e-5.
* the Adam step, per parameter tensor: Delta p = p_after - p_before agrees
  with the fp64 oracle's Adam step at 1e-5 lr + 1 ulp of the fp32 parameter
  wherever the clipped gradient is >= 1e-4 (Adam's first step is ~ -lr g/|g|,
  so entries with |g| near Adam's eps or near the gradient's rounding level
  may legitimately differ by up to 2 lr; a gradient with a flipped sign fails
  by 2 lr on every held entry).

Cases: the reference's one-update fixture (256 samples), a 32,768-sample
minibatch (65,536 actor rows: the bf16x3 MLP trunk and the split-K weight
gradients run; the fixture's 256 rows take neither), every minibatch of the
reference's recorded train() epoch with the oracle's parameters and Adam state
teacher-forced in before each step, and BASELINE configs[1] (4,096 mazes,
T=32: rollout replayed in the oracle on a column subset, then one
26,214-sample minibatch update), and the bench's own loop (horizon 16,
bootstrap=True: values, bootstrapped advantages and one minibatch update).
"""
import copy

import numpy as np
import pytest
import torch

from marlmaze.PPO import PPO
from oracle import ppo as oppo
from oracle.env import OracleEnv

pytestmark = pytest.mark.gpu

LR = 0.00014


def _agent(**kw):
    for k, v in dict(load=False, verbose=False, save=False, lr=LR).items():
        kw.setdefault(k, v)
    return PPO(2, **kw)


def _oracle_nets(fx, dtype=torch.float32, parity=True):
    a, c = oppo.OActor(parity=parity), oppo.OCritic()
    a.load_state_dict({k[6:]: torch.as_tensor(fx[k]) for k in fx.files if k.startswith("actor/")})
    c.load_state_dict({k[7:]: torch.as_tensor(fx[k]) for k in fx.files if k.startswith("critic/")})
    return a.to(dtype), c.to(dtype)


def _to_gpu(agent, actor, critic):
    agent.actor.load_state_dict({k: v.detach().cuda() for k, v in actor.state_dict().items()})
    agent.critic.load_state_dict({k: v.detach().cuda() for k, v in critic.state_dict().items()})


def _gpu_grads(agent):
    return ({k: p.grad.detach().cpu() for k, p in agent.actor.named_parameters()},
            {k: p.grad.detach().cpu() for k, p in agent.critic.named_parameters()})


def _close(got, ref, what):
    assert abs(got - ref) <= 1e-5 * abs(ref) + 1e-6, (what, got, ref)


def _check_grads(got, ref, tag, ref32=None, rel=1e-5):
    """Per tensor: max|g - g64| <= rel max|g64|, or -- for a tensor on which the
    reference's own fp32 arithmetic (ref32) is further than that from g64 -- no
    further from g64 than twice the reference's own error (see module doc)."""
    assert set(got) == set(ref)
    bad = []
    for k in ref:
        r = ref[k].double()
        scale = r.abs().max().item()
        err = (got[k].double() - r).abs().max().item()
        bound, err32 = rel * scale, float("nan")
        if ref32 is not None:
            err32 = (ref32[k].double() - r).abs().max().item()
            bound = max(bound, 2.0 * err32)
        if err > rel * scale:
            print(f"{tag} {k}: err {err / scale:.2e} of max|g|, fp32 oracle {err32 / scale:.2e}")
        if err > bound + 1e-12:
            bad.append((k, err / scale))
    assert not bad, (tag, bad)


def _check_delta(before, after, ref_before, ref_after, ref_grad, coef, tag, ulps=1.0):
    """Delta p of the GPU step vs the reference step's, per tensor (see module doc)."""
    for k in ref_grad:
        d_gpu = after[k].double() - before[k].double()
        d_ref = ref_after[k].double() - ref_before[k].double()
        sel = (ref_grad[k].double() * coef).abs() >= 1e-4
        assert (d_gpu - d_ref).abs().max().item() <= 2.0001 * LR, (tag, k)
        if sel.any():
            ulp = torch.as_tensor(np.spacing(np.abs(after[k].float().numpy())), dtype=torch.float64)
            excess = ((d_gpu - d_ref).abs() - 1e-5 * LR - ulps * ulp)[sel]
            assert excess.max().item() <= 0, (tag, k, excess.max().item(), int(sel.sum()), sel.numel())


def _minibatch(fx, S, noise=0.0):
    """S samples: the fixture's rows tiled, with fresh advantages, returns and
    old log-probs so that the rows differ; noise > 0 also perturbs every
    observation (so that every row -- not only the 256 fixture rows -- is a
    distinct input)."""
    if S == fx["obs"].shape[0] and not noise:
        return tuple(torch.as_tensor(fx[k]) for k in ("obs", "actions", "old_logp", "advs", "rtgs", "masks"))
    g = torch.Generator().manual_seed(S)
    idx = torch.arange(S) % fx["obs"].shape[0]
    old = torch.as_tensor(fx["old_logp"])[idx] + 0.3 * torch.randn(S, generator=g)
    obs = torch.as_tensor(fx["obs"])[idx]
    if noise:
        obs = obs + noise * torch.randn(obs.shape, generator=g)
    return (obs, torch.as_tensor(fx["actions"])[idx], old,
            torch.randn(S, generator=g), torch.randn(S, generator=g), torch.as_tensor(fx["masks"])[idx])


def _patterns(ag, batch, actor64, critic64):
    """The GPU forwards' ReLU patterns on this batch (actor rows interleaved 2m + i,
    critic rows m), after checking that every unit on which they differ from the
    fp64 oracle's own forward has a pre-activation within rounding of 0 (5e-6 of
    its layer's largest |pre-activation| in that row): a ReLU at ~0 may fall either
    way under any change of summation order, fp32 CPU torch included."""
    obs = batch[0]
    M = obs.shape[0]
    with torch.no_grad():
        _, (_, _, hs, _) = ag.actor.train_forward(obs.reshape(2 * M, 65).cuda())
        _, (chs, _) = ag.critic.train_forward(obs.reshape(M, -1).cuda())
        pa = [(h > 0).cpu() for h in hs[1:]]
        pc = [(h > 0).cpu() for h in chs[1:]]
        # fp64 pre-activations of the oracle's own forward
        x = obs.reshape(2 * M, 65).double()
        x = actor64.attention(actor64.projection(x))
        pres_a = []
        for lin in actor64.layers:
            x = lin(x)
            pres_a.append(x)
            x = torch.relu(x)
        y = obs.reshape(M, -1).double()
        pres_c = []
        for lin in critic64.layers[:-1]:
            y = lin(y)
            pres_c.append(y)
            y = torch.relu(y)
    flips = 0
    for pat, pre in list(zip(pa, pres_a)) + list(zip(pc, pres_c)):
        d = pat != (pre > 0)
        if d.any():
            rowmax = pre.abs().max(1, keepdim=True).values.expand_as(pre)
            assert (pre[d].abs() <= 5e-6 * rowmax[d]).all(), pre[d].abs().max().item()
            flips += int(d.sum())
    return (pa, pc), flips


def _step_and_compare(ag, actor, critic, batch, tag, grad_rel=1e-5):
    """Gradients, losses, norms and the Adam step of one minibatch, GPU vs oracle.
    The fp64 truth is evaluated at the GPU forward's ReLU pattern (_patterns); the
    reference's own fp32 arithmetic (ref32, the loosening bound) at its own."""
    actor64, critic64 = copy.deepcopy(actor).double(), copy.deepcopy(critic).double()
    pats, flips = _patterns(ag, batch, actor64, critic64)
    if flips:
        print(f"{tag}: {flips} ReLU units at ~0 differ from the fp64 oracle's pattern")
    ra, rc, rga32, rgc32 = oppo.minibatch_grads(actor, critic, *batch)
    _, _, rga, rgc = oppo.minibatch_grads(actor64, critic64, *batch, patterns=pats)
    if flips:  # the fp32 oracle's own error is measured against fp64 at its own pattern
        _, _, oga, ogc = oppo.minibatch_grads(actor64, critic64, *batch)
        rga32 = {k: v - oga[k] + rga[k] for k, v in rga32.items()}
        rgc32 = {k: v - ogc[k] + rgc[k] for k, v in rgc32.items()}
    gb = [t.cuda() for t in batch]
    al, cl = ag.minibatch_grads(*gb)
    _close(float(al), ra, tag + " actor loss")
    _close(float(cl), rc, tag + " critic loss")
    ga, gc = _gpu_grads(ag)
    _check_grads(ga, rga, tag + " actor", rga32, grad_rel)
    _check_grads(gc, rgc, tag + " critic", rgc32, grad_rel)
    # the whole step: clip_grad_norm_ + Adam, GPU vs the fp64 oracle
    before_a = {k: v.detach().cpu().clone() for k, v in ag.actor.state_dict().items()}
    before_c = {k: v.detach().cpu().clone() for k, v in ag.critic.state_dict().items()}
    rb_a = copy.deepcopy(actor64.state_dict())
    rb_c = copy.deepcopy(critic64.state_dict())
    aopt = torch.optim.Adam(actor64.parameters(), lr=LR)
    copt = torch.optim.Adam(critic64.parameters(), lr=LR)
    ref = oppo.minibatch_step(actor64, critic64, aopt, copt, *(t.double() if t.is_floating_point() else t
                                                               for t in batch), patterns=pats)
    got = [float(x) for x in ag.minibatch_step(*gb)]
    for g, r, w in zip(got, ref, ("aloss", "closs", "gnorm_a", "gnorm_c")):
        _close(g, r, f"{tag} {w}")
    ca = min(1.0, 0.5 / (ref[2] + 1e-6))  # clip_grad_norm_'s coefficient (max_grad 0.5)
    cc = min(1.0, 0.5 / (ref[3] + 1e-6))
    _check_delta(before_a, {k: v.cpu() for k, v in ag.actor.state_dict().items()}, rb_a, actor64.state_dict(), rga,
                 ca, tag + " actor")
    _check_delta(before_c, {k: v.cpu() for k, v in ag.critic.state_dict().items()}, rb_c, critic64.state_dict(), rgc,
                 cc, tag + " critic")


@pytest.mark.parametrize("S", [256, 32768])
def test_minibatch_gradients_and_step_match_oracle(golden, S):
    fx = golden("nets")
    ag = _agent(n_envs=64)
    actor, critic = _oracle_nets(fx)
    _to_gpu(ag, actor, critic)
    _step_and_compare(ag, actor, critic, _minibatch(fx, S), f"S={S}")


def test_one_update_matches_reference_fixture(golden):
    """actor_after / critic_after of the reference's own update (nets.npz) vs
    the GPU step, with the oracle's gradients deciding which entries are held
    to 1e-5 lr (see module doc)."""
    fx = golden("nets")
    ag = _agent(n_envs=64)
    actor, critic = _oracle_nets(fx)
    _to_gpu(ag, actor, critic)
    batch = _minibatch(fx, 256)
    _, _, rga, rgc = oppo.minibatch_grads(actor.double(), critic.double(), *batch)
    ag.minibatch_step(*(t.cuda() for t in batch))
    ca = min(1.0, 0.5 / (float(fx["actor_gnorm"]) + 1e-6))
    cc = min(1.0, 0.5 / (float(fx["critic_gnorm"]) + 1e-6))
    for net, pre, grads, coef in ((ag.actor, "actor", rga, ca), (ag.critic, "critic", rgc, cc)):
        before = {k: torch.as_tensor(fx[f"{pre}/{k}"]) for k in grads}
        after = {k: torch.as_tensor(fx[f"{pre}_after/{k}"]) for k in grads}
        # the fixture's own Delta p carries its fp32 rounding too: one more ulp
        _check_delta(before, {k: v.cpu() for k, v in net.state_dict().items()}, before, after, grads, coef, pre,
                     ulps=2.0)


def test_train_epoch_every_minibatch_teacher_forced(golden):
    """The reference's recorded train() epoch (train_small.npz: batch 600, 5 x 5
    minibatches of 120): before every GPU minibatch step the oracle's current
    parameters AND Adam state (moments, step, decayed lr) are loaded, so every
    one of the 25 steps is held to the 1e-5 bar, not only the first."""
    t = golden("train_small")
    fx = golden("nets")
    actor, critic = _oracle_nets(fx)
    aopt = torch.optim.Adam(actor.parameters(), lr=LR)
    copt = torch.optim.Adam(critic.parameters(), lr=LR)
    ag = _agent(n_envs=64, batch_size=600)
    b_obs, b_act, b_lp, b_masks, b_advs, b_vals = (torch.as_tensor(t[k]) for k in ("obs", "actions", "logp", "masks",
                                                                                     "advs", "vals"))
    b_rtgs = b_advs + b_vals  # PPO.py:46-47
    b_advs = (b_advs - torch.mean(b_advs)) / (torch.std(b_advs) + 1e-10)
    idx = t["idx"]
    mb = 600 // 5
    k = 0
    for _ in range(5):
        for opt in (aopt, copt):  # decay_lr, PPO.py:216-220
            for gr in opt.param_groups:
                gr["lr"] *= 0.997
        for start in range(0, 600, mb):
            sl = idx[start:start + mb]
            batch = (b_obs[sl], b_act[sl], b_lp[sl], b_advs[sl], b_rtgs[sl], b_masks[sl])
            _to_gpu(ag, actor, critic)
            ag.load_optim_state(ag.actor_optim, copy.deepcopy(aopt.state_dict()))
            ag.load_optim_state(ag.critic_optim, copy.deepcopy(copt.state_dict()))
            got = [float(x) for x in ag.minibatch_step(*(x.cuda() for x in batch))]
            ref = oppo.minibatch_step(actor, critic, aopt, copt, *batch)
            for g, r, w in zip(got, ref, ("aloss", "closs", "gnorm_a", "gnorm_c")):
                _close(g, r, f"minibatch {k} {w}")
            # the oracle is the reference here (bit-exact at 4 threads, test_oracle_golden.py)
            _close(ref[0], float(t["actor_loss"][k]), f"oracle minibatch {k}")
            _close(ref[1], float(t["critic_loss"][k]), f"oracle minibatch {k}")
            k += 1
    assert k == 25 and ag.actor_optim.param_groups[0]["lr"] == t["lr_final"]


def test_config1_rollout_and_update_4096_mazes(golden):
    """BASELINE configs[1]: 4,096 parallel 10x10 mazes, rollout of T=32 (131,072
    samples, bootstrap=False = the reference's per-episode GAE on every
    fragment), then one minibatch update of 131,072 // 5 = 26,214 samples.
    Every 16th maze column is replayed in the C oracle (bit-exact obs / masks /
    rewards / dones / advantages); the minibatch's gradients, losses, norms and
    Adam step are checked against the oracle."""
    n, T = 4096, 32
    cfg = dict(default_size=(10, 10), max_timestep=1200)
    ag = _agent(n_envs=n, horizon=T, batch_size=n * T, bootstrap=False, sample_seed=11,
                env_config=dict(cfg, seed_base=0))
    b = ag.rollout()
    cols = np.arange(0, n, 16)
    ora = OracleEnv(len(cols), seeds=cols.astype(np.uint64), **cfg)
    oo, om = ora.reset_all()
    obs = b["obs"].cpu().numpy()[:, cols]
    masks = b["masks"].cpu().numpy()[:, cols].astype(bool)
    act = b["act"].cpu().numpy()[:, cols]
    R = b["rew"].cpu().numpy()[:, cols]
    D = b["done"].cpu().numpy()[:, cols].astype(bool)
    assert np.array_equal(obs[0], oo) and np.array_equal(masks[0], om)
    for s in range(T):
        oo, om, orw, od = ora.step_all(act[s], auto_reset=True)
        assert np.array_equal(obs[s + 1], oo) and np.array_equal(masks[s + 1], om), s
        assert np.array_equal(R[s], orw) and np.array_equal(D[s], od), s
    V = b["val"].cpu().numpy()[:, cols]
    A = b["adv"].cpu().numpy()[:, cols]
    for c in range(len(cols)):
        s0, ref = 0, []
        for s in range(T):
            if D[s, c] or s == T - 1:
                dd = D[s0:s + 1, c].copy()
                dd[-1] = True
                ref.append(oppo.gae_fp32(list(R[s0:s + 1, c].astype(np.float64)), V[s0:s + 1, c], dd))
                s0 = s + 1
        assert np.array_equal(A[:, c], np.concatenate(ref)), c
    # one minibatch of the update (PPO.py:46-85): normalised advantages, the first shuffled slice
    B = n * T
    adv = b["adv"].reshape(B)
    rtg = adv + b["val"].reshape(B)
    adv = (adv - adv.mean()) / (adv.std() + 1e-10)
    sel = torch.randperm(B, generator=torch.Generator().manual_seed(0))[:B // 5].cuda()
    batch = (b["obs"][:T].reshape(B, 2, 65)[sel].cpu(), b["act"].reshape(B, 2, 2)[sel].float().cpu(),
             b["logp"].reshape(B)[sel].cpu(), adv[sel].cpu(), rtg[sel].cpu(),
             b["masks"][:T].reshape(B, 2, 6)[sel].bool().cpu())
    actor, critic = oppo.OActor(), oppo.OCritic()
    actor.load_state_dict({k: v.cpu() for k, v in ag.actor.state_dict().items()})
    critic.load_state_dict({k: v.cpu() for k, v in ag.critic.state_dict().items()})
    # rollout actor inputs are the 4 facing one-hots (quirk Q1), so the minibatch's gradient sums
    # collapse onto 4 activation vectors and cancel (see the module doc): held to the default 1e-5
    _step_and_compare(ag, actor, critic, batch, "configs[1]")


def test_bench_rollout_bootstrap_and_update(golden):
    """The bench's loop (bench.py: fixed horizon T=16, bootstrap=True -- the
    open last segment of every env's fragment is bootstrapped with V(s_T), which
    the reference never does) at 4,096 of its 65,536 mazes.  Every 16th maze
    column is replayed in the C oracle (bit-exact obs / masks / rewards / dones);
    the batched critic values V(s_0 .. s_T), V(s_T) included, against the fp32
    oracle critic at 1e-5 of max|V|; the advantages bit-exact against
    oracle.ppo.gae_bootstrap_fp32 on the same values; returns = adv + V; then one
    minibatch of the update against the oracle at the 1e-5 bar."""
    n, T = 4096, 16
    cfg = dict(default_size=(10, 10), max_timestep=1200)
    ag = _agent(n_envs=n, horizon=T, batch_size=n * T, bootstrap=True, sample_seed=13,
                env_config=dict(cfg, seed_base=0))
    assert ag.bootstrap
    act1 = ag.rollout()["act"].cpu().numpy()
    ag._carry_over()  # as get_batch: the next fragment starts from the last observation
    b = ag.rollout()  # the second fragment: episodes carried over from the first, mid-episode starts
    cols = np.arange(0, n, 16)
    obs = b["obs"].cpu().numpy()[:, cols]
    masks = b["masks"].cpu().numpy()[:, cols].astype(bool)
    act = b["act"].cpu().numpy()[:, cols]
    R = b["rew"].cpu().numpy()[:, cols]
    D = b["done"].cpu().numpy()[:, cols].astype(bool)
    # the oracle env is brought to this fragment's first state by the first fragment's actions
    ora = OracleEnv(len(cols), seeds=cols.astype(np.uint64), **cfg)
    oo, om = ora.reset_all()
    for s in range(T):
        oo, om, _, _ = ora.step_all(act1[s][cols], auto_reset=True)
    assert np.array_equal(obs[0], oo) and np.array_equal(masks[0], om)
    for s in range(T):
        oo, om, orw, od = ora.step_all(act[s], auto_reset=True)
        assert np.array_equal(obs[s + 1], oo) and np.array_equal(masks[s + 1], om), s
        assert np.array_equal(R[s], orw) and np.array_equal(D[s], od), s
    critic = oppo.OCritic()
    critic.load_state_dict({k: v.cpu() for k, v in ag.critic.state_dict().items()})
    V = b["val"].cpu().numpy()[:, cols]
    LV = b["last_val"].cpu().numpy()[cols]
    with torch.no_grad():
        rv = np.stack([critic(torch.as_tensor(obs[s])).view(-1).numpy() for s in range(T + 1)])
    got = np.concatenate([V, LV[None]])
    assert np.abs(got - rv).max() <= 1e-5 * np.abs(rv).max(), np.abs(got - rv).max() / np.abs(rv).max()
    A = b["adv"].cpu().numpy()[:, cols]
    open_end = 0
    for c in range(len(cols)):
        ref = oppo.gae_bootstrap_fp32(list(R[:, c].astype(np.float64)), V[:, c], D[:, c], LV[c])
        assert np.array_equal(A[:, c], ref), c
        open_end += not D[-1, c]
    assert open_end > 0  # the bootstrap branch ran
    assert torch.equal(b["rtg"], b["adv"] + b["val"])
    B = n * T
    adv = b["adv"].reshape(B)
    rtg = adv + b["val"].reshape(B)
    adv = (adv - adv.mean()) / (adv.std() + 1e-10)
    sel = torch.randperm(B, generator=torch.Generator().manual_seed(1))[:B // 5].cuda()
    batch = (b["obs"][:T].reshape(B, 2, 65)[sel].cpu(), b["act"].reshape(B, 2, 2)[sel].float().cpu(),
             b["logp"].reshape(B)[sel].cpu(), adv[sel].cpu(), rtg[sel].cpu(),
             b["masks"][:T].reshape(B, 2, 6)[sel].bool().cpu())
    actor = oppo.OActor()
    actor.load_state_dict({k: v.cpu() for k, v in ag.actor.state_dict().items()})
    _step_and_compare(ag, actor, critic, batch, "bench loop, bootstrap")


def test_main_py_hyperparameters_minibatch(golden):
    """The drop-in of INTEGRATION.md section 1, main.py:17 -- PPO(agent_amount=2,
    batch_size=15000, lr=0.00014): its minibatch is 15000 // 5 = 3,000 samples
    (PPO.py:27), i.e. 6,000 actor rows and 3,000 critic rows, all on the
    hand-written engine (no library GEMM at any row count).  Gradients, losses,
    norms and the Adam step vs the oracle at the 1e-5 bar."""
    fx = golden("nets")
    ag = _agent(n_envs=64, batch_size=15000)
    assert ag.mbatch_size == 3000
    actor, critic = _oracle_nets(fx)
    _to_gpu(ag, actor, critic)
    _step_and_compare(ag, actor, critic, _minibatch(fx, 3000), "main.py minibatch")


@pytest.mark.parametrize("S", [3000, 32768])
def test_minibatch_parity_mode_false(golden, S):
    """parity_mode=False (each feature embedding reads its own slice of the
    observation: the slicing networks.py:59-63 evidently intends; the oracle's
    OActor(parity=False) restates it -- no reference counterpart, so the oracle
    is the only anchor): every observation perturbed so that all S rows are
    distinct inputs to the whole actor (not 4 one-hot classes, Q1).  The full
    update -- gradients of every parameter, losses, norms, Adam step -- vs the
    oracle at the 1e-5 bar."""
    fx = golden("nets")
    ag = _agent(n_envs=64, parity_mode=False)
    actor, critic = _oracle_nets(fx, parity=False)
    _to_gpu(ag, actor, critic)
    _step_and_compare(ag, actor, critic, _minibatch(fx, S, noise=0.5), f"parity_mode=False S={S}")


def test_rollout_forward_4096_mazes_matches_oracle(golden):
    """BASELINE configs[1]'s rollout forward: the critic on the 4,096 mazes'
    [4096, 130] observations and the actor (trunk + heads) on their 8,192 agent
    rows, at the shipped checkpoint's weights (ckpt_logits.npz) and at 1e-5 of
    the fp32 oracle; the fused head + sampler kernel's logits too."""
    from marlmaze import ops

    c = golden("ckpt_logits")
    n = 4096
    ag = _agent(n_envs=n, horizon=4, env_config=dict(default_size=(10, 10), max_timestep=1200, seed_base=0))
    ag.actor.load_state_dict({k[6:]: torch.as_tensor(c[k]) for k in c.files if k.startswith("actor/")})
    ag.critic.load_state_dict({k[7:]: torch.as_tensor(c[k]) for k in c.files if k.startswith("critic/")})
    actor, critic = oppo.OActor(), oppo.OCritic()
    actor.load_state_dict({k: v.cpu() for k, v in ag.actor.state_dict().items()})
    critic.load_state_dict({k: v.cpu() for k, v in ag.critic.state_dict().items()})
    ag._ensure_env()
    obs = ag._bufs["obs"][0]
    masks = ag._bufs["masks"][0]
    with torch.no_grad():
        v = ag.critic(obs).cpu()
        mv, mk = ag.actor(obs.reshape(2 * n, 65))
        h = ag.actor.trunk(obs.reshape(2 * n, 65))
        w, b = ag.actor.heads()
        lg = torch.empty(2 * n, 6, device="cuda")
        ops.head_sample(h, w, b, masks.reshape(2 * n, 6), 1, 0, logits=lg)
        rv = critic(obs.cpu())
        rmv, rmk = actor(obs.cpu().reshape(2 * n, 65))
    for got, ref, what in ((v, rv, "values"), (mv.cpu(), rmv, "move"), (mk.cpu(), rmk, "mark"),
                           (lg[:, :5].cpu(), rmv, "head_sample move"), (lg[:, 5:].cpu(), rmk, "head_sample mark")):
        err = (got.double() - ref.double()).abs().max().item()
        assert err <= 1e-5 * ref.abs().max().item() + 1e-6, (what, err)


def test_update_calls_no_library_gemm(golden, monkeypatch):
    """Every GEMM of the update -- at main.py's 3,000-sample minibatch -- and of
    a 4,096-maze rollout runs on the hand-written kernels: the torch GEMM entry
    points are poisoned for the duration."""
    def boom(*a, **k):
        raise AssertionError("a library GEMM was called on the product path")

    import torch.nn.functional as F
    fx = golden("nets")
    ag = _agent(n_envs=4096, horizon=2, batch_size=15000,
                env_config=dict(default_size=(10, 10), max_timestep=1200, seed_base=0))
    batch = [t.cuda() for t in _minibatch(fx, 3000)]
    for mod, name in ((torch, "mm"), (torch, "addmm"), (torch, "bmm"), (torch, "matmul"), (torch, "_addmm_activation"),
                      (F, "linear"), (torch.Tensor, "mm"), (torch.Tensor, "matmul"), (torch.Tensor, "__matmul__"),
                      (torch.Tensor, "addmm")):
        monkeypatch.setattr(mod, name, boom)
    ag.rollout()
    ag.minibatch_step(*batch)
    torch.cuda.synchronize()


def test_update_range_guard_redoes_at_x3(golden):
    """The update's range guard (PPO._range_guarded): with the trunk's and the critic's first-layer weights
    scaled so that the hidden activations exceed fp16's range (2^16), the x2 update raises the library's
    range flag, and the update is redone from the snapshot at x3 -- its parameters, Adam moments and step
    counts then equal, bit for bit, those of the same update run at x3 from the start, and are finite.
    An in-range update is not redone and equals the unguarded x2 passes bit for bit."""
    fx = golden("nets")
    actor, critic = _oracle_nets(fx)
    with torch.no_grad():
        actor.layers[0].weight.mul_(2.0 ** 17)
        critic.layers[0].weight.mul_(2.0 ** 17)
    S = 4096
    obs, act, old, adv, rtg, masks = (t.cuda() for t in _minibatch(fx, S, noise=0.05))
    vals = rtg - adv

    from marlmaze import x3

    def run(prec):
        x3.range_flag(clear=True)  # (no flag left over from an earlier test)
        ag = _agent(n_envs=64, sample_seed=7)
        _to_gpu(ag, actor, critic)
        ag.set_gemm_prec(prec)
        ag.update(obs, act, old, masks, adv, vals, index_list=torch.arange(S))
        torch.cuda.synchronize()
        return ag

    guarded, plain = run("x2"), run("x3")
    assert guarded.range_redos == 1 and plain.range_redos == 0
    assert guarded.gemm_prec == "x2"  # the networks stay on x2 after the redo
    assert torch.isfinite(guarded.flat.data).all()
    assert torch.equal(guarded.flat.data, plain.flat.data)
    assert torch.equal(guarded.actor_optim.exp_avg, plain.actor_optim.exp_avg)
    assert torch.equal(guarded.actor_optim.exp_avg_sq, plain.actor_optim.exp_avg_sq)
    assert guarded.actor_optim.t == plain.actor_optim.t == 25
    # in range: no redo, and the same arithmetic as the update without the guard
    actor2, critic2 = _oracle_nets(fx)
    x3.range_flag(clear=True)
    ag = _agent(n_envs=64, sample_seed=7)
    _to_gpu(ag, actor2, critic2)
    ag.update(obs, act, old, masks, adv, vals, index_list=torch.arange(S))
    assert ag.range_redos == 0 and ag.gemm_prec == "x2" and torch.isfinite(ag.flat.data).all()


def test_rollout_range_flag_discards_the_batch():
    """A rollout whose x2 actor GEMMs left fp16's range (the trunk's first-layer weights x 2^17: its hidden
    activations pass 2^16) raises the library's range flag.  The update on that batch is thrown away -- its
    actions and old log-probs did not come from the fp32 policy -- so the parameters and the Adam state are
    unchanged and hist is NaN; both networks run at x3 from then on, and the next batch (collected at x3)
    trains normally: no redo, finite parameters.  ``train()`` does both in one epoch.  A stale flag from
    GEMMs outside this agent's rollouts (update() on given tensors) is not a rollout flag."""
    from marlmaze import x3

    n, T = 64, 16
    kw = dict(n_envs=n, horizon=T, batch_size=n * T, epochs=1, sample_seed=9, bootstrap=False,
              env_config=dict(default_size=(10, 10), max_timestep=40, seed_base=0))
    ag = _agent(**kw)
    with torch.no_grad():
        ag.actor.layers[0].weight.mul_(2.0 ** 17)
    x3.invalidate_packs()
    batch = ag.get_batch()
    before = ag.flat.data.clone()
    m_before = ag.actor_optim.exp_avg.clone()
    hist = ag.update(batch[0], batch[1], batch[2], batch[5], batch[6], batch[7])
    torch.cuda.synchronize()
    assert ag.last_update_discarded and ag.batches_discarded == 1 and ag.range_switched
    assert ag.gemm_prec == "x3" and ag.actor.gemm_prec == "x3" and ag.critic.gemm_prec == "x3"
    assert torch.isnan(hist).all()
    assert torch.equal(ag.flat.data, before) and torch.equal(ag.actor_optim.exp_avg, m_before)
    assert ag.actor_optim.t == 0
    batch = ag.get_batch()
    hist = ag.update(batch[0], batch[1], batch[2], batch[5], batch[6], batch[7])
    assert not ag.last_update_discarded and ag.range_redos == 0 and ag.batches_discarded == 1
    K = hist.shape[0]  # minibatch steps of one update (Q8: 6 x 5 here)
    assert torch.isfinite(hist).all() and torch.isfinite(ag.flat.data).all() and ag.actor_optim.t == K
    # train(): the discarded batch is re-collected inside the epoch
    bg = _agent(**kw)
    with torch.no_grad():
        bg.actor.layers[0].weight.mul_(2.0 ** 17)
    x3.invalidate_packs()
    bg.train()
    assert bg.batches_discarded == 1 and bg.actor_optim.t == K and np.isfinite(bg.history[-1]["actor_loss"])
    # a stale flag (an out-of-range x2 GEMM outside any rollout of this agent) does not discard an update on
    # given tensors
    cg = _agent(n_envs=64)
    x3.gemm(torch.full((64, 264), 2.0 ** 17, device="cuda"), x3.pack(torch.ones(264, 264, device="cuda"), prec="x2"))
    fx_obs, fx_act, fx_lp, _, _, fx_masks, fx_adv, fx_val = batch
    cg.update(fx_obs, fx_act, fx_lp, fx_masks, fx_adv, fx_val)
    assert not cg.last_update_discarded and cg.gemm_prec == "x2" and cg.range_redos == 0


@pytest.mark.parametrize("S", [3000, 26214, 100000])
def test_side_streams_update_is_bit_identical(golden, monkeypatch, S):
    """The update's critic on a side stream beside the actor (PPO.CRITIC_STREAM) and the actor's weight
    gradients on another beside its input-gradient chain (networks.WGRAD_STREAM) run the same kernels on the
    same inputs: every gradient, both losses and the Adam step equal the one-stream update bit for bit
    (main.py's 3,000-sample minibatch, configs[1]'s 26,214, and a large one)."""
    from marlmaze import PPO as ppo_mod
    from marlmaze import networks as nets_mod

    fx = golden("nets")
    batch = [t.cuda() for t in _minibatch(fx, S, noise=0.05)]
    res = []
    for mode in ("off", "on"):
        monkeypatch.setattr(ppo_mod, "CRITIC_STREAM", mode)
        monkeypatch.setattr(nets_mod, "WGRAD_STREAM", mode == "on")
        actor, critic = _oracle_nets(fx)
        ag = _agent(n_envs=64)
        _to_gpu(ag, actor, critic)
        out = ag.minibatch_step(*batch)
        torch.cuda.synchronize()
        res.append((torch.stack(out).cpu(), ag.flat.data.clone(), ag.flat.grad.clone()))
    for a, b in zip(*res):
        assert torch.equal(a, b)
