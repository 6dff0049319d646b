"""The fp16 actor/critic (BASELINE configs[4]: 262,144 10x10 mazes over 8
MI355X, fp16 actor/critic, 6 logits = 5 moves + 1 mark) against the fp32
oracle (oracle/ppo.py, pinned to the reference's own networks and update).

PPO(dtype="f16") runs every actor-MLP and critic GEMM -- forward, input
gradient and weight gradient -- on the fp16 MFMA (operands rounded to fp16,
fp32 accumulation); storage, the fp32 master weights, clipping and Adam are
unchanged, and the front-end (projection + attention) stays fp32.  The
reference has no fp16 mode, so the bar is a stated tolerance, from the fp16
unit roundoff 2^-11 = 4.9e-4 per operand (measured values in brackets):

* logits and values: max|got - ref| <= 2e-3 max|ref| over the batch [7.0e-4, 4.7e-4];
* one update minibatch (32,768 samples): losses within 1e-3 relative + 1e-5;
  each parameter's gradient ||g - g64|| <= 5e-3 ||g64|| [<= 1.5e-3] and the
  cosine with the exact gradient >= 0.9999 [0.999999];
* configs[4]'s per-GPU share (32,768 mazes): rollout + the whole update run,
  losses finite; one full-size minibatch (209,714 actor rows) of that rollout
  held to the gradient bar above against the fp32 oracle itself (torch CPU,
  16 threads, ~5 s) and against the fp32-class engine.
"""
import copy

import numpy as np
import pytest
import torch

from marlmaze.PPO import PPO
from oracle import ppo as oppo

pytestmark = pytest.mark.gpu


def _agent(**kw):
    for k, v in dict(load=False, verbose=False, save=False, lr=0.00014, dtype="f16").items():
        kw.setdefault(k, v)
    return PPO(2, **kw)


def _oracle_nets(fx):
    a, c = oppo.OActor(), oppo.OCritic()
    a.load_state_dict({k[6:]: torch.as_tensor(fx[k]) for k in fx.files if k.startswith("actor/")})
    c.load_state_dict({k[7:]: torch.as_tensor(fx[k]) for k in fx.files if k.startswith("critic/")})
    return a, c


def _to_gpu(agent, actor, critic):
    agent.actor.load_state_dict({k: v.detach().cuda() for k, v in actor.state_dict().items()})
    agent.critic.load_state_dict({k: v.detach().cuda() for k, v in critic.state_dict().items()})


def _batch(fx, S):
    g = torch.Generator().manual_seed(S)
    idx = torch.arange(S) % fx["obs"].shape[0]
    old = torch.as_tensor(fx["old_logp"])[idx] + 0.3 * torch.randn(S, generator=g)
    return (torch.as_tensor(fx["obs"])[idx], torch.as_tensor(fx["actions"])[idx], old,
            torch.randn(S, generator=g), torch.randn(S, generator=g), torch.as_tensor(fx["masks"])[idx])


@pytest.mark.parametrize("S", [256, 32768])
def test_f16_forward_vs_fp32_oracle(golden, S):
    fx = golden("nets")
    ag = _agent(n_envs=64)
    actor, critic = _oracle_nets(fx)
    _to_gpu(ag, actor, critic)
    # non-trivial heads: the init scales them by 0.01, which would hide the trunk's error
    with torch.no_grad():
        for net in (actor, ag.actor):
            net.move_head.weight.mul_(30.0)
            net.mark_head.weight.mul_(30.0)
    obs = _batch(fx, S)[0]
    with torch.no_grad():
        ml, kl = ag.actor(obs.reshape(-1, 65).cuda())
        got = torch.cat([ml, kl], 1).cpu()
        rm, rk = actor(obs.reshape(-1, 65))
        ref = torch.cat([rm, rk], 1)
        v = ag.critic(obs.cuda()).cpu()
        rv = critic(obs)
    e_logit = (got - ref).abs().max().item() / ref.abs().max().item()
    e_val = (v - rv).abs().max().item() / rv.abs().max().item()
    print(f"f16 S={S}: logits {e_logit:.2e}, values {e_val:.2e} of max|ref|")
    assert e_logit <= 2e-3 and e_val <= 2e-3, (e_logit, e_val)


def test_f16_rollout_forward_65536_rows_vs_fp32_oracle(golden):
    """configs[4]'s rollout step on one GPU: 32,768 mazes = 65,536 actor rows, which run the fused trunk
    (k_trunk3, enabled to 131,072 rows at f16) and, in the rollout, the fused trunk + heads + draws.  Both
    forms' logits against the fp32 oracle actor (oracle.ppo.OActor, the reference's arithmetic) at the
    bar above: max|got - ref| <= 2e-3 max|ref|."""
    from marlmaze import networks, ops, x3

    fx = golden("nets")
    ag = _agent(n_envs=64)
    actor, critic = _oracle_nets(fx)
    with torch.no_grad():  # non-trivial heads (see above)
        actor.move_head.weight.mul_(30.0)
        actor.mark_head.weight.mul_(30.0)
    _to_gpu(ag, actor, critic)
    M = 65536
    assert M <= networks._trunk_max_rows("f16")
    g = torch.Generator().manual_seed(65536)
    obs = torch.as_tensor(fx["obs"]).reshape(-1, 65)
    obs = obs[torch.arange(M) % obs.shape[0]] * (1 + 0.05 * torch.rand(M, 65, generator=g))  # distinct rows
    masks = torch.ones(M, 6, dtype=torch.uint8)
    xg = obs.cuda()
    with torch.no_grad():
        ml, kl = ag.actor(xg)  # Actor.logits: the fused trunk at 65,536 rows + the heads
        got = torch.cat([ml, kl], 1).cpu()
        h0 = ag.actor._front(xg)
        params = ag.actor._mlp_params()
        packs = [x3.pack(w, prec="f16") for w in params[0::2]]
        assert x3.trunk3_head_sample_ok(M, h0, packs, "f16")
        hw, hb = ag.actor.heads()
        act = torch.empty((M, 2), dtype=torch.int8, device="cuda")
        lg = torch.empty((M, 6), device="cuda")
        x3.trunk3_head_sample(h0, packs, params[1::2], hw.contiguous(), hb.contiguous(), masks.cuda(), 5, 0, act,
                              logits=lg)
        threads = torch.get_num_threads()
        torch.set_num_threads(min(threads, 16))  # the box's CPU share
        try:
            rm, rk = actor(obs)
        finally:
            torch.set_num_threads(threads)
        ref = torch.cat([rm, rk], 1)
    e_fwd = (got - ref).abs().max().item() / ref.abs().max().item()
    e_hs = (lg.cpu() - ref).abs().max().item() / ref.abs().max().item()
    print(f"f16 rollout forward at {M} rows: Actor.logits {e_fwd:.2e}, trunk3_head_sample {e_hs:.2e} of max|ref|")
    assert e_fwd <= 2e-3 and e_hs <= 2e-3, (e_fwd, e_hs)
    del ops


def test_f16_minibatch_gradients_vs_fp64_oracle(golden):
    fx = golden("nets")
    ag = _agent(n_envs=64)
    actor, critic = _oracle_nets(fx)
    _to_gpu(ag, actor, critic)
    batch = _batch(fx, 32768)
    ra, rc, _, _ = oppo.minibatch_grads(actor, critic, *batch)
    _, _, ga64, gc64 = oppo.minibatch_grads(copy.deepcopy(actor).double(), copy.deepcopy(critic).double(), *batch)
    al, cl = ag.minibatch_grads(*(t.cuda() for t in batch))
    assert abs(float(al) - ra) <= 1e-3 * abs(ra) + 1e-5, (float(al), ra)
    assert abs(float(cl) - rc) <= 1e-3 * abs(rc) + 1e-5, (float(cl), rc)
    worst = []
    for net, ref in ((ag.actor, ga64), (ag.critic, gc64)):
        for k, p in net.named_parameters():
            g, r = p.grad.detach().cpu().double().flatten(), ref[k].double().flatten()
            rel = (g - r).norm().item() / max(r.norm().item(), 1e-30)
            cos = torch.dot(g, r).item() / max(g.norm().item() * r.norm().item(), 1e-30)
            worst.append((rel, cos, k))
    worst.sort(reverse=True)
    print("f16 worst gradient tensors:", [(f"{r:.2e}", f"{c:.6f}", k) for r, c, k in worst[:4]])
    assert all(rel <= 5e-3 and cos >= 0.9999 for rel, cos, _ in worst), worst[:4]


def test_f16_config4_per_gpu_share():
    """BASELINE configs[4] on one GPU: 32,768 mazes (262,144 / 8), 10x10, one
    rollout (T=16) and the reference update (5 x 5 minibatches).  Before the
    update, one full-size minibatch (a fifth of the 524,288 rollout samples:
    209,714 actor rows) is held to the same gradient bar as the 32,768-sample
    case above, against the fp32-class engine (PPO dtype "f32", itself held to
    the fp64 oracle at 1e-5 in test_gpu_update_parity.py) at the same
    parameters -- and against the fp32 oracle (oracle.ppo.minibatch_grads, the
    reference's arithmetic) on the same rows."""
    n, T = 32768, 16
    ag = _agent(n_envs=n, horizon=T, batch_size=n * T, epochs=1, sample_seed=4,
                env_config=dict(default_size=(10, 10), max_timestep=1200, seed_base=0))
    b_obs, b_act, b_lp, _, _, b_masks, b_advs, b_vals = ag.get_batch()
    mb = b_obs.shape[0] // 5
    adv = (b_advs - b_advs.mean()) / (b_advs.std() + 1e-10)
    batch = (b_obs[:mb], b_act[:mb], b_lp[:mb], adv[:mb], (b_advs + b_vals)[:mb], b_masks[:mb])
    ref = _agent(n_envs=64, dtype="f32")
    ref.actor.load_state_dict(ag.actor.state_dict())
    ref.critic.load_state_dict(ag.critic.state_dict())
    actor, critic = oppo.OActor(), oppo.OCritic()
    actor.load_state_dict({k: v.cpu() for k, v in ag.actor.state_dict().items()})
    critic.load_state_dict({k: v.cpu() for k, v in ag.critic.state_dict().items()})
    threads = torch.get_num_threads()
    torch.set_num_threads(min(threads, 16))  # the box's CPU share
    try:
        oal, ocl, oga, ogc = oppo.minibatch_grads(actor, critic, *(t.cpu() for t in batch))
    finally:
        torch.set_num_threads(threads)
    al, cl = ag.minibatch_grads(*batch)
    assert abs(float(al) - oal) <= 1e-3 * abs(oal) + 1e-5, (float(al), oal)
    assert abs(float(cl) - ocl) <= 1e-3 * abs(ocl) + 1e-5, (float(cl), ocl)
    worst = []
    for net, og in ((ag.actor, oga), (ag.critic, ogc)):
        for k, p in net.named_parameters():
            g, r = p.grad.detach().cpu().double().flatten(), og[k].double().flatten()
            rel = (g - r).norm().item() / max(r.norm().item(), 1e-30)
            cos = torch.dot(g, r).item() / max(g.norm().item() * r.norm().item(), 1e-30)
            worst.append((rel, cos, k))
    worst.sort(reverse=True)
    print("f16 full-size minibatch vs the fp32 oracle, worst gradient tensors:",
          [(f"{r:.2e}", f"{c:.6f}", k) for r, c, k in worst[:4]])
    assert all(rel <= 5e-3 and cos >= 0.9999 for rel, cos, _ in worst), worst[:4]
    ral, rcl = ref.minibatch_grads(*batch)
    assert abs(float(al) - float(ral)) <= 1e-3 * abs(float(ral)) + 1e-5, (float(al), float(ral))
    assert abs(float(cl) - float(rcl)) <= 1e-3 * abs(float(rcl)) + 1e-5, (float(cl), float(rcl))
    worst = []
    for net, rnet in ((ag.actor, ref.actor), (ag.critic, ref.critic)):
        rg = dict(rnet.named_parameters())
        for k, p in net.named_parameters():
            g, r = p.grad.detach().double().flatten(), rg[k].grad.detach().double().flatten()
            rel = (g - r).norm().item() / max(r.norm().item(), 1e-30)
            cos = torch.dot(g, r).item() / max(g.norm().item() * r.norm().item(), 1e-30)
            worst.append((rel, cos, k))
    worst.sort(reverse=True)
    print("f16 full-size minibatch, worst gradient tensors:", [(f"{r:.2e}", f"{c:.6f}", k) for r, c, k in worst[:4]])
    assert all(rel <= 5e-3 and cos >= 0.9999 for rel, cos, _ in worst), worst[:4]
    del ref
    hist = ag.update(b_obs, b_act, b_lp, b_masks, b_advs, b_vals)
    ag.history.append(dict(actor_loss=float(hist[-1, 0]), critic_loss=float(hist[-1, 1])))
    h = ag.history[-1]
    assert np.isfinite([h["actor_loss"], h["critic_loss"]]).all()
    assert all(torch.isfinite(p).all() for p in list(ag.actor.parameters()) + list(ag.critic.parameters()))
