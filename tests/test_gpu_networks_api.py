"""The explicit backward used outside PPO's flat buffers (Actor / Critic as
stand-alone modules, networks.py:13-106) and .grad handling around it.

* A stand-alone Actor's heads are separate tensors (not the back-to-back pair
  update.FlatParams lays out), so train_backward copies the heads' gradients
  into their own .grad.  Inside an x3.deferred() scope that copy must read a
  finished result: the gradients must equal, bit for bit, those of the same
  backward outside the scope.
* nn.Module.zero_grad() (set_to_none=True) drops the .grad views of PPO's flat
  gradient buffer.  The explicit backward re-binds them, so the all-reduce and
  mm_clip_adam, which read the flat buffer, still see every gradient.
"""
import numpy as np
import pytest
import torch

from marlmaze import x3
from marlmaze.PPO import PPO
from marlmaze.networks import Actor
from oracle import ppo as oppo

pytestmark = pytest.mark.gpu


def _actor_from_fixture(fx):
    a = Actor([264, 264, 264]).cuda()
    a.load_state_dict({k[6:]: torch.as_tensor(fx[k]).cuda() for k in fx.files if k.startswith("actor/")})
    return a


def _grads(mod):
    return {k: p.grad.detach().clone() for k, p in mod.named_parameters()}


@pytest.mark.parametrize("rows", [512, 20000])
def test_standalone_actor_backward_inside_deferred(golden, rows):
    fx = golden("nets")
    actor = _actor_from_fixture(fx)
    obs = torch.as_tensor(fx["obs"]).reshape(-1, 65)
    x = obs[torch.arange(rows) % obs.shape[0]].cuda().contiguous()
    g = torch.Generator().manual_seed(rows)
    dz = (torch.randn((rows, 6), generator=g) / rows).cuda()
    z, saved = actor.train_forward(x)
    actor.train_backward(saved, dz)
    ref = _grads(actor)
    actor.zero_grad(set_to_none=True)
    z2, saved2 = actor.train_forward(x)
    with x3.deferred():
        actor.train_backward(saved2, dz)
    got = _grads(actor)
    assert torch.equal(z, z2)
    for k in ref:
        assert torch.equal(got[k], ref[k]), k
    # and the gradients are the autograd ones of the same actor (loose: summation order differs)
    a64 = oppo.OActor()
    a64.load_state_dict({k[6:]: torch.as_tensor(fx[k]) for k in fx.files if k.startswith("actor/")})
    a64 = a64.double()
    ml, kl = a64(x.cpu().double())
    (torch.cat([ml, kl], 1) * dz.cpu().double()).sum().backward()
    for k, p in a64.named_parameters():
        r = p.grad.double()
        cos = torch.nn.functional.cosine_similarity(got[k].cpu().double().flatten(), r.flatten(), 0).item()
        assert cos > 0.9999 or r.abs().max().item() == 0, (k, cos)


def test_zero_grad_set_to_none_rebinds_flat_buffer(golden):
    fx = golden("nets")
    ag = PPO(2, load=False, verbose=False, save=False, lr=0.00014, n_envs=16)
    ag.actor.load_state_dict({k[6:]: torch.as_tensor(fx[k]).cuda() for k in fx.files if k.startswith("actor/")})
    ag.critic.load_state_dict({k[7:]: torch.as_tensor(fx[k]).cuda() for k in fx.files if k.startswith("critic/")})
    batch = tuple(torch.as_tensor(fx[k]).cuda() for k in ("obs", "actions", "old_logp", "advs", "rtgs", "masks"))
    params = list(ag.actor.parameters()) + list(ag.critic.parameters())
    ag.minibatch_grads(*batch)
    ref = [p.grad.clone() for p in params]
    ag.flat.grad.fill_(float("nan"))  # (the alignment padding between parameters stays NaN: never written)
    ag.actor.zero_grad()  # set_to_none=True: the .grad views are gone
    ag.critic.zero_grad()
    assert all(p.grad is None for p in params)
    ag.minibatch_grads(*batch)
    lo, hi = ag.flat.grad.data_ptr(), ag.flat.grad.data_ptr() + 4 * ag.flat.numel
    for p, r in zip(params, ref):
        assert lo <= p.grad.data_ptr() < hi  # a view of the flat buffer again
        assert torch.equal(p.grad, r) and torch.equal(ag.flat.moment_view(ag.flat.grad, p), r)
        assert np.isfinite(r.cpu().numpy()).all()


@pytest.mark.parametrize("M", [1, 63, 4096, 70001, 17 * 65536 + 5])
def test_fused_critic_value_matches_oracle(golden, M):
    """mm_critic_value (the rollout's V, networks.py:87-102) against the fp64 oracle critic: the three layers on
    the fp32 MFMA in one launch, at 1e-5 of max |V| (ragged row counts: partial 16-row tiles; the bench's batched
    rollout size, where each persistent wavefront walks many tiles).  Each row's value is independent of the
    batch it sits in, bit for bit: the same rows permuted, and the first rows alone."""
    from marlmaze.networks import Critic

    fx = golden("nets")
    cr = Critic(2, hidden_sizes=[64, 64]).cuda()
    cr.load_state_dict({k[7:]: torch.as_tensor(fx[k]).cuda() for k in fx.files if k.startswith("critic/")})
    obs = torch.as_tensor(fx["obs"]).reshape(-1, 130)
    g = torch.Generator().manual_seed(M)
    x = obs[torch.randint(0, obs.shape[0], (M,), generator=g)] + 0.1 * torch.randn(M, 130, generator=g)
    v = torch.full((M,), float("nan"), device="cuda")
    cr.value_into(x.cuda(), v)
    oc = oppo.OCritic()
    oc.load_state_dict({k[7:]: torch.as_tensor(fx[k]) for k in fx.files if k.startswith("critic/")})
    with torch.no_grad():
        ref = oc.double()(x.double()).squeeze(-1)
    err = (v.cpu().double() - ref).abs().max().item()
    assert err <= 1e-5 * ref.abs().max().item() + 1e-6, err
    perm = torch.randperm(M, generator=g)
    vp = torch.empty(M, device="cuda")
    cr.value_into(x[perm].cuda(), vp)
    assert torch.equal(vp.cpu(), v.cpu()[perm])
    m = min(M, 37)
    vs = torch.empty(m, device="cuda")
    cr.value_into(x[:m].cuda(), vs)
    assert torch.equal(vs, v[:m])
