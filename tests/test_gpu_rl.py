"""GPU parity of the GAE scan and the action sampler (libmarlmaze.so)."""
import numpy as np
import pytest
import torch

from marlmaze import ops
from oracle import ppo as oppo

pytestmark = pytest.mark.gpu


def test_gae_matches_reference_vectors(golden):
    g = golden("gae")
    for i in range(int(g["n"])):
        r = torch.as_tensor(g[f"L{i}/rew"].astype(np.float32)).cuda()[:, None]
        v = torch.as_tensor(g[f"L{i}/val"]).cuda()[:, None]
        d = torch.as_tensor(g[f"L{i}/done"]).cuda()[:, None]
        adv, rtg = ops.gae(r, v, d)
        assert np.array_equal(adv[:, 0].cpu().numpy(), g[f"L{i}/adv"].astype(np.float32)), i
        assert np.array_equal(rtg[:, 0].cpu().numpy(), (g[f"L{i}/adv"].astype(np.float32) + g[f"L{i}/val"]))


def _split_episodes(r, v, d):
    """oracle: per-column episodes (segment end = episode end), reference GAE each."""
    T, N = r.shape
    out = np.zeros((T, N), np.float32)
    for n in range(N):
        s = 0
        for t in range(T):
            if d[t, n] or t == T - 1:
                dd = d[s:t + 1, n].copy()
                dd[-1] = True
                out[s:t + 1, n] = oppo.gae_fp32(list(r[s:t + 1, n].astype(np.float64)), v[s:t + 1, n], dd)
                s = t + 1
    return out


@pytest.mark.parametrize("algo", ["auto", "column", "walk"])
@pytest.mark.parametrize("T,N", [(1, 7), (16, 257), (64, 1000)])
def test_gae_time_major_matches_oracle(T, N, algo):
    rng = np.random.default_rng(T * 1000 + N)
    r = rng.choice(np.float32([0, 0, 0, 0.5, 1]), size=(T, N)).astype(np.float32)
    v = rng.normal(0, 1, (T, N)).astype(np.float32)
    d = rng.random((T, N)) < 0.1
    adv, rtg = ops.gae(torch.as_tensor(r).cuda(), torch.as_tensor(v).cuda(), torch.as_tensor(d).cuda(), algo=algo)
    assert np.array_equal(adv.cpu().numpy(), _split_episodes(r, v, d))
    assert np.array_equal(rtg.cpu().numpy(), adv.cpu().numpy() + v)


def _long_episodes(rng, T, N, max_len=1200):
    """done flags of whole episodes of 1 .. max_len steps (the reference's
    episodes end by exit or by max_timestep truncation, maze.py:116-121)."""
    d = np.zeros((T, N), bool)
    for n in range(N):
        t = -1
        while True:
            t += int(rng.integers(1, max_len + 1))
            if t >= T:
                break
            d[t, n] = True
    return d


def _bootstrap_ref(r, v, d, lv):
    """numpy fp32 emulation of the recursion with a bootstrap value V(s_T)."""
    T, N = r.shape
    f = np.float32
    g, gl = f(0.99), f(0.99 * 0.95)
    a = np.zeros(N, np.float32)
    vn, dn = lv.copy(), np.zeros(N, bool)
    ref = np.zeros((T, N), np.float32)
    for t in range(T - 1, -1, -1):
        boot = (g * vn).astype(np.float32)
        boot = np.where(dn, (boot * f(0)).astype(np.float32), boot)
        delta = np.where(d[t], (r[t] - v[t]).astype(np.float32), ((r[t] + boot).astype(np.float32) - v[t]))
        a = (delta + np.where(d[t], f(0), gl) * a).astype(np.float32)
        ref[t] = a
        vn, dn = v[t], d[t]
    return ref


@pytest.mark.parametrize("T,N", [(15600, 1), (5000, 3), (700, 64)])
def test_gae_long_episodes(T, N):
    """Whole-episode batches (PPO.py:108-141: one maze, ~15,600 steps, episodes
    up to max_timestep=1200): the episode-parallel walk is bit-identical to the
    per-episode reference recursion; the shuffle scan is within 1e-5 of it."""
    rng = np.random.default_rng(T + N)
    r = rng.choice(np.float32([0, 0, 0, 0.5, 1, -0.25]), size=(T, N)).astype(np.float32)
    v = rng.normal(0, 1, (T, N)).astype(np.float32)
    d = _long_episodes(rng, T, N)
    ref = _split_episodes(r, v, d)
    tr, tv, td = (torch.as_tensor(x).cuda() for x in (r, v, d))
    for algo in ("auto", "walk", "column"):
        adv, rtg = ops.gae(tr, tv, td, algo=algo)
        assert np.array_equal(adv.cpu().numpy(), ref), algo
        assert np.array_equal(rtg.cpu().numpy(), ref + v), algo
    adv, rtg = ops.gae(tr, tv, td, algo="scan")
    scale = np.abs(ref).max(0, keepdims=True)
    np.testing.assert_allclose(adv.cpu().numpy(), ref, rtol=1e-5, atol=(1e-5 * scale).max())
    # a bootstrapped last fragment (the horizon cut) on the same data
    lv = rng.normal(0, 1, N).astype(np.float32)
    ref_b = _bootstrap_ref(r, v, d, lv)
    for algo in ("walk", "column"):
        adv, _ = ops.gae(tr, tv, td, last_value=torch.as_tensor(lv).cuda(), algo=algo)
        assert np.array_equal(adv.cpu().numpy(), ref_b), algo
    adv, _ = ops.gae(tr, tv, td, last_value=torch.as_tensor(lv).cuda(), algo="scan")
    np.testing.assert_allclose(adv.cpu().numpy(), ref_b, rtol=1e-5, atol=1e-5 * np.abs(ref_b).max())


def test_gae_bootstrap_and_scale():
    T, N = 32, 65536  # configs: 65,536 mazes, T=32
    rng = np.random.default_rng(0)
    r = rng.choice(np.float32([0, 0.5, 1]), size=(T, N)).astype(np.float32)
    v = rng.normal(0, 1, (T, N)).astype(np.float32)
    d = rng.random((T, N)) < 0.02
    lv = rng.normal(0, 1, N).astype(np.float32)
    adv, _ = ops.gae(*(torch.as_tensor(x).cuda() for x in (r, v, d)), last_value=torch.as_tensor(lv).cuda())
    assert np.array_equal(adv.cpu().numpy(), _bootstrap_ref(r, v, d, lv))


def _random_masks(rng, M):
    m = rng.random((M, 6)) < 0.6
    none = ~m[:, :5].any(1)
    m[none, rng.integers(0, 5, none.sum())] = True
    return m


def test_sampler_logp_and_legality():
    M = 2 * 50000
    rng = np.random.default_rng(3)
    ml = rng.normal(0, 2, (M, 5)).astype(np.float32)
    kl = rng.normal(0, 2, (M, 1)).astype(np.float32)
    mk = _random_masks(rng, M)
    a, lp, jl = ops.sample(*(torch.as_tensor(x).cuda() for x in (ml, kl, mk.astype(np.uint8))), seed=7, offset=0)
    a = a.cpu().numpy().astype(np.int64)
    assert mk[np.arange(M), a[:, 0]].all()  # legal moves only
    assert (a[~mk[:, 5], 1] == 0).all()  # no mark where not allowed
    # log-prob formula of PPO.get_log_probs / get_action on the CPU (torch)
    o = torch.as_tensor
    ref = oppo.log_probs(lambda x: (o(ml), o(kl)), 0, o(np.zeros((M, 1, 65), np.float32)),
                         o(a[:, None, :].astype(np.float32)), o(mk[:, None, :]))
    np.testing.assert_allclose(lp.cpu().numpy(), ref.numpy(), rtol=1e-5, atol=1e-6)
    j = lp.cpu().numpy().reshape(-1, 2)
    assert np.array_equal(jl.cpu().numpy(), (j[:, 0] + j[:, 1]).astype(np.float32))
    # determinism (counter-based): same (seed, offset) -> same draw; new offset -> new draw
    a2, _, _ = ops.sample(*(torch.as_tensor(x).cuda() for x in (ml, kl, mk.astype(np.uint8))), seed=7, offset=0)
    a3, _, _ = ops.sample(*(torch.as_tensor(x).cuda() for x in (ml, kl, mk.astype(np.uint8))), seed=7, offset=1)
    assert np.array_equal(a2.cpu().numpy(), a)
    assert not np.array_equal(a3.cpu().numpy(), a)


def test_sampler_distribution():
    M = 400000
    logits = np.float32([1.0, -0.5, 0.3, 2.0, -1.0])
    ml = np.tile(logits, (M, 1))
    kl = np.full((M, 1), 0.7, np.float32)
    mk = np.ones((M, 6), bool)
    mk[:, 2] = False
    a, _, _ = ops.sample(*(torch.as_tensor(x).cuda() for x in (ml, kl, mk.astype(np.uint8))), seed=11, offset=5)
    a = a.cpu().numpy()
    p = np.exp(logits - logits.max()) * mk[0, :5]
    p /= p.sum()
    freq = np.bincount(a[:, 0], minlength=5) / M
    assert np.abs(freq - p).max() < 4 * np.sqrt(p.max() / M) + 1e-4
    pm = 1 / (1 + np.exp(-0.7))
    assert abs(a[:, 1].mean() - pm) < 4 * np.sqrt(pm * (1 - pm) / M)


def test_head_sample_matches_unfused_path():
    """F3: heads GEMM + sampler fused == actor heads (torch) then mm_sample on
    the same Philox counters: logits at fp32 tolerance, the same draws."""
    from marlmaze.networks import Actor

    torch.manual_seed(1)
    actor = Actor([264, 264, 264]).cuda()
    with torch.no_grad():  # larger head weights than the 0.01 init so the draws are not trivially uniform
        actor.move_head.weight.mul_(100.0)
        actor.mark_head.weight.mul_(100.0)
    M = 40001
    x = torch.rand(M, 65, device="cuda")
    g = torch.Generator(device="cuda").manual_seed(2)
    masks = (torch.rand(M, 6, device="cuda", generator=g) < 0.7).to(torch.uint8)
    with torch.no_grad():
        h = actor.trunk(x)
        w, b = actor.heads()
        ml, kl = actor(x)
        a0, lp0, j0 = ops.sample(ml, kl.view(-1), masks, seed=7, offset=3)
        logits = torch.empty(M, 6, device="cuda")
        a1, lp1, j1 = ops.head_sample(h, w, b, masks, seed=7, offset=3, logits=logits)
    torch.testing.assert_close(logits[:, :5], ml, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(logits[:, 5], kl.view(-1), rtol=1e-5, atol=1e-5)
    same = (a0 == a1).all(1)
    assert same.float().mean().item() > 0.999  # a draw can flip only where a logit difference lands on the CDF
    fin = same & torch.isfinite(lp0)
    torch.testing.assert_close(lp1[fin], lp0[fin], rtol=1e-5, atol=1e-5)
    legal = masks[torch.arange(M, device="cuda"), a1[:, 0].long()].bool() | (masks[:, :5].sum(1) == 0)
    assert legal.all()
    jr = lp1.view(-1)[: M - 1:2] + lp1.view(-1)[1:M:2]
    torch.testing.assert_close(j1[: (M - 1) // 2 + 0][: jr.numel()], jr, rtol=0, atol=0, equal_nan=True)
    # the update's heads forward (mm_heads_fwd) takes mm_head_sample's arithmetic: the same logits bit for bit,
    # so the PPO ratio of a fresh batch is exactly 1 at the rollout's parameters
    with torch.no_grad():
        z = actor.logits(x)
    assert torch.equal(z, logits)


@pytest.mark.parametrize("K", [128, 264, 1024])
def test_heads_fwd_vs_fp64(K):
    """mm_heads_fwd at the unrolled width (264) and the runtime-loop widths, ragged row counts, against fp64."""
    from marlmaze.networks import _heads_fwd

    g = torch.Generator(device="cuda").manual_seed(K)
    for M in (1, 31, 33, 5000):
        h = torch.rand(M, K, device="cuda", generator=g) * 3
        w = torch.randn(6, K, device="cuda", generator=g) * 0.05
        b = torch.randn(6, device="cuda", generator=g)
        z = _heads_fwd(h, w, b)
        ref = h.double() @ w.double().T + b.double()
        err = (z.double() - ref).abs().max().item()
        assert err <= 1e-5 * ref.abs().max().item(), (K, M, err)
