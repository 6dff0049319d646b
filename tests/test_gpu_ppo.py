"""GPU parity of the PPO path: networks, log-probs, the minibatch update, a
teacher-forced reference train() epoch, and the vectorised rollout loop.

Tolerance: 1e-5 relative on losses / returns / logits (BASELINE parity bar),
with a small absolute floor (1e-6) for values that are ~0 (the actor loss of a
normalised advantage batch).  Parameters after Adam are compared at the scale
of one Adam step in test_gpu_update_parity.py (with per-parameter gradients).
"""
import copy

import numpy as np
import pytest
import torch

from marlmaze.PPO import PPO
from marlmaze import ops
from oracle import ppo as oppo
from oracle.env import OracleEnv

pytestmark = pytest.mark.gpu

RTOL, ATOL = 1e-5, 1e-6


def _agent(**kw):
    kw.setdefault("load", False)
    kw.setdefault("verbose", False)
    kw.setdefault("save", False)
    return PPO(2, **kw)


def _load(agent, fx, prefix_a="actor/", prefix_c="critic/"):
    agent.actor.load_state_dict({k[len(prefix_a):]: torch.as_tensor(fx[k]) for k in fx.files if k.startswith(prefix_a)})
    agent.critic.load_state_dict({k[len(prefix_c):]: torch.as_tensor(fx[k]) for k in fx.files
                                  if k.startswith(prefix_c)})


def test_forward_matches_reference(golden):
    n = golden("nets")
    ag = _agent(n_envs=64)
    _load(ag, n)
    o = torch.as_tensor(n["obs"]).cuda()
    with torch.no_grad():
        mv, mr = ag.actor(o.reshape(-1, 65))
        v = ag.critic(o)
    np.testing.assert_allclose(mv.cpu().numpy(), n["move_logits"], rtol=RTOL, atol=ATOL)
    np.testing.assert_allclose(mr.cpu().numpy(), n["mark_logits"], rtol=RTOL, atol=ATOL)
    np.testing.assert_allclose(v.cpu().numpy(), n["values"], rtol=RTOL, atol=ATOL)
    mk = torch.as_tensor(n["masks"]).cuda()
    ac = torch.as_tensor(n["actions"]).cuda()
    with torch.no_grad():
        for i in range(2):
            np.testing.assert_allclose(ag.get_log_probs(i, o, ac, mk).cpu().numpy(), n[f"logp{i}"],
                                       rtol=RTOL, atol=ATOL)
        joint = ag.policy_logp(o, ac, mk)
    np.testing.assert_allclose(joint.cpu().numpy(), n["logp0"] + n["logp1"], rtol=RTOL, atol=ATOL)


def test_checkpoint_forward(golden):
    """The shipped PPO.pth weights (as data) reproduce the reference logits."""
    c = golden("ckpt_logits")
    ag = _agent(n_envs=64)
    _load(ag, c)
    o = torch.as_tensor(c["obs"]).cuda()
    with torch.no_grad():
        mv, mr = ag.actor(o.reshape(-1, 65))
        v = ag.critic(o)
    np.testing.assert_allclose(mv.cpu().numpy(), c["move_logits"], rtol=RTOL, atol=1e-5)
    np.testing.assert_allclose(mr.cpu().numpy(), c["mark_logits"], rtol=RTOL, atol=1e-5)
    np.testing.assert_allclose(v.cpu().numpy(), c["values"], rtol=RTOL, atol=1e-5)


def test_minibatch_update_matches_reference(golden):
    n = golden("nets")
    ag = _agent(n_envs=64, lr=0.00014)
    _load(ag, n)
    t = {k: torch.as_tensor(n[k]).cuda() for k in ("obs", "actions", "old_logp", "advs", "rtgs", "masks")}
    al, cl, ga, gc = (float(x) for x in ag.minibatch_step(t["obs"], t["actions"], t["old_logp"], t["advs"],
                                                           t["rtgs"], t["masks"]))
    for got, ref in ((al, n["actor_loss"]), (cl, n["critic_loss"]), (ga, n["actor_gnorm"]), (gc, n["critic_gnorm"])):
        assert abs(got - float(ref)) <= RTOL * abs(float(ref)) + ATOL, (got, float(ref))
    # parameters after the step: test_gpu_update_parity.py (per-tensor Delta p vs actor_after / critic_after)


def test_train_epoch_teacher_forced(golden):
    """The reference's recorded PPO.train() epoch (batch 600) replayed on the GPU,
    free-running: parameters drift from the reference's by summation-order
    rounding amplified through 25 Adam steps, so minibatches after the first are
    held to 1e-4 here; test_gpu_update_parity.py teacher-forces the oracle's
    parameters and Adam state before every minibatch and holds all 25 to 1e-5."""
    t = golden("train_small")
    n = golden("nets")
    ag = _agent(n_envs=64, batch_size=600, lr=0.00014)
    _load(ag, n)  # nets.npz holds the seed-3234 initial weights train_small started from
    b = [torch.as_tensor(t[k]).cuda() for k in ("obs", "actions", "logp", "masks", "advs", "vals")]
    hist = ag.update(*b, index_list=t["idx"]).cpu().numpy()
    np.testing.assert_allclose(hist[:, 0], t["actor_loss"], rtol=1e-4, atol=2e-5)
    np.testing.assert_allclose(hist[:, 1], t["critic_loss"], rtol=1e-4, atol=1e-6)
    # first minibatch (identical start parameters): the 1e-5 bar
    assert abs(hist[0, 0] - t["actor_loss"][0]) <= RTOL * abs(t["actor_loss"][0]) + ATOL
    assert abs(hist[0, 1] - t["critic_loss"][0]) <= RTOL * abs(t["critic_loss"][0]) + ATOL
    assert ag.actor_optim.param_groups[0]["lr"] == t["lr_final"]


def test_get_gaes_api(golden):
    g = golden("gae")
    ag = _agent(n_envs=64)
    for i in range(int(g["n"])):
        vals = [torch.tensor([[float(v)]]) for v in g[f"L{i}/val"]]
        adv = ag.get_GAEs(list(g[f"L{i}/rew"]), vals, list(g[f"L{i}/done"]))
        assert adv.dtype == np.float64 and np.array_equal(adv, g[f"L{i}/adv"])


def test_get_action_api():
    ag = _agent(n_envs=64, sample_seed=3)
    obs = [0.0] * 65
    mask = [True, False, True, False, False, True]
    for _ in range(20):
        (move, mark), lp = ag.get_action(obs, mask)
        assert move in (0, 2) and mark in (0, 1) and lp.shape == (1, 1) and torch.isfinite(lp).all()


def test_rollout_loop_matches_oracle():
    """Actions sampled on the GPU, replayed in the oracle: obs/masks/rewards/
    dones of the whole rollout agree bit-exactly; GAE equals the reference
    formula per episode fragment; stored log-probs equal a recomputation."""
    n, T = 512, 40
    cfg = dict(default_size=(6, 6), max_timestep=30)
    ag = _agent(n_envs=n, horizon=T, batch_size=5 * (n * T // 5), bootstrap=False, sample_seed=5,
                env_config=dict(cfg, seed_base=100))
    b = ag.rollout()
    ora = OracleEnv(n, seeds=np.arange(n, dtype=np.uint64) + np.uint64(100), **cfg)
    oo, om = ora.reset_all()
    obs = b["obs"].cpu().numpy()
    masks = b["masks"].cpu().numpy().astype(bool)
    act = b["act"].cpu().numpy()
    assert np.array_equal(obs[0], oo) and np.array_equal(masks[0], om)
    R = b["rew"].cpu().numpy()
    D = b["done"].cpu().numpy().astype(bool)
    for t in range(T):
        assert masks[t][np.arange(n)[:, None], np.arange(2)[None, :], act[t, :, :, 0]].all(), t
        oo, om, orw, od = ora.step_all(act[t], auto_reset=True)
        assert np.array_equal(obs[t + 1], oo) and np.array_equal(masks[t + 1], om), t
        assert np.array_equal(R[t], orw) and np.array_equal(D[t], od), t
    V = b["val"].cpu().numpy()
    A = b["adv"].cpu().numpy()
    for col in range(0, n, 37):
        s0, ref = 0, []
        for t in range(T):
            if D[t, col] or t == T - 1:
                dd = D[s0:t + 1, col].copy()
                dd[-1] = True
                ref.append(oppo.gae_fp32(list(R[s0:t + 1, col].astype(np.float64)), V[s0:t + 1, col], dd))
                s0 = t + 1
        assert np.array_equal(A[:, col], np.concatenate(ref)), col
    with torch.no_grad():
        lp = ag.policy_logp(b["obs"][:T].reshape(-1, 2, 65), b["act"].reshape(-1, 2, 2).float(),
                            b["masks"][:T].reshape(-1, 2, 6))
    np.testing.assert_allclose(lp.cpu().numpy(), b["logp"].reshape(-1).cpu().numpy(), rtol=1e-5, atol=2e-6)
    assert D.any()


def test_train_runs_and_learns_something():
    ag = _agent(n_envs=1024, horizon=8, batch_size=8190, epochs=2, sample_seed=9,
                env_config=dict(default_size=(4, 4), max_timestep=40, seed_base=0))
    ag.train()
    assert len(ag.history) == 2
    assert all(np.isfinite([h["actor_loss"], h["critic_loss"]]).all() for h in ag.history)
    assert ag.history[-1]["episodes"] > 0


@pytest.mark.parametrize("algo", ["mfma", "valu"])
@pytest.mark.parametrize("parity", [True, False])
def test_fused_front_matches_torch(parity, algo, monkeypatch):
    """csrc/actor_front.hip forward+backward == the module-by-module torch path
    (both backward algorithms: the MFMA attention products and the VALU form)."""
    from marlmaze import networks
    from marlmaze.networks import Actor, _FusedFront, front_params

    monkeypatch.setattr(networks, "FRONT_BWD_ALGO", algo)

    torch.manual_seed(0)
    actor = Actor([264, 264, 264], parity_mode=parity).cuda()
    with torch.no_grad():  # non-trivial attention weights
        for p in actor.parameters():
            p.mul_(3.0)
    B = 3000
    x = torch.randn(B, 65, device="cuda")
    dh = torch.randn(B, 460, device="cuda")
    pr, at = actor.projection, actor.attention
    params = front_params(pr, at)
    href = at(pr(x))
    gref = torch.autograd.grad(href, params, dh)
    # fp64 truth: the fused kernels' summation order differs from torch's (both are fp32 roundings of it)
    a64 = copy.deepcopy(actor).double()
    p64 = front_params(a64.projection, a64.attention)
    h64 = a64.attention(a64.projection(x.double()))
    g64 = torch.autograd.grad(h64, p64, dh.double())
    h = _FusedFront.apply(x, parity, *params)
    # weights x3: large attention logits amplify summation-order differences
    e_ours = (h.double() - h64).abs().max().item()
    e_torch = (href.double() - h64).abs().max().item()
    assert e_ours <= 2.0 * e_torch + 1e-6, (e_ours, e_torch)
    np.testing.assert_allclose(h.detach().cpu().numpy(), href.detach().cpu().numpy(), rtol=1e-4, atol=5e-4)
    g = torch.autograd.grad(h, params, dh)
    for a, b, t in zip(g, gref, g64):
        e_ours = (a.double() - t).abs().max().item()
        e_torch = (b.double() - t).abs().max().item()
        # within torch's own fp32 error or 1e-5 of the tensor's max (the kernel's long fp32 sums over
        # samples are fixed-order and serial per thread; torch reduces pairwise)
        assert e_ours <= max(2.0 * e_torch, 1e-5 * t.abs().max().item()), (e_ours, e_torch)
        np.testing.assert_allclose(a.cpu().numpy(), b.cpu().numpy(), rtol=1e-4, atol=1e-3 * b.abs().max().item())


@pytest.mark.parametrize("B", [1, 15, 17, 3001, 131072])
@pytest.mark.parametrize("parity", [True, False])
def test_front_forward_row2_bit_identical(parity, B):
    """k_front_fwd2 (two query rows per lane) writes the same bits as
    k_front_fwd (one row per lane): same per-row arithmetic; ragged B (not a
    multiple of the 16 samples per workgroup iteration) and the persistent
    grid's multi-iteration case (131,072 rows)."""
    import ctypes

    from marlmaze import _lib
    from marlmaze.networks import Actor, front_params

    torch.manual_seed(2)
    actor = Actor([264, 264, 264], parity_mode=parity).cuda()
    with torch.no_grad():
        for p in actor.parameters():
            p.mul_(3.0)
    x = torch.randn(B, 65, device="cuda")
    params = front_params(actor.projection, actor.attention)
    L = _lib.lib()
    ws = torch.empty(L.mm_actor_front_ws_len(), dtype=torch.float32, device="cuda")
    ptrs = [p.data_ptr() for p in params]
    wp = (ctypes.c_void_p * 23)(*ptrs[:23])
    bp = (ctypes.c_void_p * 23)(*ptrs[23:46])
    s = _lib.stream_ptr()
    _lib.check(L.mm_actor_front_prep(wp, bp, ptrs[46], ptrs[47], ptrs[48], _lib.ptr(ws), s), "prep")
    hs = []
    for algo in ("row1", "row2"):
        h = torch.full((B + 1, 460), float("nan"), device="cuda")  # one guard row past B
        _lib.check(L.mm_actor_front_fwd_ex(_lib.ptr(ws), _lib.ptr(x), 65, B, int(parity), _lib.ptr(h),
                                           _lib.FRONT_FWD[algo], s), algo)
        hs.append(h)
    torch.cuda.synchronize()
    assert torch.isfinite(hs[1][:B]).all()
    assert torch.isnan(hs[1][B]).all()  # nothing written past B
    assert torch.equal(hs[0][:B], hs[1][:B])


@pytest.mark.parametrize("B", [1, 2, 15, 17, 3001, 131072])
@pytest.mark.parametrize("parity", [True, False])
def test_front_forward_mfma_vs_fp64(parity, B):
    """k_front_fwd_mfma (S^T on the fp32 MFMA, ctx^T = V^T P^T on the x2 f16 MFMA, h = t + ctx
    accumulated in the MFMA) against an fp64 evaluation of the same modules: within twice the VALU
    kernel's error or 1e-6 of max|h| (the x2 GEMMs' bar), every row written and nothing past B (ragged B: odd counts leave
    a wavefront's second sample and a workgroup's tail empty; 131,072 rows: the persistent grid's
    multi-iteration case), and the fp16 form the round to nearest of the fp32 one."""
    import copy
    import ctypes

    from marlmaze import _lib
    from marlmaze.networks import Actor, front_params

    torch.manual_seed(2)
    actor = Actor([264, 264, 264], parity_mode=parity).cuda()
    with torch.no_grad():  # non-trivial attention weights
        for p in actor.parameters():
            p.mul_(3.0)
    x = torch.randn(B, 65, device="cuda")
    params = front_params(actor.projection, actor.attention)
    L = _lib.lib()
    ws = torch.empty(L.mm_actor_front_ws_len(), dtype=torch.float32, device="cuda")
    ptrs = [p.data_ptr() for p in params]
    wp = (ctypes.c_void_p * 23)(*ptrs[:23])
    bp = (ctypes.c_void_p * 23)(*ptrs[23:46])
    s = _lib.stream_ptr()
    _lib.check(L.mm_actor_front_prep(wp, bp, ptrs[46], ptrs[47], ptrs[48], _lib.ptr(ws), s), "prep")
    hs = {}
    for algo in ("row1", "mfma"):
        h = torch.full((B + 1, 460), float("nan"), device="cuda")  # one guard row past B
        _lib.check(L.mm_actor_front_fwd_ex(_lib.ptr(ws), _lib.ptr(x), 65, B, int(parity), _lib.ptr(h),
                                           _lib.FRONT_FWD[algo], s), algo)
        hs[algo] = h
    h16 = torch.full((B + 1, 460), float("nan"), device="cuda", dtype=torch.float16)
    _lib.check(L.mm_actor_front_fwd_h16_ex(_lib.ptr(ws), _lib.ptr(x), 65, B, int(parity), _lib.ptr(h16),
                                           _lib.FRONT_FWD["mfma"], s), "h16 mfma")
    torch.cuda.synchronize()
    h = hs["mfma"]
    assert torch.isfinite(h[:B]).all()
    assert torch.isnan(h[B]).all()  # nothing written past B
    assert torch.isnan(h16[B]).all()
    assert torch.equal(h16[:B], h[:B].half())
    a64 = copy.deepcopy(actor).double()
    with torch.no_grad():
        h64 = a64.attention(a64.projection(x.double()))
    e_mfma = (h[:B].double() - h64).abs().max().item()
    e_row1 = (hs["row1"][:B].double() - h64).abs().max().item()
    # the attention-weighted sum runs on the x2 f16 MFMA (FRONT_FM_PV=1: operands split hi + 2^-11 lo, 2^-22
    # relative per product): the x2 GEMMs' 1e-6 bar, relative to max|h|
    assert e_mfma <= max(2.0 * e_row1, 1e-6 * h64.abs().max().item()), (e_mfma, e_row1)


@pytest.mark.parametrize("parity", [True, False])
def test_front_backward_mfma_vs_fp64(parity, monkeypatch):
    """The front-end's parameter gradients against an fp64 evaluation of the
    same modules: the MFMA backward (bf16x3 products, fp32-class) is as close to
    fp64 as the VALU fp32 backward -- within twice its error, and within 1e-5
    of each tensor's max|g| (sums over 20,000 samples)."""
    from marlmaze import networks
    from marlmaze.networks import Actor, _FusedFront, front_params

    torch.manual_seed(1)
    actor = Actor([264, 264, 264], parity_mode=parity).cuda()
    with torch.no_grad():
        for p in actor.parameters():
            p.mul_(3.0)
    B = 20000
    x = torch.randn(B, 65, device="cuda")
    if parity:  # the facing one-hot the env writes (the actor reads only obs[0:4], Q1)
        x[:, :4] = torch.nn.functional.one_hot(torch.randint(0, 4, (B,), device="cuda"), 4).float()
    dh = torch.randn(B, 460, device="cuda") / B
    params = front_params(actor.projection, actor.attention)
    a64 = Actor([264, 264, 264], parity_mode=parity).double()
    a64.load_state_dict({k: v.detach().cpu().double() for k, v in actor.state_dict().items()})
    p64 = front_params(a64.projection, a64.attention)
    h64 = a64.attention(a64.projection(x.cpu().double()))
    g64 = torch.autograd.grad(h64, p64, dh.cpu().double())
    errs = {}
    for algo in ("mfma", "valu"):
        monkeypatch.setattr(networks, "FRONT_BWD_ALGO", algo)
        h = _FusedFront.apply(x, parity, *params)
        g = torch.autograd.grad(h, params, dh)
        errs[algo] = [((a.double().cpu() - b).abs().max() / b.abs().max().clamp_min(1e-30)).item()
                      for a, b in zip(g, g64)]
    worst = max(range(len(g64)), key=lambda k: errs["mfma"][k])
    print(f"front bwd vs fp64 (parity={parity}): mfma max {errs['mfma'][worst]:.2e}, valu {errs['valu'][worst]:.2e}")
    for k in range(len(g64)):
        assert errs["mfma"][k] <= max(2 * errs["valu"][k], 1e-5), (k, errs["mfma"][k], errs["valu"][k])


def test_checkpoint_round_trip_reference_format(tmp_path, golden):
    """F1 (PPO.py:222-238): a checkpoint written the reference's way (CPU
    torch Actor/Critic + Adam state dicts) loads into the GPU PPO, training
    continues from its Adam state, and the GPU PPO's own checkpoint loads back
    on the CPU with weights_only=True into the reference-shaped modules."""
    c = golden("ckpt_logits")
    actor, critic = oppo.OActor(), oppo.OCritic()
    actor.load_state_dict({k[6:]: torch.as_tensor(c[k]) for k in c.files if k.startswith("actor/")})
    critic.load_state_dict({k[7:]: torch.as_tensor(c[k]) for k in c.files if k.startswith("critic/")})
    aopt = torch.optim.Adam(actor.parameters(), lr=1.4e-4)
    copt = torch.optim.Adam(critic.parameters(), lr=1.4e-4)
    for opt, m in ((aopt, actor), (copt, critic)):  # give Adam a state, as a trained reference run has
        opt.zero_grad()
        sum(p.sum() for p in m.parameters()).backward()
        opt.step()
    ref_path = str(tmp_path / "PPO.pth")
    torch.save({"actor": actor.state_dict(), "critic": critic.state_dict(), "actor_optim": aopt.state_dict(),
                "critic_optim": copt.state_dict()}, ref_path)
    ag = PPO(2, n_envs=64, load=True, model_path=ref_path, verbose=False, save=False)
    for k, v in actor.state_dict().items():
        assert torch.equal(ag.actor.state_dict()[k].cpu(), v), k
    st = ag.actor_optim.state_dict()["state"]
    assert float(st[0]["step"]) == 1.0 and torch.equal(st[0]["exp_avg"].cpu(), aopt.state_dict()["state"][0]["exp_avg"])
    o = torch.as_tensor(c["obs"]).cuda()
    with torch.no_grad():
        mv, _ = ag.actor(o.reshape(-1, 65))
    mv_ref, _ = actor(o.reshape(-1, 65).cpu())
    np.testing.assert_allclose(mv.cpu().numpy(), mv_ref.detach().numpy(), rtol=RTOL, atol=1e-5)
    # the GPU side writes a CPU-loadable checkpoint with the reference keys
    ag.model_path = str(tmp_path / "PPO_gpu.pth")
    ag.save_parameters()
    sd = torch.load(ag.model_path, weights_only=True)
    assert set(sd) == {"actor", "critic", "actor_optim", "critic_optim"}
    actor2 = oppo.OActor()
    actor2.load_state_dict(sd["actor"])
    aopt2 = torch.optim.Adam(actor2.parameters(), lr=1.4e-4)
    aopt2.load_state_dict(sd["actor_optim"])
    assert all(not t.is_cuda for t in sd["actor"].values())


@pytest.mark.parametrize("M,N,K", [(1, 264, 460), (777, 264, 264), (20000, 460, 264), (5000, 64, 132),
                                   (300, 6, 264), (4100, 272, 8)])
def test_x3_gemm_accuracy(M, N, K):
    """csrc/x3mlp.hip: the bf16x3-split GEMMs (A pre-split or fp32, bias + ReLU
    epilogue, fp32 or fragment-order output) are as accurate as an fp32 GEMM:
    error vs fp64 relative to sum|a b| below 1e-6 (fp32 GEMMs: ~3e-7)."""
    from marlmaze import x3

    g = torch.Generator(device="cuda").manual_seed(M)
    a = torch.randn(M, K, device="cuda", generator=g)
    w = torch.randn(N, K, device="cuda", generator=g) * 0.05
    bias = torch.randn(N, device="cuda", generator=g)
    ref = torch.relu(a.double() @ w.double().t() + bias.double())
    scale = a.double().abs() @ w.double().abs().t() + bias.double().abs()
    tw = x3.pack(w)
    for src in (a, x3.pack(a)):
        c, _ = x3.nt(src, tw, bias=bias, relu=True)
        assert ((c.double() - ref).abs() / scale).max().item() < 1e-6
    c2, _ = x3.nt(a, tw)
    assert ((c2.double() - a.double() @ w.double().t()).abs() / scale).max().item() < 1e-6
    if N <= 272:  # fragment-order (TP) output == the fp32 output's split, exactly
        ctp = x3.TP(M, N, "cuda")
        x3.nt(a, tw, bias=bias, relu=True, out_tp=ctp, want_f32=False)
        c, _ = x3.nt(a, tw, bias=bias, relu=True)
        assert torch.equal(x3.unpack(ctp), c)
    # the packed operand round-trips exactly (three bf16 parts carry all 24 bits)
    assert torch.equal(x3.unpack(x3.pack(a)), a)
    assert torch.equal(x3.unpack(x3.pack(w.t().contiguous(), trans=True)), w)


@pytest.mark.parametrize("M", [5, 1000, 40000])
def test_x3_relu_bits(M):
    """ReLU bit masks: written by a forward GEMM (mbits_out), applied by the next
    layer's input-gradient GEMM (mbits_in) == (dY W) * (y > 0) of torch."""
    from marlmaze import x3

    g = torch.Generator(device="cuda").manual_seed(M)
    h = torch.randn(M, 264, device="cuda", generator=g)
    w1 = torch.randn(264, 264, device="cuda", generator=g) * 0.06
    b1 = torch.randn(264, device="cuda", generator=g) * 0.1
    w2 = torch.randn(264, 264, device="cuda", generator=g) * 0.06
    dy = torch.randn(M, 264, device="cuda", generator=g)
    mb = x3.mbits(M, "cuda")
    y, _ = x3.nt(h, x3.pack(w1), bias=b1, relu=True, mbits_out=mb)
    dx, _ = x3.nt(dy, x3.pack(w2, trans=True), mbits_in=mb)
    ref = (dy.double() @ w2.double()) * (y > 0)
    scale = dy.double().abs() @ w2.double().abs()
    assert ((dx.double() - ref).abs() / scale).max().item() < 1e-6
    assert torch.equal(dx == 0, (y <= 0) | (ref == 0))


@pytest.mark.parametrize("heads", [False, True])
def test_x3_trunk_gradients_vs_fp64(heads):
    """The actor MLP on the x3 GEMMs -- _EngineTrunk (trunk) and _EngineActor (trunk +
    heads: forward, ReLU bits, the fused heads backward, input / weight / bias
    gradients with the bias sums from the GEMM epilogues) -- against an fp64
    evaluation linearised at the same ReLU pattern (a ReLU whose input is within
    fp32 rounding of 0 may flip under any change of summation order, for the
    fp32 library GEMMs just as here, so the pattern is taken from the forward
    under test).  Tolerance: 1e-6 of max|ref| for outputs, 2e-5 for gradients
    (sums over 40,000 rows)."""
    from marlmaze import x3
    from marlmaze.networks import Actor, _EngineActor, _EngineTrunk

    torch.manual_seed(1)
    actor = Actor([264, 264, 264]).cuda()
    M = 40000
    h0 = torch.randn(M, 460, device="cuda").requires_grad_(True)
    params = [t for lin in actor.layers for t in (lin.weight, lin.bias)]
    wh, bh = (t.detach().clone().requires_grad_(True) for t in actor.heads())
    with torch.no_grad():
        wh.mul_(100.0)  # heads at the scale of the hidden layers (init is x0.01)
    if heads:
        dout = torch.randn(M, 6, device="cuda")
        out = _EngineActor.apply("x3", h0, wh, bh, *params)
        inputs = [h0, wh, bh] + params
    else:
        dout = torch.randn(M, 264, device="cuda")
        out = _EngineTrunk.apply("x3", h0, *params)
        inputs = [h0] + params
    got = [out.detach()] + list(torch.autograd.grad(out, inputs, dout))
    pattern = []  # the x3 forward's ReLU pattern (the same GEMMs the functions run)
    with torch.no_grad():
        h = h0.detach()
        for i in range(3):
            h, _ = x3.nt(h, x3.pack(params[2 * i]), bias=params[2 * i + 1], relu=True)
            pattern.append(h > 0)
    in64 = [t.detach().double().cpu().requires_grad_(True) for t in inputs]
    x64 = in64[0]
    p64 = in64[3:] if heads else in64[1:]
    h = x64
    for i in range(3):
        h = (h @ p64[2 * i].t() + p64[2 * i + 1]) * pattern[i].cpu()
    if heads:
        h = h @ in64[1].t() + in64[2]
    ref = [h.detach()] + list(torch.autograd.grad(h, in64, dout.double().cpu()))
    for n, (a, r) in enumerate(zip(got, ref)):
        tol = 1e-6 if n == 0 else 2e-5
        err = (a.double().cpu() - r).abs().max().item() / r.abs().max().item()
        assert err < tol, (n, err)


@pytest.mark.parametrize("M", [1, 300, 20000])
def test_fused_policy_loss_matches_torch(M):
    """mm_ppo_loss / mm_ppo_loss_bwd (PPO.py:62-72 with get_log_probs
    PPO.py:154-168) == the torch formula on the same head logits: loss at 1e-6
    relative, d loss / d heads at 1e-6 of its max.  Ratios are spread around the
    clip range so that both sides of min() and the clamp's edges are exercised."""
    from marlmaze.PPO import _PolicyLoss

    g = torch.Generator(device="cuda").manual_seed(M)
    heads = torch.randn(2 * M, 6, device="cuda", generator=g) * 2
    masks = torch.rand(2 * M, 6, device="cuda", generator=g) < 0.7
    masks[:, 4] = True  # stay is always legal (maze_agent.py:136)
    mv = torch.where(masks[:, :5], torch.rand(2 * M, 5, device="cuda", generator=g), torch.zeros(())).argmax(1)
    mark = (torch.rand(2 * M, device="cuda", generator=g) < 0.5) & masks[:, 5]
    act = torch.stack([mv, mark.long()], 1)
    adv = torch.randn(M, device="cuda", generator=g)

    def logp_torch(z):
        ml = z[:, :5].masked_fill(~masks[:, :5], float("-inf"))
        lp = torch.log_softmax(ml, -1).gather(1, act[:, 0:1]).squeeze(1)
        kl = z[:, 5].masked_fill(~masks[:, 5], float("-inf"))
        p = torch.sigmoid(kl)
        p = torch.where(act[:, 1] != 0, p, 1 - p)
        return (lp + torch.log(p)).view(M, 2).sum(1)

    with torch.no_grad():
        old = logp_torch(heads) + torch.randn(M, device="cuda", generator=g) * 0.3  # ratios around 1
    z1 = heads.clone().requires_grad_(True)
    cur = logp_torch(z1)
    r = torch.exp(cur - old)
    ref = -torch.mean(torch.min(r * adv, torch.clamp(r, 0.8, 1.2) * adv))
    gref, = torch.autograd.grad(ref, z1)
    z2 = heads.clone().requires_grad_(True)
    loss = _PolicyLoss.apply(z2, masks, act.to(torch.int8), old, adv, 0.2)
    got, = torch.autograd.grad(loss, z2)
    assert abs(loss.item() - ref.item()) <= 1e-6 * abs(ref.item()) + 1e-7, (loss.item(), ref.item())
    assert (got - gref).abs().max().item() <= 1e-6 * gref.abs().max().item() + 1e-9


@pytest.mark.parametrize("n", [512, 4096])
def test_graph_rollout_equals_eager(n):
    """PPO(graph_rollout=True) -- the fixed-horizon rollout captured once as a HIP
    graph and replayed (the sampler's Philox base offset read from the device)
    -- gives bit-identical batches to the uncaptured rollout over several
    iterations (episodes and auto-resets crossing the batches), including after
    an update changed the weights the graph reads in place."""
    cfg = dict(default_size=(6, 6), max_timestep=20, seed_base=7)
    T = 8
    ags = [_agent(n_envs=n, horizon=T, batch_size=n * T, sample_seed=5, env_config=cfg, graph_rollout=g)
           for g in (False, True)]
    for it in range(4):
        outs = []
        for ag in ags:
            b = ag.rollout()
            outs.append({k: b[k].clone() for k in ("obs", "masks", "act", "logp", "val", "rew", "done", "adv", "rtg")})
            if it == 1:  # one update step: the captured graph must see the new weights
                B = T * n
                idx = torch.arange(B, device="cuda")[: B // 5]
                ag.minibatch_step(b["obs"][:T].reshape(B, 2, 65)[idx], b["act"].reshape(B, 2, 2)[idx],
                                  b["logp"].reshape(B)[idx], b["adv"].reshape(B)[idx], b["rtg"].reshape(B)[idx],
                                  b["masks"][:T].reshape(B, 2, 6)[idx])
            ag._carry_over()
        for k in outs[0]:
            assert torch.equal(outs[0][k], outs[1][k]), (it, k)
    assert ags[1]._graph is not None and ags[0]._sample_offset == ags[1]._sample_offset


@pytest.mark.parametrize("bootstrap", [False, True])
def test_batched_rollout_critic_equals_per_step(bootstrap, monkeypatch):
    """The rollout's critic values from one launch after the env loop (PPO.ROLLOUT_BATCHED_CRITIC, the
    default) are bit-identical to the per-step form (one launch per step, before the step's actions): the
    values depend on the stored observations only and mm_critic_value's arithmetic per row does not depend
    on the rows launched beside it.  Every other buffer of the batch is identical too."""
    from marlmaze import PPO as ppo_mod

    cfg = dict(default_size=(6, 6), max_timestep=20, seed_base=11)
    T, n = 8, 512
    outs = []
    for batched in (False, True):
        monkeypatch.setattr(ppo_mod, "ROLLOUT_BATCHED_CRITIC", batched)
        ag = _agent(n_envs=n, horizon=T, batch_size=n * T, sample_seed=9, env_config=cfg, bootstrap=bootstrap)
        res = []
        for _ in range(3):
            b = ag.rollout()
            res.append({k: b[k].clone() for k in ("obs", "act", "logp", "val", "rew", "done", "adv", "rtg")})
            ag._carry_over()
        outs.append(res)
    for it in range(3):
        for k in outs[0][it]:
            assert torch.equal(outs[0][it][k], outs[1][it][k]), (bootstrap, it, k)


@pytest.mark.parametrize("dtype", ["f32", "f16"])
def test_fresh_batch_logp_matches_rollout(dtype):
    """Before the first optimizer step, the update's log-probs of a fresh rollout batch equal the rollout's
    (PPO ratio 1): the update's actor forward takes the same trunk kernels per row and its heads
    (mm_heads_fwd) the rollout's fused-head arithmetic (mm_head_sample), for fp32-class and fp16 GEMMs alike;
    only the log-softmax formula differs (torch's vs the sampler's), hence 1e-5."""
    torch.manual_seed(5)
    ag = _agent(n_envs=512, horizon=8, dtype=dtype, sample_seed=3,
                env_config=dict(default_size=(10, 10), max_timestep=1200, seed_base=0))
    with torch.no_grad():
        ag.actor.move_head.weight.mul_(30.0)  # non-trivial policies (the 0.01 init makes every logit ~0)
        ag.actor.mark_head.weight.mul_(30.0)
    b_obs, b_act, b_lp, _, _, b_masks, _, _ = ag.get_batch()
    with torch.no_grad():
        lp = ag.policy_logp(b_obs, b_act, b_masks)
    fin = torch.isfinite(b_lp)
    assert fin.float().mean().item() > 0.99
    err = (lp[fin] - b_lp[fin]).abs().max().item()
    assert err <= 1e-5, (dtype, err)
