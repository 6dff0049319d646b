"""The fused small-M actor trunk (mm_trunk3, csrc/x3mlp.hip k_trunk3): the rollout's three ReLU layers
(networks.py:35-36 under no_grad) in one launch.  It must equal the three per-layer GEMMs it replaces BIT
FOR BIT (same fragment conversion, same MFMA sequence per output tile, same epilogue), at every precision,
at ragged row counts and at shapes other than the actor's; the rollout-level parity against the fp32
oracle is test_gpu_ppo.py's / test_gpu_update_parity.py's (the 4,096-maze rollout forward runs it)."""
import pytest
import torch

from marlmaze import networks, x3

pytestmark = pytest.mark.gpu


def _layers(K0, Ns, prec, g):
    ws, bs, packs = [], [], []
    k = K0
    for n in Ns:
        w = torch.randn(n, k, device="cuda", generator=g) * (1.0 / k ** 0.5)
        b = torch.randn(n, device="cuda", generator=g) * 0.1
        ws.append(w)
        bs.append(b)
        packs.append(x3.pack(w, prec=prec))
        k = n
    return ws, bs, packs


def _three_gemms(h0, packs, bs):
    h = h0
    for p, b in zip(packs, bs):
        h = x3.gemm(h, p, bias=b, relu=True)
    return h


@pytest.mark.parametrize("prec", ["x2", "f16", "x3"])
@pytest.mark.parametrize("M", [1, 17, 31, 32, 33, 47, 48, 49, 300, 4096, 8192, 8195, 16383])
def test_trunk3_equals_three_gemms(prec, M):
    g = torch.Generator(device="cuda").manual_seed(M * 7 + len(prec))
    _, bs, packs = _layers(460, (264, 264, 264), prec, g)
    h0 = torch.relu(torch.randn(M, 460, device="cuda", generator=g))
    assert x3.trunk3_ok(M, h0, packs, prec)
    y = x3.trunk3(h0, packs, bs)
    ref = _three_gemms(h0, packs, bs)  # M < 16,384: the streaming kernel k_x3nt
    assert torch.equal(y, ref)


@pytest.mark.parametrize("prec,K0,Ns", [("x2", 64, (128, 64, 272)), ("x2", 128, (100, 36, 17)),
                                        ("x2", 512, (272, 272, 1)), ("f16", 96, (48, 272, 264)),
                                        ("x3", 256, (256, 264, 264)), ("x3", 96, (16, 40, 8))])
def test_trunk3_other_shapes(prec, K0, Ns):
    g = torch.Generator(device="cuda").manual_seed(K0 + sum(Ns))
    _, bs, packs = _layers(K0, Ns, prec, g)
    M = 1000
    h0 = torch.randn(M, K0, device="cuda", generator=g)
    y = x3.trunk3(h0, packs, bs)
    assert y.shape == (M, Ns[-1])
    assert torch.equal(y, _three_gemms(h0, packs, bs))


def test_trunk3_strided_input_and_output_and_no_bias():
    g = torch.Generator(device="cuda").manual_seed(3)
    _, _, packs = _layers(460, (264, 264, 264), "x2", g)
    big = torch.randn(2000, 472, device="cuda", generator=g)
    h0 = big[:, :460]  # lda 472
    out = torch.full((2000, 280), 7.0, device="cuda")
    y = x3.trunk3(h0, packs, [None, None, None], out=out[:, :264])
    assert torch.equal(y, _three_gemms(h0.contiguous(), packs, [None, None, None]))
    assert bool((out[:, 264:] == 7.0).all())  # nothing written past N


# the precision's GEMM bar (tests/test_gpu_gemm.py TOL), relative to the |.|-composition of the three layers
_GEMM_TOL = {"x3": 1e-6, "x2": 1e-6, "f16": 2e-3}


@pytest.mark.parametrize("prec,M", [("x2", 20000), ("x2", 32768), ("x3", 16384), ("f16", 32768), ("f16", 65536),
                                    ("f16", 131072)])
def test_trunk3_large_m_matches_b_resident_path(prec, M):
    """Every row count up to networks._TRUNK_MAX_ROWS_DEFAULT[prec] (x2 32,768, x3 16,384, f16 131,072 --
    configs[4]'s rollout runs 65,536 rows a step): at >= 16,384 rows the per-layer GEMMs run on k_bres (another
    k-tail form and accumulation order, so not bit-identical), and the fused trunk equals them at the
    precision's GEMM bar: |y - y_layers| <= TOL * S3, where S3 = |.|-composition of the three layers
    (s1 = |h0| |W0|^T + |b0|, s2 = s1 |W1|^T + |b1|, S3 = s2 |W2|^T + |b2|: the bound a per-layer relative
    error propagates under).  Both are also held to the fp64 composition at 3 x TOL (one rounding per layer)."""
    assert M <= networks._TRUNK_MAX_ROWS_DEFAULT[prec]
    g = torch.Generator(device="cuda").manual_seed(11 + M)
    ws, bs, packs = _layers(460, (264, 264, 264), prec, g)
    h0 = torch.relu(torch.randn(M, 460, device="cuda", generator=g))
    assert x3.trunk3_ok(M, h0, packs, prec)
    y, ref = x3.trunk3(h0, packs, bs), _three_gemms(h0, packs, bs)
    h64, s = h0.double(), h0.double().abs()
    for w, b in zip(ws, bs):
        h64 = torch.relu(h64 @ w.double().t() + b.double())
        s = s @ w.double().abs().t() + b.double().abs()
    tol = _GEMM_TOL[prec]
    e_layers = ((y.double() - ref.double()).abs() / s).max().item()
    e_fused, e_ref = (((t.double() - h64).abs() / s).max().item() for t in (y, ref))
    print(f"trunk3 {prec} M={M}: fused vs per-layer {e_layers:.2e}, fused vs fp64 {e_fused:.2e}, "
          f"per-layer vs fp64 {e_ref:.2e} (of S3)")
    assert e_layers <= tol, e_layers
    assert e_fused <= 3 * tol and e_ref <= 3 * tol, (e_fused, e_ref)


@pytest.mark.parametrize("prec,M", [("x2", 32768), ("f16", 131072)])
def test_trunk3_head_sample_at_its_row_limit(prec, M):
    """The rollout's fused form (trunk + heads + draws) at its largest enabled row count: legal actions,
    log-probs consistent with its own logits (1e-5), logits at the precision's bar against the per-layer
    GEMMs + the fp32 heads."""
    from marlmaze import ops

    g = torch.Generator(device="cuda").manual_seed(200 + M)
    ws, bs, packs = _layers(460, (264, 264, 264), prec, g)
    hw, hb = _heads(g)
    h0 = torch.relu(torch.randn(M, 460, device="cuda", generator=g))
    mk = _masks(M, g)
    assert x3.trunk3_head_sample_ok(M, h0, packs, prec)
    act = torch.full((M, 2), -9, dtype=torch.int8, device="cuda")
    lp, jl, lg = torch.empty(M, device="cuda"), torch.empty(M // 2, device="cuda"), torch.empty(M, 6, device="cuda")
    x3.trunk3_head_sample(h0, packs, bs, hw, hb, mk, 77, 0, act, lp, jl, logits=lg)
    ref_h = _three_gemms(h0, packs, bs)
    ref_lg = ref_h @ hw.t() + hb
    s = (ref_h.abs() @ hw.abs().t() + hb.abs()).double()
    assert (((lg.double() - ref_lg.double()).abs()) / s).max().item() <= 3 * _GEMM_TOL[prec]
    mv = act[:, 0].long()
    assert bool(((mv >= 0) & (mv < 5)).all()) and bool(mk.gather(1, mv.view(-1, 1)).bool().all())
    # log-probs from the kernel's own logits (the draw's arithmetic)
    ml = lg[:, :5].masked_fill(~mk[:, :5].bool(), float("-inf"))
    want = torch.log_softmax(ml, 1).gather(1, mv.view(-1, 1)).squeeze(1)
    p = torch.sigmoid(lg[:, 5].masked_fill(~mk[:, 5].bool(), float("-inf")))
    want = want + torch.log(torch.where(act[:, 1] != 0, p, 1 - p))
    assert torch.allclose(lp, want, rtol=1e-5, atol=1e-5)
    assert torch.allclose(jl, lp.view(-1, 2).sum(1), rtol=1e-6, atol=1e-6)
    del ops


def test_actor_trunk_uses_fused_launch_bit_identically(monkeypatch):
    torch.manual_seed(4)
    actor = networks.Actor(hidden_sizes=(264, 264, 264)).cuda()
    x = torch.randn(8192, 65, device="cuda")
    with torch.no_grad():
        y = actor.trunk(x)
        monkeypatch.setattr(networks, "TRUNK_MAX_ROWS", 0)
        y0 = actor.trunk(x)
    assert torch.equal(y, y0)


def test_trunk3_rejects_unsupported_shapes():
    g = torch.Generator(device="cuda").manual_seed(5)
    _, _, packs = _layers(460, (264, 300, 264), "x2", g)  # N1 > 272
    h0 = torch.randn(64, 460, device="cuda", generator=g)
    assert not x3.trunk3_ok(64, h0, packs, "x2")
    _, _, packs = _layers(460, (264, 264, 264), "x2", g)
    assert not x3.trunk3_ok(64, torch.randn(64, 458, device="cuda"), packs, "x2")  # h0 width != W0's


def test_trunk3_two_row_tile_form_equals(monkeypatch):
    """MARLMAZE_TRUNK_RT=2 / MARLMAZE_TRUNK_D=3 select the other instantiations (read once per process by
    the library: here through a subprocess-free check of both env-independent forms is not possible, so
    the x3 path -- which takes the two-row-tile form at the actor's shape -- stands for it)."""
    g = torch.Generator(device="cuda").manual_seed(9)
    _, bs, packs = _layers(460, (264, 264, 264), "x3", g)
    h0 = torch.relu(torch.randn(1000, 460, device="cuda", generator=g))
    assert torch.equal(x3.trunk3(h0, packs, bs), _three_gemms(h0, packs, bs))


# ---- the trunk + heads + draws in one launch (mm_trunk3_head_sample) ----

def _heads(g, K=264):
    return (torch.randn(6, K, device="cuda", generator=g) * 0.2, torch.randn(6, device="cuda", generator=g) * 0.1)


def _masks(M, g):
    mk = (torch.rand(M, 6, device="cuda", generator=g) < 0.6).to(torch.uint8)
    mk[:, 4] = 1  # at least one legal move per row (an all-illegal row's log-prob is NaN either way)
    return mk.contiguous()


@pytest.mark.parametrize("prec", ["x2", "f16", "x3"])
@pytest.mark.parametrize("M", [1, 2, 33, 300, 4096, 8192, 8193])
def test_trunk3_head_sample_equals_trunk_then_head_sample(prec, M):
    from marlmaze import ops

    g = torch.Generator(device="cuda").manual_seed(100 + M + len(prec))
    _, bs, packs = _layers(460, (264, 264, 264), prec, g)
    hw, hb = _heads(g)
    h0 = torch.relu(torch.randn(M, 460, device="cuda", generator=g))
    mk = _masks(M, g)
    assert x3.trunk3_head_sample_ok(M, h0, packs, prec)
    off_dev = torch.tensor([7], dtype=torch.int64, device="cuda")
    act = torch.full((M, 2), -9, dtype=torch.int8, device="cuda")
    lp, jl = torch.empty(M, device="cuda"), torch.empty((M + 1) // 2, device="cuda")
    lg, h3 = torch.empty(M, 6, device="cuda"), torch.empty(M, 264, device="cuda")
    L = x3._lib.lib()
    x3.trunk3_head_sample(h0, packs, bs, hw, hb, mk, 1234, 5, act, lp, jl, logits=lg, offset_dev=off_dev, h3=h3)
    ref_h = x3.trunk3(h0, packs, bs)
    act_r = torch.empty((M, 2), dtype=torch.int8, device="cuda")
    lp_r, jl_r = torch.empty(M, device="cuda"), torch.empty((M + 1) // 2, device="cuda")
    lg_r = torch.empty(M, 6, device="cuda")
    ops.head_sample(ref_h, hw, hb, mk, 1234, 5, actions=act_r, logp=lp_r, joint_logp=jl_r, logits=lg_r,
                    offset_dev=off_dev)
    assert torch.equal(h3, ref_h)
    assert torch.equal(lg, lg_r)
    assert torch.equal(act, act_r)
    assert torch.equal(lp, lp_r) and torch.equal(jl, jl_r)
    del L


def test_actor_sample_actions_fused_equals_unfused(monkeypatch):
    from marlmaze import ops

    torch.manual_seed(6)
    actor = networks.Actor(hidden_sizes=(264, 264, 264)).cuda()
    g = torch.Generator(device="cuda").manual_seed(6)
    M = 8192
    x = torch.randn(M, 65, device="cuda", generator=g)
    mk = _masks(M, g)
    hw, hb = actor.heads()
    outs = []
    for rows in (None, 0):
        monkeypatch.setattr(networks, "TRUNK_MAX_ROWS", rows)
        act = torch.empty((M, 2), dtype=torch.int8, device="cuda")
        lp, jl = torch.empty(M, device="cuda"), torch.empty(M // 2, device="cuda")
        with torch.no_grad():
            actor.sample_actions(x, hw, hb, mk, 99, 3, act, lp, jl)
        outs.append((act, lp, jl))
    for a, b in zip(*outs):
        assert torch.equal(a, b)
    del ops
