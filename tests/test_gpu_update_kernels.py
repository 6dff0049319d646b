"""The update's small kernels (csrc/update_kernels.hip) and the flat optimizer
(marlmaze/update.py) against torch:

* mm_colsum -- the bias gradients' column sums -- vs fp64;
* mm_mse_loss + mm_losses_final -- nn.MSELoss (PPO.py:78-80) and its gradient;
* mm_clip_adam -- clip_grad_norm_ + torch.optim.Adam (PPO.py:74-85), several
  steps, clipping active and inactive, the data-parallel grad_scale;
* FlatAdam's state_dict / load_state_dict in torch.optim.Adam's format.

Tolerances: sums within fp32 summation error of fp64 (1e-6 of sum |x|); the
optimizer within 1e-6 relative of torch's fp32 step (the same operations per
element; only the gradient norm's summation order differs, fp64 here).
"""
import copy

import pytest
import torch
import torch.nn as nn

from marlmaze import update, x3

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("R,N", [(1, 5), (7, 264), (26215, 264), (26215, 64), (13108, 130), (1000, 1), (3000, 6)])
def test_colsum_matches_fp64(R, N):
    """Within fp32 summation error of the fp64 column sums, deterministic, and
    every column written (ragged R over the slabs, N not a multiple of 64)."""
    torch.manual_seed(R + N)
    x = torch.randn(R, N, device="cuda")
    got = x3.colsum(x)
    ref = x.double().sum(0)
    scale = x.double().abs().sum(0)
    assert torch.isfinite(got).all()
    assert ((got.double() - ref).abs() <= 1e-6 * scale + 1e-7).all()
    assert torch.equal(got, x3.colsum(x))  # fixed order: bit-reproducible
    one = x3.colsum(x, slabs=1)
    assert ((one.double() - ref).abs() <= 1e-6 * scale + 1e-7).all()


@pytest.mark.parametrize("M", [1, 255, 3000, 209715])
def test_mse_loss_and_gradient(M):
    g = torch.Generator(device="cuda").manual_seed(M)
    v = torch.randn(M, device="cuda", generator=g)
    r = torch.randn(M, device="cuda", generator=g)
    part, dv = update.mse_loss(v, r)
    out = torch.empty(2, device="cuda")
    pp = torch.zeros(3, device="cuda")
    update.losses_final(pp, part, M, out)
    vv = v.clone().requires_grad_(True)
    ref = nn.MSELoss()(vv, r)
    ref.backward()
    assert abs(out[1].item() - ref.item()) <= 1e-6 * ref.item()
    assert out[0].item() == 0.0
    assert (dv - vv.grad).abs().max().item() <= 1e-7 * vv.grad.abs().max().item()


def _nets(seed):
    torch.manual_seed(seed)
    a = nn.Sequential(nn.Linear(37, 50), nn.ReLU(), nn.Linear(50, 6)).cuda()
    c = nn.Sequential(nn.Linear(13, 9), nn.Linear(9, 1)).cuda()
    return a, c


@pytest.mark.parametrize("max_norm,scale", [(0.5, 1.0), (1e4, 1.0), (0.5, 0.5)])
def test_clip_adam_matches_torch(max_norm, scale):
    """Two networks stepped together by mm_clip_adam == clip_grad_norm_ + Adam
    per network (torch fp32, single-tensor Adam like the reference's CPU one),
    over 4 steps with changing gradients and a decaying lr."""
    a, c = _nets(0)
    ra, rc = copy.deepcopy(a), copy.deepcopy(c)
    flat = update.FlatParams([list(a.parameters()), list(c.parameters())])
    mom = (torch.zeros_like(flat.data), torch.zeros_like(flat.data))
    oa = update.FlatAdam(flat, 0, a.parameters(), lr=1e-3, moments=mom)
    oc = update.FlatAdam(flat, 1, c.parameters(), lr=1e-3, moments=mom)
    ta = torch.optim.Adam(ra.parameters(), lr=1e-3, foreach=False)
    tc = torch.optim.Adam(rc.parameters(), lr=1e-3, foreach=False)
    g = torch.Generator(device="cuda").manual_seed(1)
    norms = torch.empty(2, device="cuda")
    for step in range(4):
        for o in (oa, oc, ta, tc):
            o.param_groups[0]["lr"] *= 0.997
        for p, q in zip(list(a.parameters()) + list(c.parameters()), list(ra.parameters()) + list(rc.parameters())):
            gr = torch.randn(p.shape, device="cuda", generator=g) * (0.3 + step)
            p.grad.copy_(gr)
            q.grad = gr * scale
        update.clip_adam([oa, oc], max_norm, norms=norms, grad_scale=scale)
        na = torch.nn.utils.clip_grad_norm_(ra.parameters(), max_norm)
        nc = torch.nn.utils.clip_grad_norm_(rc.parameters(), max_norm)
        ta.step()
        tc.step()
        assert abs(norms[0].item() - na.item()) <= 1e-6 * na.item()
        assert abs(norms[1].item() - nc.item()) <= 1e-6 * nc.item()
        for p, q in zip(list(a.parameters()) + list(c.parameters()), list(ra.parameters()) + list(rc.parameters())):
            assert (p - q).abs().max().item() <= 1e-6 * q.abs().max().item() + 1e-9, step


def test_flat_adam_state_dict_round_trip():
    """A torch.optim.Adam state (the reference's checkpoint format) loads into
    FlatAdam, and FlatAdam's state_dict is that format again; a further step of
    both agrees."""
    a, _ = _nets(3)
    ra = copy.deepcopy(a).cpu()
    ta = torch.optim.Adam(ra.parameters(), lr=2e-4)
    for _ in range(3):
        ta.zero_grad()
        sum((p * p).sum() for p in ra.parameters()).backward()
        ta.step()
    a.load_state_dict({k: v.cuda() for k, v in ra.state_dict().items()})
    flat = update.FlatParams([list(a.parameters())])
    oa = update.FlatAdam(flat, 0, a.parameters(), lr=1.0)
    oa.load_state_dict(copy.deepcopy(ta.state_dict()))
    assert oa.t == 3 and oa.param_groups[0]["lr"] == 2e-4
    sd = oa.state_dict()
    ref = ta.state_dict()
    assert set(sd["state"]) == set(ref["state"]) and sd["param_groups"][0]["params"] == ref["param_groups"][0]["params"]
    for i, st in ref["state"].items():
        assert float(sd["state"][i]["step"]) == float(st["step"])
        assert torch.equal(sd["state"][i]["exp_avg"].cpu(), st["exp_avg"])
        assert torch.equal(sd["state"][i]["exp_avg_sq"].cpu(), st["exp_avg_sq"])
    # one more step each
    ta.zero_grad()
    sum((p * p).sum() for p in ra.parameters()).backward()
    for p, q in zip(a.parameters(), ra.parameters()):
        p.grad.copy_(q.grad.cuda())
    ta.step()
    update.clip_adam([oa], 0.0)
    for p, q in zip(a.parameters(), ra.parameters()):
        assert (p.cpu() - q).abs().max().item() <= 1e-6 * q.abs().max().item()


# ---- the batched forms (one launch for a backward's packs / reductions): bit-identical to the single ----

def test_colsum_deferred_bit_identical():
    """x3.deferred(): 20 column sums (two mm_colsum_multi launches of <= 16) == mm_colsum each."""
    torch.manual_seed(5)
    shapes = [(1, 5), (7, 264), (26215, 264), (13108, 130), (1000, 1), (3000, 6), (8, 64), (15, 3)] * 2
    shapes += [(209715, 64), (64, 272), (17, 17), (4096, 6)]
    xs = [torch.randn(R, N, device="cuda") for R, N in shapes]
    ref = [x3.colsum(x) for x in xs]
    outs = [torch.full((x.shape[1],), float("nan"), device="cuda") for x in xs]
    with x3.deferred():
        for x, o in zip(xs, outs):
            x3.colsum(x, out=o)
    for r, o in zip(ref, outs):
        assert torch.equal(r, o)


@pytest.mark.parametrize("prec", ["x3", "f16"])
def test_wgrad_deferred_bit_identical(prec):
    """x3.deferred(): weight gradients as partials + one mm_wsum_multi == mm_gemm_wgrad."""
    torch.manual_seed(6)
    shapes = [(3000, 264, 264), (26215, 64, 130), (5, 6, 264), (13108, 1, 64), (4096, 264, 460), (33, 64, 64)]
    cases = []
    for M, N, K in shapes:
        s = 2.0 ** 10 if prec == "f16" else 1.0
        cases.append((torch.randn(M, N, device="cuda") / M, torch.randn(M, K, device="cuda"), s))
    ref = [x3.wgrad(dy, x, prec=prec, dscale=s) for dy, x, s in cases]
    outs = [torch.full((dy.shape[1], x.shape[1]), float("nan"), device="cuda") for dy, x, _ in cases]
    with x3.deferred():
        for (dy, x, s), o in zip(cases, outs):
            x3.wgrad(dy, x, prec=prec, dscale=s, out=o)
        assert all(torch.isnan(o).all() for o in outs)  # not reduced yet
    for r, o in zip(ref, outs):
        assert torch.equal(r, o)


def test_pack_many_equals_pack():
    """pack_many (mm_gemm_tp_pack_multi, 18 packs over two precisions) writes the same TP planes as
    pack, and the pack() calls that follow in the scope return those TPs."""
    torch.manual_seed(7)
    mats = [torch.randn(r, c, device="cuda") for r, c in [(264, 460), (264, 264), (6, 264), (1, 64), (64, 130),
                                                             (64, 64), (272, 272), (3, 5), (300, 33)]]
    specs = [(m, t, p) for m in mats for t in (False, True) for p in ("x3",)]
    specs += [(mats[0], False, "f16"), (mats[4], True, "f16")]
    with x3.cached_packs():
        tps = x3.pack_many(specs)
        for (m, t, p), tp in zip(specs, tps):
            assert x3.pack(m, trans=t, prec=p) is tp
    for (m, t, p), tp in zip(specs, tps):
        ref = x3.pack(m, trans=t, prec=p)
        assert (ref.R, ref.C, ref.prec) == (tp.R, tp.C, tp.prec)
        assert torch.equal(ref.buf, tp.buf)
