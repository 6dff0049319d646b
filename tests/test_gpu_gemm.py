"""The precision-generic actor/critic GEMMs of csrc/x3mlp.hip against fp64.

* mm_gemm_wgrad -- the weight gradient dW = dY^T X of every nn.Linear in the
  update (networks.py:35-41, 87-106 under autograd), both precisions, every
  shape the actor and critic use (incl. the column-blocked 264 x 460 and the
  8-byte-row critic input [M, 130]).
* mm_gemm_nt in fp16 (configs[4]) and on 8-byte rows (the critic's [M, 130]
  observations), forward (bias + ReLU + bits) and input-gradient forms.

Tolerances, relative to sum |a b| per output element (the bound any
reordering of an fp32 sum obeys at ~n eps):
  x3 (bf16x3, fp32-class): 1e-6 (measured 2-4e-7; the fp32 library GEMMs 3e-7);
  x2 (fp16 hi + 2^-11 lo pairs, fp32-class): 1e-6 (operands to 2^-22 relative; the sum in fp32);
  f16 (one fp16 product, operands rounded to 11 bits): 2e-3 (two roundings of
  2^-12 each, plus the fp32 sum).
"""
import pytest
import torch

from marlmaze import x3

pytestmark = pytest.mark.gpu

TOL = {"x3": 1e-6, "x2": 1e-6, "f16": 2e-3}


def _rel_err(got, ref, scale):
    return ((got.double() - ref).abs() / scale.clamp_min(1e-30)).max().item()


@pytest.mark.parametrize("prec", ["x3", "x2", "f16"])
@pytest.mark.parametrize("M,N,K", [(419430, 264, 264), (70001, 264, 460), (40000, 6, 264), (209715, 64, 130),
                                   (30000, 64, 64), (30000, 1, 64), (100, 264, 264), (1, 6, 264), (37, 5, 9),
                                   (1, 264, 460), (300, 264, 264), (6000, 264, 460), (8192, 264, 264),
                                   (4096, 64, 130), (3000, 1, 64)])
def test_wgrad_matches_fp64(prec, M, N, K):
    g = torch.Generator(device="cuda").manual_seed(M + N + K)
    dy = torch.randn(M, N, device="cuda", generator=g)
    x = torch.randn(M, K, device="cuda", generator=g)
    dscale = 1.0
    if prec != "x3":  # gradients of a mean over M rows are ~1/M: scaled into the fp16 normal range
        dy *= 1.0 / M
        dscale = float(2.0 ** int(torch.tensor(float(M)).log2().floor()))
    dw = x3.wgrad(dy, x, prec=prec, dscale=dscale)
    ref = dy.double().t().mm(x.double())
    scale = dy.double().abs().t().mm(x.double().abs())
    err = _rel_err(dw, ref, scale)
    assert dw.shape == (N, K) and err < TOL[prec], err
    # deterministic: a fixed summation order
    assert torch.equal(dw, x3.wgrad(dy, x, prec=prec, dscale=dscale))


def test_wgrad_strided_and_empty():
    """Row strides > width (a column slice of a wider buffer); M = 0 -> zeros."""
    g = torch.Generator(device="cuda").manual_seed(5)
    big = torch.randn(5000, 300, device="cuda", generator=g)
    dy, x = big[:, :64], big[:, 100:230]
    dw = x3.wgrad(dy, x)
    ref = dy.double().t().mm(x.double())
    assert _rel_err(dw, ref, dy.double().abs().t().mm(x.double().abs())) < 1e-6
    z = x3.wgrad(torch.empty(0, 6, device="cuda"), torch.empty(0, 264, device="cuda"))
    assert torch.equal(z, torch.zeros(6, 264, device="cuda"))


@pytest.fixture(params=["auto", "stream"])
def algo(request):
    """Both forward kernels: "auto" = B resident in LDS (k_bres) where the shape fits, "stream" = k_x3nt."""
    prev = x3.set_algo(request.param)
    yield request.param
    x3.set_algo(prev)


@pytest.mark.parametrize("prec", ["x3", "x2", "f16"])
@pytest.mark.parametrize("M,N,K", [(40000, 264, 460), (40000, 264, 264), (40000, 6, 264), (40000, 64, 130),
                                   (40000, 1, 64), (777, 64, 64), (40000, 460, 264), (16411, 264, 264),
                                   (20000, 96, 52),
                                   # the reference's own row counts: the single-sample API, main.py's 3,000-sample
                                   # minibatches (6,000 actor rows), a 4,096-maze rollout step (8,192 actor rows)
                                   (1, 264, 460), (2, 264, 264), (300, 264, 264), (300, 6, 264), (6000, 264, 460),
                                   (6000, 460, 264), (8192, 264, 264), (8192, 6, 264), (4096, 64, 130), (3000, 1, 64)])
def test_gemm_forward_and_input_gradient(prec, M, N, K, algo):
    """Forward (bias + ReLU + bit mask) and the input-gradient form (bits of the
    layer below, per-tile column sums) in both precisions, 16- and 8-byte rows,
    both kernels (below 16,384 rows both settings run the streaming kernel, with
    4-tile column blocks where the row blocks alone would not fill the chip);
    ragged M (16,411: a partial last row tile and 32-row unit), K
    with a 16-wide final step (264, 460, 130) or a partial 32-wide one (52); N = 460: no
    bit masks (N <= 272), the plain input-gradient form."""
    g = torch.Generator(device="cuda").manual_seed(M + N + K)
    a = torch.randn(M, K, device="cuda", generator=g)
    w = torch.randn(N, K, device="cuda", generator=g) * 0.1
    b = torch.randn(N, device="cuda", generator=g)
    bits = x3.mbits(M, "cuda") if N <= 272 else None
    y = x3.gemm(a, x3.pack(w, prec=prec), bias=b, relu=True, mbits_out=bits)
    pre = a.double() @ w.double().t() + b.double()
    scale = a.double().abs() @ w.double().abs().t() + b.double().abs()
    assert _rel_err(y, pre.clamp_min(0), scale) < TOL[prec]
    # the bits record y > 0 exactly
    w2 = torch.randn(48, N, device="cuda", generator=g) * 0.1  # the next layer's weight [out, in]
    dy = torch.randn(M, 48, device="cuda", generator=g) / M
    # the product's fp16 dY scale (networks._grad_scale): 2^floor(log2 M) for gradients of a mean over M rows
    ascale = 1.0 if prec == "x3" else float(2.0 ** int(torch.tensor(float(M)).log2().floor()))
    if bits is None:  # the plain input-gradient form (the first layer's dx)
        dx = x3.gemm(dy, x3.pack(w2, trans=True, prec=prec), ascale=ascale)
        ref = dy.double() @ w2.double()
        assert _rel_err(dx, ref, dy.double().abs() @ w2.double().abs()) < TOL[prec]
        return
    cs = x3.colsum_buf(M, N, "cuda")
    dx = x3.gemm(dy, x3.pack(w2, trans=True, prec=prec), mbits_in=bits, colsum=cs, ascale=ascale)
    ref = (dy.double() @ w2.double()) * (y > 0)
    sc = dy.double().abs() @ w2.double().abs()
    assert _rel_err(dx, ref, sc) < TOL[prec]
    assert torch.equal(dx == 0, (y <= 0) | (dx == 0))
    ref_cs = dx.double().sum(0)
    assert ((cs.double().sum(0) - ref_cs).abs() <= 1e-5 * dx.double().abs().sum(0) + 1e-30).all()


def test_gemm_rejects_bad_shapes():
    from marlmaze import _lib

    a = torch.randn(100, 130, device="cuda")
    with pytest.raises(_lib.MMError):  # 8-byte rows: only narrow outputs
        x3.gemm(a, x3.pack(torch.randn(264, 130, device="cuda")))
    with pytest.raises(_lib.MMError):  # x3 operands are exact splits: no scaling
        x3.gemm(torch.randn(100, 64, device="cuda"), x3.pack(torch.randn(8, 64, device="cuda")), ascale=2.0)


@pytest.mark.parametrize("M,N,K", [(40000, 264, 264), (40000, 264, 460), (3000, 264, 264)])
def test_x2_dynamic_range(M, N, K, algo):
    """x2 keeps 22 significand bits for 2^-14 <= |x s| <= 2^15 (the 2^11-scaled lo part stays out of the fp16
    subnormals): operands spread over 2^-12 .. 2^12 per element, forward and scaled input-gradient forms and the
    weight gradient, at the fp32-class bar."""
    g = torch.Generator(device="cuda").manual_seed(M + K)
    spread = lambda *shape: torch.randn(*shape, device="cuda", generator=g) * torch.exp2(  # noqa: E731
        torch.randint(-12, 13, shape, device="cuda", generator=g).float())
    a = spread(M, K)
    w = spread(N, K) * 2.0**-6
    y = x3.gemm(a, x3.pack(w, prec="x2"))
    ref = a.double() @ w.double().t()
    assert _rel_err(y, ref, a.double().abs() @ w.double().abs().t()) < TOL["x2"]
    dy = spread(M, N) / M
    s = float(2.0 ** int(torch.tensor(float(M)).log2().floor()))
    dx = x3.gemm(dy, x3.pack(w, trans=True, prec="x2"), ascale=s)
    assert _rel_err(dx, dy.double() @ w.double(), dy.double().abs() @ w.double().abs()) < TOL["x2"]
    dw = x3.wgrad(dy, a, prec="x2", dscale=s)
    assert _rel_err(dw, dy.double().t() @ a.double(), dy.double().abs().t() @ a.double().abs()) < TOL["x2"]


@pytest.mark.parametrize("algo", ["auto", "stream"], indirect=True)
def test_gemm_row_chunks(algo):
    """A call whose A exceeds 2^31 bytes (the kernels address A and C through buffer resources) runs in
    row chunks: 1,200,000 x 460 fp32 (2.2 GB), forward with bits and the input-gradient form, checked on
    rows either side of the chunk boundary and at the end."""
    M, N, K = 1_200_000, 264, 460
    g = torch.Generator(device="cuda").manual_seed(11)
    a = torch.randn(M, K, device="cuda", generator=g)
    w = torch.randn(N, K, device="cuda", generator=g) * 0.05
    b = torch.randn(N, device="cuda", generator=g)
    bits = x3.mbits(M, "cuda")
    y = x3.gemm(a, x3.pack(w), bias=b, relu=True, mbits_out=bits)
    cap = ((2**31 - 1) // (4 * K) - 32) // 256 * 256
    rows = torch.cat([torch.arange(0, 64), torch.arange(cap - 64, cap + 64), torch.arange(M - 64, M)]).cuda()
    pre = a[rows].double() @ w.double().t() + b.double()
    scale = a[rows].double().abs() @ w.double().abs().t() + b.double().abs()
    assert _rel_err(y[rows], pre.clamp_min(0), scale) < TOL["x3"]
    w2 = torch.randn(48, N, device="cuda", generator=g) * 0.1
    dy = torch.randn(M, 48, device="cuda", generator=g)
    cs = x3.colsum_buf(M, N, "cuda")
    dx = x3.gemm(dy, x3.pack(w2, trans=True), mbits_in=bits, colsum=cs)
    ref = (dy[rows].double() @ w2.double()) * (y[rows] > 0)
    assert _rel_err(dx[rows], ref, dy[rows].double().abs() @ w2.double().abs()) < TOL["x3"]
    assert torch.allclose(cs.double().sum(0), dx.double().sum(0), rtol=1e-5, atol=1e-3)


@pytest.mark.parametrize("M,N,K", [(40000, 264, 264), (40000, 264, 460), (3000, 64, 130)])
def test_x2_range_guard(M, N, K):
    """Operands beyond fp16's range (|x s| >= 2^16: hi would round to inf, the product to inf / NaN where
    fp32 stays finite): the x2 kernels raise the library's range flag (mm_gemm_range_flag), and the checked
    forms redo the GEMM at x3 -- forward, scaled input gradient and weight gradient at the fp32-class bar.
    In-range operands never raise it."""
    g = torch.Generator(device="cuda").manual_seed(M + N + K)
    x3.range_flag(clear=True)
    a = torch.randn(M, K, device="cuda", generator=g)
    w = torch.randn(N, K, device="cuda", generator=g) * 0.05
    x3.gemm(a, x3.pack(w, prec="x2"))
    assert int(x3.range_flag().item()) == 0  # in range: no flag
    big = a * 2.0**17  # activations beyond 2^16
    ref = big.double() @ w.double().t()
    scale = big.double().abs() @ w.double().abs().t()
    y = x3.gemm(big, x3.pack(w, prec="x2"))
    assert int(x3.range_flag().item()) == 1 and not torch.isfinite(y).all()  # detected (not silent)
    y = x3.gemm(big, x3.pack(w, prec="x2"), checked=True)
    assert torch.isfinite(y).all() and _rel_err(y, ref, scale) < TOL["x2"]
    # the input-gradient form: dY of a mean over M rows scaled by 2^floor(log2 M), here beyond 2^16 after it
    dy = torch.randn(M, N, device="cuda", generator=g) * 4.0
    s = float(2.0 ** int(torch.tensor(float(M)).log2().floor()))
    dx = x3.gemm(dy, x3.pack(w, trans=True, prec="x2"), ascale=s, checked=True)
    assert _rel_err(dx, dy.double() @ w.double(), dy.double().abs() @ w.double().abs()) < TOL["x2"]
    # the weight gradient: X beyond 2^16, and dY whose scaled values are
    dw = x3.wgrad(dy, big, prec="x2", dscale=s, checked=True)
    refw = dy.double().t() @ big.double()
    assert _rel_err(dw, refw, dy.double().abs().t() @ big.double().abs()) < TOL["x2"]
    assert int(x3.range_flag().item()) == 0  # the checked forms leave the flag clear
    # forms the x3 redo cannot reproduce (fp16 operands / output, an output scale) are refused, not redone wrong
    wf = x3.pack(w, prec="f16")
    with pytest.raises(ValueError):
        x3.gemm(a.half(), wf, checked=True)
    with pytest.raises(ValueError):
        x3.gemm(a, wf, out=torch.empty((M, N), dtype=torch.float16, device="cuda"), checked=True)
    with pytest.raises(ValueError):
        x3.wgrad((dy * s).half(), a, prec="f16", cscale=1.0 / s, checked=True)
    with pytest.raises(ValueError):
        x3.wgrad(dy, a.half(), prec="f16", checked=True)


@pytest.mark.parametrize("M", [419430, 70001, 3296, 33, 1])
@pytest.mark.parametrize("N,K", [(264, 264), (264, 460)])
def test_wgrad_dma_staging_equals_register_staging(M, N, K):
    """The x2 trunk weight gradients on k_wgrad_dma (raw rows staged by LDS-DMA into a two-stage ring) and
    on k_wgrad_rect (staged through registers): the same fragment images and MFMA order, so the same
    partials and sums bit for bit -- at full, ragged (a partial last 32-row step, slices of one step) and
    strided (lddy / ldx > width) operands -- and the fp32-class bar against fp64."""
    g = torch.Generator(device="cuda").manual_seed(M + N + K)
    big = torch.randn(M, N + 8, device="cuda", generator=g) / max(M, 1)
    dy = big[:, 4:4 + N]
    xb = torch.randn(M, K + 12, device="cuda", generator=g)
    x = xb[:, :K]
    s = float(2.0 ** int(torch.tensor(float(M)).log2().floor()))
    prev = x3.set_wgrad_algo("dma")
    try:
        d_dma = x3.wgrad(dy, x, prec="x2", dscale=s)
        x3.set_wgrad_algo("reg")
        d_reg = x3.wgrad(dy, x, prec="x2", dscale=s)
    finally:
        x3.set_wgrad_algo(prev)
    assert torch.equal(d_dma, d_reg)
    ref = dy.double().t() @ x.double()
    assert _rel_err(d_dma, ref, dy.double().abs().t() @ x.double().abs()) < TOL["x2"]
