"""fp16 activation storage of the f16 networks (mm_gemm_nt_h, mm_gemm_wgrad_h, mm_heads_fwd_h16): every
consumer rounds an activation to fp16 anyway or reads it exactly, so each fp16-storage form must equal the
fp32-storage form on the same (fp16-representable) values BIT FOR BIT -- and the f16 update built on them
stays at test_gpu_f16.py's bars against the fp32 oracle (that file runs with fp16 storage on)."""
import pytest
import torch

from marlmaze import networks, x3

pytestmark = pytest.mark.gpu

M = 40000  # >= the B-resident kernel's row threshold (fp16 A runs there only)


def _h16(M, K, g):
    return torch.relu(torch.randn(M, K, device="cuda", generator=g)).half()


@pytest.mark.parametrize("N,K", [(264, 264), (64, 64), (1, 64)])
def test_gemm_fp16_a_equals_fp32_a(N, K):
    g = torch.Generator(device="cuda").manual_seed(N + K)
    a16 = _h16(M, K, g)
    w = x3.pack(torch.randn(N, K, device="cuda", generator=g) * 0.1, prec="f16")
    b = torch.randn(N, device="cuda", generator=g)
    assert x3.a16_ok(M, N, K)
    relu = N > 1
    # (zeroed: the kernels leave the mask words' padding bits unwritten)
    mb16, mb32 = (x3.mbits(M, "cuda").zero_(), x3.mbits(M, "cuda").zero_()) if relu else (None, None)
    y16 = x3.gemm(a16, w, bias=b, relu=relu, mbits_out=mb16)
    y32 = x3.gemm(a16.float(), w, bias=b, relu=relu, mbits_out=mb32)
    assert torch.equal(y16, y32)
    if relu:
        assert torch.equal(mb16, mb32)


@pytest.mark.parametrize("N,K", [(264, 460), (264, 264), (64, 130), (64, 64)])
def test_gemm_fp16_out_is_rounded_fp32_out(N, K):
    g = torch.Generator(device="cuda").manual_seed(7 * N + K)
    a = torch.randn(M, K, device="cuda", generator=g)
    w = x3.pack(torch.randn(N, K, device="cuda", generator=g) * 0.1, prec="f16")
    b = torch.randn(N, device="cuda", generator=g)
    mb16, mb32 = x3.mbits(M, "cuda").zero_(), x3.mbits(M, "cuda").zero_()  # (padding bits unwritten)
    out16 = torch.empty(M, N, dtype=torch.float16, device="cuda")
    y16 = x3.gemm(a, w, bias=b, relu=True, mbits_out=mb16, out=out16)
    y32 = x3.gemm(a, w, bias=b, relu=True, mbits_out=mb32)
    assert y16.dtype == torch.float16
    assert torch.equal(y16, y32.half())
    assert torch.equal(mb16, mb32)  # the bits come from the fp32 value (> 0), as without fp16 storage


@pytest.mark.parametrize("prec,N,K", [("f16", 264, 264), ("f16", 64, 64), ("f16", 1, 64), ("x3", 6, 264)])
def test_wgrad_fp16_x_equals_fp32_x(prec, N, K):
    g = torch.Generator(device="cuda").manual_seed(3 * N + K)
    dy = torch.randn(M, N, device="cuda", generator=g) / M
    x16 = _h16(M, K, g)
    s = networks._grad_scale(M, prec)
    d16 = x3.wgrad(dy, x16, prec=prec, dscale=s)
    d32 = x3.wgrad(dy, x16.float(), prec=prec, dscale=s)
    assert torch.equal(d16, d32)


def test_heads_fwd_fp16_h_equals_fp32_h():
    g = torch.Generator(device="cuda").manual_seed(11)
    h16 = _h16(M, 264, g)
    w = torch.randn(6, 264, device="cuda", generator=g) * 0.1
    b = torch.randn(6, device="cuda", generator=g)
    assert torch.equal(networks._heads_fwd(h16, w, b), networks._heads_fwd(h16.float(), w, b))


def test_f16_train_forward_stores_fp16_and_matches_fp32_storage(monkeypatch):
    """The actor's f16 train_forward keeps fp16 hidden activations, each equal to the fp32-storage run's
    rounded to fp16 (the next layer's f16 GEMM rounds its input the same way either way); the logits differ
    only through the heads' fp32 FMAs reading the rounded last layer."""
    torch.manual_seed(5)
    actor = networks.Actor(hidden_sizes=(264, 264, 264), gemm_prec="f16").cuda()
    x = torch.randn(M, 65, device="cuda")
    z, saved = actor.train_forward(x)
    hs = saved[2]
    assert all(h.dtype == torch.float16 for h in hs)  # the front-end output h0 included (F16_H0)
    monkeypatch.setattr(networks, "F16_ACT", False)
    z32, saved32 = actor.train_forward(x)
    assert all(h.dtype == torch.float32 for h in saved32[2])
    for h, h32 in zip(hs, saved32[2]):
        assert torch.equal(h, h32.half())
    assert torch.equal(z, z32) or (z - z32).abs().max() <= 2e-3 * z32.abs().max()


# ---- the input gradients stored fp16 pre-scaled: fp16(dY s), read back at scale 1 ----

S = networks._grad_scale(M, "f16")


@pytest.mark.parametrize("N,K,bits", [(264, 264, True), (64, 64, True), (460, 264, False)])
def test_dgrad_fp16_prescaled_equals_fp32(N, K, bits):
    """gemm(fp16(dY s), W^T) at ascale 1, cscale 1/s, stored fp16(. s) == fp16(s * the fp32 path's output),
    with the same ReLU mask and column sums (the MFMA operands are the same fp16 values either way)."""
    g = torch.Generator(device="cuda").manual_seed(5 * N + K)
    dy32 = torch.randn(M, K, device="cuda", generator=g) / M
    dy16 = (dy32 * S).half()
    dy32 = dy16.float() / S  # the fp32 path's dY, exactly the stored one unscaled
    w = x3.pack(torch.randn(K, N, device="cuda", generator=g) * 0.1, trans=True, prec="f16")  # W [K, N]^T
    if bits:
        mb = x3.mbits(M, "cuda").zero_()
        h = torch.randn(M, N, device="cuda", generator=g)
        x3.gemm(torch.randn(M, 64, device="cuda", generator=g), x3.pack(torch.randn(N, 64, device="cuda"),
                                                                      prec="f16"), relu=True, mbits_out=mb)
        cs32, cs16 = x3.colsum_buf(M, N, "cuda"), x3.colsum_buf(M, N, "cuda")
        o32 = x3.gemm(dy32, w, mbits_in=mb, colsum=cs32, ascale=S)
        out = torch.empty(M, N, dtype=torch.float16, device="cuda")
        o16 = x3.gemm(dy16, w, mbits_in=mb, colsum=cs16, ascale=1.0, cscale=1.0 / S, out=out, oscale=S)
        assert torch.equal(o16, (o32 * S).half())
        assert torch.equal(cs16, cs32)
        del h
    else:  # the plain first-layer form: fp32 out
        o32 = x3.gemm(dy32, w, ascale=S)
        o16 = x3.gemm(dy16, w, ascale=1.0, cscale=1.0 / S)
        assert o16.dtype == torch.float32 and torch.equal(o16, o32)


@pytest.mark.parametrize("N,K,x16", [(264, 264, True), (264, 460, False), (64, 64, True), (64, 130, False)])
def test_wgrad_fp16_prescaled_dy_equals_fp32(N, K, x16):
    g = torch.Generator(device="cuda").manual_seed(9 * N + K)
    dy16 = (torch.randn(M, N, device="cuda", generator=g) / M * S).half()
    x = _h16(M, K, g) if x16 else torch.randn(M, K, device="cuda", generator=g)
    d16 = x3.wgrad(dy16, x, prec="f16", dscale=1.0, cscale=1.0 / S)
    d32 = x3.wgrad(dy16.float() / S, x, prec="f16", dscale=S)
    assert torch.equal(d16, d32)


def test_heads_bwd_fp16_prescaled():
    g = torch.Generator(device="cuda").manual_seed(13)
    dz = torch.randn(M, 6, device="cuda", generator=g) / M
    w = torch.randn(6, 264, device="cuda", generator=g) * 0.1
    mb = x3.mbits(M, "cuda").zero_()
    x3.gemm(torch.randn(M, 64, device="cuda", generator=g), x3.pack(torch.randn(264, 64, device="cuda"), prec="f16"),
            relu=True, mbits_out=mb)
    dy32, cs32 = x3.heads_bwd(dz, w, mb)
    dy16, cs16 = x3.heads_bwd(dz, w, mb, oscale=S)
    assert dy16.dtype == torch.float16 and torch.equal(dy16, (dy32 * S).half()) and torch.equal(cs16, cs32)


def test_front_fwd_h16_is_rounded_fp32():
    torch.manual_seed(8)
    actor = networks.Actor(hidden_sizes=(264, 264, 264), gemm_prec="f16").cuda()
    x = torch.randn(3001, 65, device="cuda")
    params = networks.front_params(actor.projection, actor.attention)
    _, h32 = networks._front_fwd(x, True, params)
    _, h16 = networks._front_fwd(x, True, params, h16=True)
    assert h16.dtype == torch.float16 and torch.equal(h16, h32.half())


@pytest.mark.parametrize("M", [M, 3001])
def test_gemm_fp16_a_k460_streaming_equals_fp32_a(M):
    """The first trunk layer at K = 460 with fp16 A (the streaming kernel's ASrcF16V; the B-resident kernel
    does not take that width): equal to the fp32-A form on the same fp16 values, fp16 and fp32 outputs."""
    g = torch.Generator(device="cuda").manual_seed(M)
    a16 = torch.randn(M, 460, device="cuda", generator=g).half()
    w = x3.pack(torch.randn(264, 460, device="cuda", generator=g) * 0.05, prec="f16")
    b = torch.randn(264, device="cuda", generator=g)
    mb16, mb32 = x3.mbits(M, "cuda").zero_(), x3.mbits(M, "cuda").zero_()
    out16 = torch.empty(M, 264, dtype=torch.float16, device="cuda")
    y16 = x3.gemm(a16, w, bias=b, relu=True, mbits_out=mb16, out=out16)
    y32 = x3.gemm(a16.float(), w, bias=b, relu=True, mbits_out=mb32)
    assert torch.equal(y16, y32.half()) and torch.equal(mb16, mb32)
    assert torch.equal(x3.gemm(a16, w, bias=b, relu=True), y32)
