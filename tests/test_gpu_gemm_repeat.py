"""Repeat-launch determinism of the update's weight-gradient and GEMM kernels ("The
k_wgrad_rect zeros"): every kernel here is deterministic, so every launch on the same inputs must equal the
first launch bit for bit.  The round-4 failure (one staging load of a wave's last quarter returning zeros)
made 1 in 30 to 65% of the launches of k_wgrad_rect differ; these cases run each update shape 30 times
(tools/diag_gemm_repeat.py runs the long form: 100 launches x 30 cases at 419,430 rows)."""
import pytest
import torch

from marlmaze import networks, x3

pytestmark = pytest.mark.gpu

M = 70001  # > the B-resident threshold, several row slices per workgroup, a partial last step
REPS = 30


@pytest.mark.parametrize("prec", ["x2", "f16", "x3"])
@pytest.mark.parametrize("N,K", [(6, 264), (264, 264), (264, 460), (64, 64), (64, 130), (1, 64)])
def test_wgrad_repeat_launches_identical(prec, N, K):
    g = torch.Generator(device="cuda").manual_seed(3 * N + K)
    dy = torch.randn(M, N, device="cuda", generator=g) / M
    x = torch.randn(M, K, device="cuda", generator=g)
    s = networks._grad_scale(M, prec)
    d0 = x3.wgrad(dy, x, prec=prec, dscale=s)
    d = torch.empty_like(d0)
    bad = 0
    for _ in range(REPS):
        x3.wgrad(dy, x, prec=prec, dscale=s, out=d)
        bad += int(not torch.equal(d.view(torch.int32), d0.view(torch.int32)))
    assert bad == 0, f"{bad} of {REPS} launches differ"


@pytest.mark.parametrize("prec", ["x2", "f16"])
@pytest.mark.parametrize("N,K", [(264, 460), (264, 264), (460, 264)])
def test_gemm_repeat_launches_identical(prec, N, K):
    g = torch.Generator(device="cuda").manual_seed(N + K)
    a = torch.randn(M, K, device="cuda", generator=g)
    wp = x3.pack(torch.randn(N, K, device="cuda", generator=g) * 0.1, prec=prec)
    b = torch.randn(N, device="cuda", generator=g)
    y0 = x3.gemm(a, wp, bias=b, relu=True)
    y = torch.empty_like(y0)
    bad = 0
    for _ in range(REPS):
        x3.gemm(a, wp, bias=b, relu=True, out=y)
        bad += int(not torch.equal(y.view(torch.int32), y0.view(torch.int32)))
    assert bad == 0, f"{bad} of {REPS} launches differ"


@pytest.mark.parametrize("N,K", [(6, 264), (264, 264), (264, 460), (64, 64)])
@pytest.mark.parametrize("xb", [True, False])
def test_wgrad_fp16_operands_repeat_launches_identical(N, K, xb):
    """The f16 update's weight-gradient forms: fp16 dY stored pre-scaled (fp16(dY s), read at scale 1, the
    result multiplied by 1 / s) with fp16 X (the stored activations, XB = 2) or fp32 X."""
    g = torch.Generator(device="cuda").manual_seed(5 * N + K + xb)
    s = networks._grad_scale(M, "f16")
    dy16 = (torch.randn(M, N, device="cuda", generator=g) / M * s).half()
    x = torch.relu(torch.randn(M, K, device="cuda", generator=g))
    x = x.half() if xb else x
    d0 = x3.wgrad(dy16, x, prec="f16", dscale=1.0, cscale=1.0 / s)
    d = torch.empty_like(d0)
    bad = 0
    for _ in range(REPS):
        x3.wgrad(dy16, x, prec="f16", dscale=1.0, cscale=1.0 / s, out=d)
        bad += int(not torch.equal(d.view(torch.int32), d0.view(torch.int32)))
    assert bad == 0, f"{bad} of {REPS} launches differ"


@pytest.mark.parametrize("N,K,a16,c16", [(264, 264, True, True), (264, 460, True, False), (264, 264, False, True)])
def test_gemm_fp16_operands_repeat_launches_identical(N, K, a16, c16):
    """The f16 update's forward GEMMs with fp16 activations: fp16 A (the B-resident kernel's 16-byte fp16
    vector; at K = 460 the streaming kernel's fp16 A source) and / or fp16 output (EM_FWD16)."""
    g = torch.Generator(device="cuda").manual_seed(7 * N + K)
    a = torch.relu(torch.randn(M, K, device="cuda", generator=g))
    a = a.half() if a16 else a
    wp = x3.pack(torch.randn(N, K, device="cuda", generator=g) * 0.1, prec="f16")
    b = torch.randn(N, device="cuda", generator=g)
    bits = x3.mbits(M, "cuda")
    odt = torch.float16 if c16 else torch.float32
    y0 = x3.gemm(a, wp, bias=b, relu=True, mbits_out=bits, out=torch.empty((M, N), dtype=odt, device="cuda"))
    b0 = bits.clone()
    y = torch.empty_like(y0)
    bad = 0
    for _ in range(REPS):
        x3.gemm(a, wp, bias=b, relu=True, mbits_out=bits, out=y)
        bad += int(not (torch.equal(y, y0) and torch.equal(bits, b0)))
    assert bad == 0, f"{bad} of {REPS} launches differ"


def test_gemm_fp16_input_gradient_repeat_launches_identical():
    """The f16 update's input-gradient GEMM: fp16 pre-scaled dY in, the ReLU bits of the layer below and the
    per-tile column sums applied, fp16 pre-scaled dX out (EM_BWD16)."""
    g = torch.Generator(device="cuda").manual_seed(17)
    N, K = 264, 264
    s = networks._grad_scale(M, "f16")
    h = torch.relu(torch.randn(M, K, device="cuda", generator=g))
    wf = x3.pack(torch.randn(K, 460, device="cuda", generator=g) * 0.05, prec="f16")
    bits = x3.mbits(M, "cuda")
    x3.gemm(torch.randn(M, 460, device="cuda", generator=g), wf, relu=True, mbits_out=bits)
    wt = x3.pack(torch.randn(N, K, device="cuda", generator=g) * 0.1, trans=True, prec="f16")
    dy16 = (torch.randn(M, N, device="cuda", generator=g) / M * s).half()

    def run(out, cs):
        return x3.gemm(dy16, wt, mbits_in=bits, colsum=cs, ascale=1.0, cscale=1.0 / s, out=out, oscale=s)

    cs0 = x3.colsum_buf(M, K, "cuda")
    y0 = run(torch.empty((M, K), dtype=torch.float16, device="cuda"), cs0)
    y, cs = torch.empty_like(y0), torch.empty_like(cs0)
    bad = 0
    for _ in range(REPS):
        run(y, cs)
        bad += int(not (torch.equal(y, y0) and torch.equal(cs, cs0)))
    assert bad == 0, f"{bad} of {REPS} launches differ"
    del h


@pytest.mark.parametrize("prec", ["x2", "f16"])
def test_trunk3_head_sample_repeat_launches_identical(prec):
    """The rollout's fused actor step (mm_trunk3_head_sample: x2 at prefetch depth 1, f16 at depth 3):
    actions, log-probs, joint log-probs, logits and h3 of every launch equal the first's."""
    g = torch.Generator(device="cuda").manual_seed(1)
    packs = [x3.pack(torch.randn(264, k, device="cuda", generator=g) * 0.05, prec=prec) for k in (460, 264, 264)]
    bs = [torch.randn(264, device="cuda", generator=g) * 0.1 for _ in range(3)]
    hw, hb = torch.randn(6, 264, device="cuda", generator=g) * 0.2, torch.randn(6, device="cuda", generator=g) * 0.1
    M = 8192
    h0 = torch.relu(torch.randn(M, 460, device="cuda", generator=g))
    mk = (torch.rand(M, 6, device="cuda", generator=g) < 0.6).to(torch.uint8)
    mk[:, 4] = 1

    def run():
        o = dict(act=torch.empty((M, 2), dtype=torch.int8, device="cuda"), lp=torch.empty(M, device="cuda"),
                 jl=torch.empty(M // 2, device="cuda"), lg=torch.empty(M, 6, device="cuda"),
                 h3=torch.empty(M, 264, device="cuda"))
        x3.trunk3_head_sample(h0, packs, bs, hw, hb, mk, 4321, 9, o["act"], o["lp"], o["jl"], logits=o["lg"],
                              h3=o["h3"])
        return o

    o0 = run()
    bad = 0
    for _ in range(REPS):
        o = run()
        bad += int(not all(torch.equal(o[k], o0[k]) for k in o0))
    assert bad == 0, f"{bad} of {REPS} launches differ"
