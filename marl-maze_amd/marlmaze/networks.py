"""Actor / Critic of the reference (networks.py:13-106), laid out for MI355X.

Parameters keep the reference's module tree and ``state_dict`` names (so the
shipped ``PPO.pth`` loads unchanged) and are created in the reference's order,
so ``torch.manual_seed(s)`` gives the same initial weights.  ``forward`` does
not replay the reference's 23 tiny Linear calls: the projection, Q/K/V,
attention and residual run as one fused HIP kernel (csrc/actor_front.hip),
the MLP trunk, the two heads (as ONE [6, K] GEMM) and the critic on the
hand-written MFMA GEMMs of csrc/x3mlp.hip, at every batch size.  The PPO
update calls ``train_forward`` / ``train_backward``: an explicit backward
that writes every gradient straight into the parameters' .grad storage.

Quirk Q1 (networks.py:59-63): the reference never advances the slice index,
so every embedding reads ``x[:, 0:d_i]`` and the actor sees only obs[0:4].
``parity_mode=True`` (default) keeps that; ``parity_mode=False`` gives each
feature its own slice (what the code evidently intended).
"""
import ctypes
import math
import os

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

FEATURE_DIMS = [4, 4, 4, 4, 4, 4, 4, 4, 4, 4, 4, 4, 2, 2, 1, 4, 1, 1, 1, 1, 1, 1, 2]  # networks.py:8
FEATURE_AMOUNT = len(FEATURE_DIMS)
OBS_SPACE = int(np.sum(FEATURE_DIMS))  # 65
EMBEDDING_DIM = 20
KQ_DIM = 10
_SQRT_KQ = float(np.sqrt(KQ_DIM))  # networks.py:79 divides by np.sqrt(10)


class Projection(nn.Module):
    """networks.py:51-65 -- 23 Linear(d_i -> 20); forward packs them into one GEMM."""

    def __init__(self, parity_mode=True):
        super().__init__()
        self.layers = nn.ModuleList([nn.Linear(d, EMBEDDING_DIM) for d in FEATURE_DIMS])
        self.parity_mode = parity_mode
        starts = np.zeros(FEATURE_AMOUNT, np.int64) if parity_mode else np.cumsum([0] + FEATURE_DIMS[:-1])
        self.register_buffer("_starts", torch.as_tensor(starts), persistent=False)
        self.in_width = 4 if parity_mode else OBS_SPACE

    def packed(self):
        """W [460, in_width] (zero outside each feature's slice), b [460]."""
        rows = []
        for lin, d, s in zip(self.layers, FEATURE_DIMS, self._starts.tolist()):
            w = lin.weight
            left = s
            right = self.in_width - s - d
            rows.append(F.pad(w, (left, right)))
        return torch.cat(rows, 0), torch.cat([lin.bias for lin in self.layers], 0)

    def forward(self, x, packed=None):
        W, b = packed if packed is not None else self.packed()
        return F.linear(x[:, :self.in_width], W, b)  # [B, 460] = 23 embeddings of 20


class m_Attention(nn.Module):
    """networks.py:67-82 -- one self-attention layer over the 23 feature tokens."""

    def __init__(self, kq_dim=KQ_DIM):
        super().__init__()
        self.kq_dim = kq_dim
        self.keys = nn.Linear(EMBEDDING_DIM, kq_dim, bias=False)
        self.querys = nn.Linear(EMBEDDING_DIM, kq_dim, bias=False)
        self.values = nn.Linear(EMBEDDING_DIM, EMBEDDING_DIM, bias=False)

    def forward(self, h):
        B = h.shape[0]
        t = h.view(B, FEATURE_AMOUNT, EMBEDDING_DIM)
        wqkv = torch.cat([self.querys.weight, self.keys.weight, self.values.weight], 0)  # [40, 20]
        qkv = F.linear(t, wqkv)  # [B, 23, 40]
        q, k, v = qkv.split([self.kq_dim, self.kq_dim, EMBEDDING_DIM], dim=-1)
        logits = torch.bmm(q, k.transpose(1, 2)) / _SQRT_KQ  # [B, 23, 23]
        w = torch.softmax(logits, dim=-1)
        ctx = torch.bmm(w, v)
        return (t + ctx).reshape(B, FEATURE_AMOUNT * EMBEDDING_DIM)


_CUS = {}
# the front-end backward's attention products: "mfma" (fp32 MFMA tiles, csrc/actor_front.hip
# k_front_bwd_mfma; the default) or "valu" (fp32 FMA, one lane per token, k_front_bwd)
FRONT_BWD_ALGO = os.environ.get("MARLMAZE_FRONT_BWD", "mfma")


def _front_bwd_grid(B, dev):
    """Persistent grid of the front-end backward (mm_actor_front_bwd_grid: 8-sample workgroups, three per CU
    for the MFMA kernel, two for the VALU kernel)."""
    from . import _lib

    with torch.cuda.device(dev):
        grid = _lib.lib().mm_actor_front_bwd_grid(int(B), _lib.FRONT_BWD[FRONT_BWD_ALGO])
    if grid < 1:
        raise _lib.MMError(f"mm_actor_front_bwd_grid failed with status {grid}")
    return grid
# the front-end forward: "mfma" (default: both attention products on the fp32 MFMA, k_front_fwd_mfma; 13% faster
# than row1 at 419,430 rows, 4-9% at the rollout's sizes), "row1" (VALU, one query row per lane; 8 samples, three
# workgroups per CU) or "row2" (two query rows per lane, half the K/V LDS reads; 16 samples per workgroup, two
# workgroups per CU); row1 and row2 are bit-identical, mfma within fp32 rounding of them (csrc/actor_front.hip).
# "auto": row2 up to FRONT_FWD_ROW2_MAX samples (one round of its grid where row1 needs two), row1 above
FRONT_FWD_ALGO = os.environ.get("MARLMAZE_FRONT_FWD", "mfma")
FRONT_FWD_ROW2_MAX = int(os.environ.get("MARLMAZE_FRONT_FWD_ROW2_MAX", "8192"))


def _cu_count(dev):
    if dev not in _CUS:
        _CUS[dev] = torch.cuda.get_device_properties(dev).multi_processor_count
    return _CUS[dev]


class _FusedFront(torch.autograd.Function):
    """Projection + attention + residual as HIP kernels (csrc/actor_front.hip).

    apply(x [B, 65], parity, *params) with params = the 23 projection weights,
    the 23 projection biases, querys, keys, values weights (module order).  A
    tiny prep kernel folds the parameters into a workspace every call; the
    backward kernel reduces the weight gradients inside a persistent grid and
    two small kernels finish them (no per-parameter copies or pads).
    """

    @staticmethod
    def forward(ctx, x, parity, *params):
        x = x.contiguous()
        ws, h = _front_fwd(x, parity, params)
        ctx.save_for_backward(x, ws)
        ctx.parity = parity
        return h

    @staticmethod
    def backward(ctx, dh):
        from . import _lib

        x, ws = ctx.saved_tensors
        B = x.shape[0]
        dh = dh.contiguous()
        L = _lib.lib()
        grid = _front_bwd_grid(B, x.device)
        plen = L.mm_actor_front_partial_len()
        partial = torch.empty((grid, plen), dtype=torch.float32, device=x.device)
        red = torch.empty(plen, dtype=torch.float64, device=x.device)  # the fp64 sums
        g = torch.empty(L.mm_actor_front_grad_len(), dtype=torch.float32, device=x.device)
        _lib.check(L.mm_actor_front_bwd_ex(_lib.ptr(ws), _lib.ptr(x), OBS_SPACE, B, int(ctx.parity), _lib.ptr(dh),
                                           _lib.ptr(partial), grid, _lib.ptr(red), _lib.ptr(g),
                                           _lib.FRONT_BWD[FRONT_BWD_ALGO], _lib.stream_ptr()), "mm_actor_front_bwd_ex")
        n_qk, n_v = KQ_DIM * EMBEDDING_DIM, EMBEDDING_DIM * EMBEDDING_DIM
        dwq = g[0:n_qk].view(KQ_DIM, EMBEDDING_DIM)
        dwk = g[n_qk:2 * n_qk].view(KQ_DIM, EMBEDDING_DIM)
        dwv = g[2 * n_qk:2 * n_qk + n_v].view(EMBEDDING_DIM, EMBEDDING_DIM)
        o = 2 * n_qk + n_v
        n_p = FEATURE_AMOUNT * EMBEDDING_DIM * 4
        dwp = g[o:o + n_p].view(FEATURE_AMOUNT, EMBEDDING_DIM, 4)
        dbp = g[o + n_p:].view(FEATURE_AMOUNT, EMBEDDING_DIM)
        return (None, None, *(dwp[i, :, :d] for i, d in enumerate(FEATURE_DIMS)),
                *(dbp[i] for i in range(FEATURE_AMOUNT)), dwq, dwk, dwv)


def front_params(projection, attention):
    """Parameter order of _FusedFront.apply."""
    return ([lin.weight for lin in projection.layers] + [lin.bias for lin in projection.layers] +
            [attention.querys.weight, attention.keys.weight, attention.values.weight])


# The actor MLP (the 460 -> 264 -> 264 -> 264 ReLU trunk + the two heads,
# networks.py:35-41) and the critic (130 -> 64 -> 64 -> 1, networks.py:87-102)
# run on the hand-written GEMMs of csrc/x3mlp.hip at every row count, forward
# and backward:
# * precision "x3": fp32-class -- each operand split exactly into three bf16
#   parts, six bf16 MFMA products kept; "x2": fp32-class on two fp16 parts per
#   operand (x = hi + 2^-11 lo, 22 significand bits), three f16 MFMA products;
#   "f16": one fp16 MFMA product per element (BASELINE configs[4]).  Storage,
#   master weights and Adam stay fp32 in all three.  The actor heads always run at x3: the rollout's fused
#   head + sampler kernel computes them in fp32, and the update's log-probs
#   must be those of the same logits.
# * weights are packed per call into fragment-order planes (tiny); the
#   activations stay fp32 row-major and are converted inside the GEMMs;
# * the forward GEMMs record their ReLU masks as bits; the input-gradient GEMMs
#   apply them in their epilogue (no threshold_backward pass) and emit the
#   per-tile column sums of the next layer's bias gradient (summed by mm_colsum);
# * weight gradients dW = dY^T X run on mm_gemm_wgrad (row-slice partials
#   summed in a fixed order).
# The fp16 / x2 backward GEMMs scale dY by 2^floor(log2 M): the losses are means
# over M rows, so per-row gradients are ~1/M, and the scale keeps them in
# fp16's normal range; the results are unscaled (powers of two: exact).
# Shapes the engine does not take (a non-ReLU activation, layers wider than
# 272, inputs not a multiple of 4 wide) -- none of which the reference builds --
# run as plain torch ops, with a warning on the GPU.
GEMM_PRECISIONS = ("x3", "x2", "f16")
# the fp32-class arithmetic of the product (x2: half the MFMAs of x3 at the same 1e-6 GEMM bar, 0.76x the time
# of x3 over the update's shapes, tools/bench_prec.py); MARLMAZE_FP32_GEMM=x3 selects the other for A/B runs
FP32_GEMM = os.environ.get("MARLMAZE_FP32_GEMM", "x2")
if FP32_GEMM not in ("x2", "x3"):
    raise ValueError(f"MARLMAZE_FP32_GEMM must be 'x2' or 'x3', not {FP32_GEMM!r}")
_MAX_WIDTH = 272
_WARNED = set()


def _engine_ok(x, widths):
    return x.is_cuda and x.dim() == 2 and x.stride(1) == 1 and all(n <= _MAX_WIDTH for n in widths)


def _warn_torch_path(what):
    if what not in _WARNED:
        _WARNED.add(what)
        import warnings

        warnings.warn(f"marlmaze: {what} is outside the hand-written GEMM engine's shapes; it runs as plain "
                      "torch ops", RuntimeWarning, stacklevel=3)


def _grad_scale(M, prec):
    """The power-of-two dY scale of the fp16-operand backward GEMMs, f16 and x2 (1 for x3)."""
    return float(2.0 ** int(math.floor(math.log2(max(int(M), 1))))) if prec in ("f16", "x2") else 1.0


def _wgrad(dy, x, prec, out=None):
    """dW = dY^T X (mm_gemm_wgrad).  An fp16 dY is the f16 networks' pre-scaled input gradient."""
    from . import x3

    s = _grad_scale(dy.shape[0], prec)
    if dy.dtype == torch.float16:
        return x3.wgrad(dy.contiguous(), x, prec=prec, dscale=1.0, cscale=1.0 / s, out=out)
    return x3.wgrad(dy.contiguous(), x, prec=prec, dscale=s, out=out)


# f16 networks: the update's hidden activations are stored in fp16 (mm_gemm_nt_h) -- every consumer rounds
# them to fp16 anyway (the next GEMM's operand, the weight gradients' X) or reads them exactly (the heads'
# fp32 FMAs over fp16 values), so the arithmetic is that of fp32 storage at half the bytes.
# MARLMAZE_F16_ACT=0 keeps them fp32 (A/B runs).
F16_ACT = os.environ.get("MARLMAZE_F16_ACT", "1") != "0"
# ... and the front-end output h0 with them (MARLMAZE_F16_H0=0: fp32 h0)
F16_H0 = os.environ.get("MARLMAZE_F16_H0", "1") != "0"


def _act16(prec, M, widths, next_ks):
    """fp16 storage of the hidden layers' outputs: f16, and every GEMM reading one takes fp16 A at that
    shape (next_ks: (N, K) of those GEMMs)."""
    from . import x3

    return (F16_ACT and prec == "f16" and all(n % 4 == 0 for n in widths)
            and all(x3.a16_ok(M, n, k) for n, k in next_ks))


# three ReLU layers without bits (the rollout's trunk) up to this many rows run as ONE launch (mm_trunk3:
# bit-identical to the per-layer GEMMs below 16,384 rows, where those sit at their launch floor).  Per
# precision, from tools/bench_trunk.py (profiles/r05_bench_trunk_*.jsonl; fused vs three GEMMs, HIP graphs):
# x2 8,192 rows 21.8 vs 42.0 us, 49,152 124 vs 133 us; with the heads + draws (the rollout's form) x2 8,192
# 25.8 vs 49.1 us but 65,536 196 vs 177 us; f16 65,536 81 vs 123 us, 131,072 162 vs 259 us.
# MARLMAZE_TRUNK_MAX_ROWS overrides it for every precision (0: off).
_TRUNK_MAX_ROWS_DEFAULT = {"x2": 32768, "x3": 16384, "f16": 131072}
TRUNK_MAX_ROWS = int(os.environ["MARLMAZE_TRUNK_MAX_ROWS"]) if "MARLMAZE_TRUNK_MAX_ROWS" in os.environ else None


def _trunk_max_rows(prec):
    return TRUNK_MAX_ROWS if TRUNK_MAX_ROWS is not None else _TRUNK_MAX_ROWS_DEFAULT.get(prec, 0)


def _mlp_fwd(h0, ws, bs, prec, need_bits, act16=False):
    """The ReLU layers on the engine; returns the activations [h0, h1, ...] and
    the forward GEMMs' ReLU bit masks (None without need_bits).  act16: the
    layers' outputs in fp16 (f16 with bits only, see F16_ACT).  Three layers
    without bits at <= _trunk_max_rows(prec) rows: one fused launch, and only h0
    and the last layer's output are returned ([h0, None, None, h3])."""
    from . import x3

    M, dev = h0.shape[0], h0.device
    if not need_bits and not act16 and len(ws) == 3 and 0 < M <= _trunk_max_rows(prec) and h0.dtype == torch.float32:
        packs = [x3.pack(w, prec=prec) for w in ws]
        if x3.trunk3_ok(M, h0, packs, prec):
            return [h0, None, None, x3.trunk3(h0, packs, bs)], [None, None, None]
    hs, bits = [h0], []
    h = h0
    for w, b in zip(ws, bs):
        mb = x3.mbits(M, dev) if need_bits else None
        out = torch.empty((M, w.shape[0]), dtype=torch.float16, device=dev) if act16 else None
        h = x3.gemm(h, x3.pack(w, prec=prec), bias=b, relu=True, mbits_out=mb, out=out)
        hs.append(h)
        bits.append(mb)
    return hs, bits


# the actor backward's weight gradients on a side stream (MARLMAZE_WGRAD_STREAM=1; default off): a layer's
# weight gradient and its input-gradient GEMM read the same dY and nothing else in common, so the weight
# gradients (and the heads') could run beside the input-gradient chain and the front-end backward.  Measured
# slower (same box, alternating): headline 7.11M -> 6.84-6.98M env-steps/s, configs[1] 5.37M -> 5.01M --
# both sides are grids of one large-LDS workgroup per CU (k_wgrad_dma 156 KB, k_bres 152 KB), so sharing the
# CUs splits each into two rounds instead of overlapping them
# "heads": only the heads' weight gradient (x3, 6 x 264) beside the heads' backward and the trunk
WGRAD_STREAM = os.environ.get("MARLMAZE_WGRAD_STREAM", "0")
WGRAD_STREAM = False if WGRAD_STREAM == "0" else ("heads" if WGRAD_STREAM == "heads" else True)
_WSTREAMS = {}


def wgrad_stream(device):
    """The side stream of the weight gradients (one per device)."""
    st = _WSTREAMS.get(device)
    if st is None:
        st = _WSTREAMS[device] = torch.cuda.Stream(device=device)
    return st


class _OnSide:
    """with _OnSide(side, *tensors): the block's launches go to ``side`` after everything queued so far on the
    current stream, and the tensors (made on the current stream) are not reused by the caching allocator
    before the side stream's work on them is done.  side None: the current stream, nothing else."""

    def __init__(self, side, *tensors):
        self.side, self.tensors = side, tensors

    def __enter__(self):
        if self.side is not None:
            self.side.wait_stream(torch.cuda.current_stream(self.side.device))
            for t in self.tensors:
                t.record_stream(self.side)
            self.ctx = torch.cuda.stream(self.side)
            self.ctx.__enter__()
        return self

    def __exit__(self, *exc):
        if self.side is not None:
            self.ctx.__exit__(*exc)
        return False


def _mlp_bwd(ctx_bits, hs, ws, dy, cs, prec, need_dx, outs=None, wside=None):
    """Backward through the ReLU layers given dY of the last one (already through
    its ReLU) and that dY's per-tile column sums cs (None: sum dY itself).
    outs: destinations [dW0, db0, dW1, db1, ...] (or None: allocated).
    An fp16 dY is the f16 networks' pre-scaled input gradient (fp16(dY s), see
    _g16): the layers' input gradients then stay fp16 pre-scaled too.
    Returns (dx or None, [dW0, db0, dW1, db1, ...])."""
    from . import x3

    L = len(ws)
    M = dy.shape[0]
    s = _grad_scale(M, prec)
    g16 = dy.dtype == torch.float16
    grads = [None] * (2 * L)
    dx = None
    for l in range(L - 1, -1, -1):
        o_w, o_b = (outs[2 * l], outs[2 * l + 1]) if outs is not None else (None, None)
        with _OnSide(wside, dy, hs[l]):
            grads[2 * l] = _wgrad(dy, hs[l], prec, out=o_w)
        assert cs is not None or not g16, "an fp16 dY comes with its column sums"
        grads[2 * l + 1] = x3.colsum(dy if cs is None else cs, out=o_b)
        wt = x3.pack(ws[l], trans=True, prec=prec)
        # pre-scaled fp16 dY: read at scale 1, the output unscaled by 1 / s (and stored fp16(. s) again)
        ascale, cscale = (1.0, 1.0 / s) if g16 else (s, None)
        if l > 0:  # dY of layer l-1 = (dY W) * (h_l > 0): the ReLU bits of layer l-1's forward
            cs = x3.colsum_buf(M, ws[l].shape[1], dy.device)
            out = torch.empty((M, ws[l].shape[1]), dtype=torch.float16, device=dy.device) if g16 else None
            dy = x3.gemm(dy, wt, mbits_in=ctx_bits[l - 1], colsum=cs, ascale=ascale, cscale=cscale, out=out,
                         oscale=s)
        elif need_dx:
            dx = x3.gemm(dy, wt, ascale=ascale, cscale=cscale)
    return dx, grads


def _g16(prec, hs, ws, need_dx):
    """fp16 pre-scaled input gradients (f16 with fp16 activations, F16_ACT): every input-gradient GEMM
    takes fp16 A at its shape (the weight gradients take fp16 dY at the update's shapes)."""
    from . import x3

    M = hs[0].shape[0]
    if prec != "f16" or hs[-1].dtype != torch.float16:
        return False
    shapes = [(w.shape[1], w.shape[0]) for w in ws[1:]] + ([(ws[0].shape[1], ws[0].shape[0])] if need_dx else [])
    return all(n % 4 == 0 and k % 4 == 0 and x3.a16_ok(M, n, k) for n, k in shapes)


def _heads_fwd(h, wh, bh):
    """The heads (networks.py:38-41): mm_heads_fwd, fp32 FMA per row with mm_head_sample's arithmetic (the
    rollout's logits, bit for bit), a streaming GEMV over h.  Other head counts: the x3 GEMM."""
    from . import _lib, x3

    M, K = h.shape
    if h.dtype == torch.float16:  # the f16 networks' stored activations (fp32 FMAs over their exact values)
        assert wh.shape[0] == 6 and (K + 31) // 32 == 9 and K % 4 == 0, (wh.shape, K)
        h, wh, bh = h.contiguous(), wh.contiguous(), bh.contiguous()
        out = torch.empty((M, 6), dtype=torch.float32, device=h.device)
        _lib.check(_lib.lib().mm_heads_fwd_h16(_lib.ptr(h), K, K, _lib.ptr(wh), _lib.ptr(bh), M, _lib.ptr(out),
                                                _lib.stream_ptr()), "mm_heads_fwd_h16")
        return out
    if wh.shape[0] != 6 or K % 4 or K > 1024:
        return x3.gemm(h, x3.pack(wh, prec="x3"), bias=bh)
    h, wh, bh = h.contiguous(), wh.contiguous(), bh.contiguous()
    out = torch.empty((M, 6), dtype=torch.float32, device=h.device)
    step = max(1, (2 ** 31 - 1) // (4 * K))  # rows per call: the kernel's buffer resource spans < 2^31 bytes
    for r0 in range(0, M, step):
        m = min(step, M - r0)
        _lib.check(_lib.lib().mm_heads_fwd(_lib.ptr(h[r0:r0 + m]), K, K, _lib.ptr(wh), _lib.ptr(bh), m,
                                            _lib.ptr(out[r0:r0 + m]), _lib.stream_ptr()), "mm_heads_fwd")
    return out


def _heads_bwd(dz, h, wh, bits, out_w=None, out_b=None, oscale=None, wside=None):
    """The heads' backward: (dY through the last ReLU, its tile column sums, dWh, dbh).  oscale: dY
    stored fp16 pre-scaled (fp16(dY oscale), see _g16).  wside: as _mlp_bwd's."""
    from . import x3

    with _OnSide(wside, dz, h):
        dwh = _wgrad(dz, h, "x3", out=out_w)
    dbh = x3.colsum(dz, out=out_b)
    dy, cs = x3.heads_bwd(dz, wh, bits, oscale=oscale)  # (dz Wh) * (h > 0)
    return dy, cs, dwh, dbh


class _EngineTrunk(torch.autograd.Function):
    """The actor trunk alone with autograd (Actor.trunk under grad).
    apply(prec, h0, W0, b0, W1, b1, ...) -> h_last."""

    @staticmethod
    def forward(ctx, prec, h0, *params):
        hs, bits = _mlp_fwd(h0, params[0::2], params[1::2], prec, True)
        ctx.save_for_backward(*hs, *params[0::2])
        ctx.bits, ctx.prec = bits, prec
        return hs[-1]

    @staticmethod
    def backward(ctx, dh):
        L = len(ctx.bits)
        saved = ctx.saved_tensors
        hs, ws = saved[:L + 1], saved[L + 1:]
        dy = torch.ops.aten.threshold_backward(dh.contiguous(), hs[L], 0)  # through the last ReLU
        dx, grads = _mlp_bwd(ctx.bits, hs, ws, dy, None, ctx.prec, ctx.needs_input_grad[1])
        return (None, dx, *grads)


class _EngineActor(torch.autograd.Function):
    """The actor MLP on the engine with autograd: trunk (networks.py:35-36) +
    heads (:38-41).  apply(prec, h0 [M, K0], Wh [J, K], bh [J], W0, b0, W1, b1,
    ...) -> logits [M, J].  The update does not go through autograd
    (Actor.train_forward / train_backward); this serves ``Actor`` under grad."""

    @staticmethod
    def forward(ctx, prec, h0, wh, bh, *params):
        ws, bs = params[0::2], params[1::2]
        hs, bits = _mlp_fwd(h0, ws, bs, prec, True)
        z = _heads_fwd(hs[-1], wh, bh)
        ctx.save_for_backward(*hs, wh, *ws)
        ctx.bits, ctx.prec = bits, prec
        return z

    @staticmethod
    def backward(ctx, dz):
        L = len(ctx.bits)
        saved = ctx.saved_tensors
        hs, wh, ws = saved[:L + 1], saved[L + 1], saved[L + 2:]
        dy, cs, dwh, dbh = _heads_bwd(dz.contiguous(), hs[L], wh, ctx.bits[L - 1])
        dx, grads = _mlp_bwd(ctx.bits, hs, ws, dy, cs, ctx.prec, ctx.needs_input_grad[1])
        return (None, dx, dwh, dbh, *grads)


def _critic_fwd(x, params, prec, need_bits, out=None):
    """networks.py:96-102 on the engine: x [M, 130] (8-byte rows) -> ReLU(64) ->
    ReLU(64) -> V [M, 1] (into ``out`` [M, 1] when given).  f16 with bits: the
    hidden activations in fp16 (F16_ACT)."""
    from . import x3

    w0, b0, w1, b1, w2, b2 = params
    act16 = need_bits and _act16(prec, x.shape[0], [w0.shape[0], w1.shape[0]],
                                 [(w1.shape[0], w1.shape[1]), (w2.shape[0], w2.shape[1])])
    hs, bits = _mlp_fwd(x, (w0, w1), (b0, b1), prec, need_bits, act16=act16)
    return x3.gemm(hs[-1], x3.pack(w2, prec=prec), bias=b2, out=out), hs, bits


def _critic_bwd(hs, bits, params, dv, prec, outs=None):
    """The critic's parameter gradients for dV [M, 1]: the value head through the
    last ReLU in one kernel (mm_x3_heads_bwd, J = 1), the input-gradient GEMM
    through the first ReLU (bits + bias-gradient column sums), weight gradients
    on mm_gemm_wgrad.  outs: destinations in parameter order (or None)."""
    from . import x3

    w0, _, w1, _, w2, _ = params
    o = outs if outs is not None else [None] * 6
    dw2 = _wgrad(dv, hs[2], prec, out=o[4])
    db2 = x3.colsum(dv, out=o[5])
    g16 = _g16(prec, hs, (w0, w1), False)  # fp16 pre-scaled input gradients (f16 with fp16 activations)
    dy, cs = x3.heads_bwd(dv, w2, bits[1], oscale=_grad_scale(dv.shape[0], prec) if g16 else None)
    _, grads = _mlp_bwd(bits, hs[:2], (w0, w1), dy, cs, prec, False, outs=o[:4] if outs is not None else None)
    return grads + [dw2, db2]


class _EngineCritic(torch.autograd.Function):
    """The critic on the engine with autograd.  apply(prec, x [M, 130], W0, b0,
    W1, b1, W2, b2) -> V [M, 1]; no gradient for the observations."""

    @staticmethod
    def forward(ctx, prec, x, *params):
        v, hs, bits = _critic_fwd(x, params, prec, True)
        ctx.save_for_backward(*hs, *params)
        ctx.bits, ctx.prec = bits, prec
        return v

    @staticmethod
    def backward(ctx, dv):
        saved = ctx.saved_tensors
        return (None, None, *_critic_bwd(saved[:3], ctx.bits, saved[3:], dv.contiguous(), ctx.prec))


def _grad_of(p):
    """p.grad, allocated if absent (the update writes every element).  A parameter of a
    marlmaze.update.FlatParams gets its view of the flat gradient buffer back if anything replaced or
    cleared its .grad (nn.Module.zero_grad() sets it to None): the all-reduce and mm_clip_adam read the
    flat buffer, so a gradient written anywhere else would be silently lost."""
    flat = getattr(p, "_mm_flat_grad", None)
    if flat is not None:
        if p.grad is None or p.grad.data_ptr() != flat.data_ptr():
            p.grad = flat
        return p.grad
    if p.grad is None:
        p.grad = torch.empty_like(p)
    return p.grad


class Actor(nn.Module):
    """networks.py:13-48.  forward(x) -> [move_logits [B,5], mark_logit [B,1]]."""

    def __init__(self, hidden_sizes=(164, 164, 164, 164, 164), activation=nn.ReLU, parity_mode=True,
                 gemm_prec=None):
        super().__init__()
        hidden_sizes = list(hidden_sizes)
        gemm_prec = FP32_GEMM if gemm_prec is None else gemm_prec
        assert gemm_prec in GEMM_PRECISIONS
        self.gemm_prec = gemm_prec  # the MLP GEMMs' precision on the GPU (the front-end stays fp32)
        self.projection = Projection(parity_mode)
        self.attention = m_Attention()
        self.layers = nn.ModuleList()
        self.activation = activation
        self.layers.append(nn.Linear(FEATURE_AMOUNT * EMBEDDING_DIM, hidden_sizes[0]))
        for a, b in zip(hidden_sizes[:-1], hidden_sizes[1:]):
            self.layers.append(nn.Linear(a, b))
        self.move_head = nn.Linear(hidden_sizes[-1], 5)
        self.mark_head = nn.Linear(hidden_sizes[-1], 1)
        self.initialize_weights()

    def initialize_weights(self):  # networks.py:43-48
        for layer in self.layers:
            nn.init.orthogonal_(layer.weight)
        with torch.no_grad():
            self.move_head.weight *= 0.01
            self.mark_head.weight *= 0.01

    def _adjacent(self, a, b):
        """[a; b] as one view when b's storage directly follows a's (the flat parameter
        layout of marlmaze.update places the two heads so), else None."""
        if (a.is_contiguous() and b.is_contiguous() and a.untyped_storage().data_ptr() == b.untyped_storage().data_ptr()
                and b.data_ptr() == a.data_ptr() + a.numel() * a.element_size()):
            n = a.shape[1:] if a.dim() > 1 else ()
            return torch.as_strided(a, (a.shape[0] + b.shape[0],) + tuple(n), a.stride(), a.storage_offset())
        return None

    def heads(self):
        """[move_head; mark_head] as one [6, K] weight and [6] bias (views when the
        parameters are laid out adjacently -- the same view objects while the
        parameters stay where they are, so packs of them are cached -- else
        concatenated copies)."""
        mw, kw, mb, kb = self.move_head.weight, self.mark_head.weight, self.move_head.bias, self.mark_head.bias
        key = tuple((t.data_ptr(), t.shape) for t in (mw, kw, mb, kb))
        hit = self.__dict__.get("_heads_view")
        if hit is not None and hit[0] == key:
            return hit[1], hit[2]
        w, b = self._adjacent(mw, kw), self._adjacent(mb, kb)
        if w is not None and b is not None:
            self.__dict__["_heads_view"] = (key, w, b)
            return w, b
        return (w if w is not None else torch.cat([mw, kw], 0), b if b is not None else torch.cat([mb, kb], 0))

    def pack_specs(self):
        """The weight packs (x3.pack_many specs) of one train_forward + train_backward."""
        ws = [lin.weight for lin in self.layers]
        return ([(w, False, self.gemm_prec) for w in ws] + [(self.heads()[0], False, "x3")]
                + [(w, True, self.gemm_prec) for w in ws])

    def forward(self, x):
        heads = self.logits(x)
        return [heads[:, :5], heads[:, 5:6]]

    def _mlp_params(self):
        return [t for lin in self.layers for t in (lin.weight, lin.bias)]

    def logits(self, x):
        """[B, 6] = [5 move logits | mark logit] (both heads of networks.py:38-41)."""
        w, b = self.heads()
        h = self._front(x)
        if self._engine(h):
            params = self._mlp_params()
            if torch.is_grad_enabled() and (h.requires_grad or any(p.requires_grad for p in params + [w, b])):
                return _EngineActor.apply(self.gemm_prec, h, w, b, *params)  # trunk + heads, fused backward
            with torch.no_grad():
                hs, _ = _mlp_fwd(h, params[0::2], params[1::2], self.gemm_prec, False)
                return _heads_fwd(hs[-1], w, b)
        return F.linear(self._mlp(h), w, b)

    def trunk(self, x):
        """Everything up to the last hidden layer (networks.py:31-36)."""
        return self._mlp(self._front(x))

    def sample_actions(self, x, head_w, head_b, masks, seed, offset, actions, logp=None, joint_logp=None,
                       offset_dev=None):
        """The rollout's actor step (PPO.py:170-186): front-end, trunk, heads and the action draws
        (ops.head_sample's).  At <= _trunk_max_rows(prec) rows without autograd the trunk, heads and draws run as
        ONE launch (mm_trunk3_head_sample, bit-identical to trunk + ops.head_sample)."""
        from . import ops, x3

        h0 = self._front(x)
        M = h0.shape[0]
        if (not torch.is_grad_enabled() and len(self.layers) == 3 and 0 < M <= _trunk_max_rows(self.gemm_prec) and h0.is_cuda
                and h0.dtype == torch.float32 and self._engine(h0)):
            params = self._mlp_params()
            packs = [x3.pack(w, prec=self.gemm_prec) for w in params[0::2]]
            if x3.trunk3_head_sample_ok(M, h0, packs, self.gemm_prec):
                x3.trunk3_head_sample(h0, packs, params[1::2], head_w.contiguous(), head_b.contiguous(),
                                      masks.to(torch.uint8).contiguous(), seed, offset, actions, logp, joint_logp,
                                      offset_dev=offset_dev)
                return actions, logp, joint_logp
        return ops.head_sample(self._mlp(h0), head_w, head_b, masks, seed, offset, actions=actions, logp=logp,
                               joint_logp=joint_logp, offset_dev=offset_dev)

    def _front(self, x):
        """Projection + attention (networks.py:31-34)."""
        x = torch.as_tensor(x, dtype=torch.float32, device=self.move_head.weight.device).reshape(-1, OBS_SPACE)
        if x.is_cuda:  # product path: fused HIP front-end (no fallback on the GPU)
            return _FusedFront.apply(x, self.projection.parity_mode, *front_params(self.projection, self.attention))
        return self.attention(self.projection(x))  # host reference path (CPU tests only)

    def _engine(self, h):
        ok = (self.activation is nn.ReLU and _engine_ok(h, [lin.weight.shape[0] for lin in self.layers])
              and all(lin.weight.shape[1] % 4 == 0 for lin in self.layers))
        if h.is_cuda and not ok:
            _warn_torch_path("this Actor's MLP")
        return ok

    def _mlp(self, h):
        """The hidden layers (networks.py:35-36)."""
        if self._engine(h):
            params = self._mlp_params()
            if torch.is_grad_enabled() and (h.requires_grad or any(p.requires_grad for p in params)):
                return _EngineTrunk.apply(self.gemm_prec, h, *params)
            with torch.no_grad():
                hs, _ = _mlp_fwd(h, params[0::2], params[1::2], self.gemm_prec, False)
            return hs[-1]
        act = self.activation()
        for lin in self.layers:
            h = act(F.linear(h, lin.weight, lin.bias))
        return h

    # ---- the update's explicit forward / backward (no autograd; GPU) ----
    def train_forward(self, x):
        """x [M, 65] f32 on the GPU -> (head logits z [M, 6], saved state for
        train_backward).  The forward of get_log_probs' actor calls (PPO.py:66-68)."""
        x = x.contiguous()
        params = self._mlp_params()
        wl = [lin.weight for lin in self.layers]
        act16 = (_act16(self.gemm_prec, x.shape[0], [w_.shape[0] for w_ in wl],
                        [(w_.shape[0], w_.shape[1]) for w_ in wl[1:]]) and (wl[-1].shape[0] + 31) // 32 == 9)
        # with fp16 activations the front-end output is stored fp16 too (the first GEMM -- the streaming
        # kernel's fp16 A source at K = 460 -- and its weight gradient round it to fp16 anyway)
        h16 = act16 and F16_H0 and wl[0].shape[1] % 4 == 0
        ws, h0 = _front_fwd(x, self.projection.parity_mode, front_params(self.projection, self.attention), h16=h16)
        if not self._engine(h0):
            raise ValueError("Actor.train_forward needs the GPU engine's shapes (ReLU, widths <= 272)")
        hs, bits = _mlp_fwd(h0, params[0::2], params[1::2], self.gemm_prec, True, act16=act16)
        w, b = self.heads()
        z = _heads_fwd(hs[-1], w, b)
        return z, (x, ws, hs, bits)

    def train_backward(self, saved, dz):
        """Every parameter's gradient for d loss / d z (dz [M, 6]), written into
        the parameters' .grad storage (allocated when absent)."""
        x, ws, hs, bits = saved
        L = len(self.layers)
        w, _ = self.heads()
        gw = self._adjacent(_grad_of(self.move_head.weight), _grad_of(self.mark_head.weight))
        gb = self._adjacent(_grad_of(self.move_head.bias), _grad_of(self.mark_head.bias))
        params = self._mlp_params()
        g16 = _g16(self.gemm_prec, hs, params[0::2], True)
        from . import x3

        # the weight gradients beside the input-gradient chain (only their row-slice partials are launched in
        # a deferred() scope, so the side stream never writes a .grad; the sums run after the join below)
        wside = wgrad_stream(dz.device) if (WGRAD_STREAM and dz.is_cuda and x3._DEFER) else None
        cur = torch.cuda.current_stream(dz.device) if wside is not None else None
        dy, cs, dwh, dbh = _heads_bwd(dz.contiguous(), hs[L], w, bits[L - 1], out_w=gw, out_b=gb,
                                      oscale=_grad_scale(dz.shape[0], self.gemm_prec) if g16 else None,
                                      wside=wside if gw is not None else None)
        if gw is None:
            self.move_head.weight.grad.copy_(dwh[:5])
            self.mark_head.weight.grad.copy_(dwh[5:])
        if gb is None:
            self.move_head.bias.grad.copy_(dbh[:5])
            self.mark_head.bias.grad.copy_(dbh[5:])
        params = self._mlp_params()
        dh0, _ = _mlp_bwd(bits, hs, params[0::2], dy, cs, self.gemm_prec, True,
                          outs=[_grad_of(p) for p in params], wside=wside if WGRAD_STREAM is True else None)
        _front_bwd_to(ws, x, self.projection.parity_mode, dh0,
                      [_grad_of(p) for p in front_params(self.projection, self.attention)])
        if wside is not None:
            cur.wait_stream(wside)  # the partials are written before the deferred sums read them


def _front_fwd_algo(B):
    if FRONT_FWD_ALGO == "auto":
        return "row2" if B <= FRONT_FWD_ROW2_MAX else "row1"
    return FRONT_FWD_ALGO


def _front_fwd(x, parity, params, h16=False):
    """The fused front-end forward (no autograd): (workspace, h [B, 460]); h16: h stored fp16
    (mm_actor_front_fwd_h16, the f16 networks' update: its consumers round h to fp16 anyway)."""
    from . import _lib

    from . import x3

    L = _lib.lib()
    B = x.shape[0]
    stream = _lib.stream_ptr()

    def prep():  # the folded maps depend on the weights only: once per rollout inside x3.cached_packs()
        ws = torch.empty(L.mm_actor_front_ws_len(), dtype=torch.float32, device=x.device)
        ptrs = [p.data_ptr() for p in params]
        wp = (ctypes.c_void_p * FEATURE_AMOUNT)(*ptrs[:FEATURE_AMOUNT])
        bp = (ctypes.c_void_p * FEATURE_AMOUNT)(*ptrs[FEATURE_AMOUNT:2 * FEATURE_AMOUNT])
        wq, wk, wv = params[2 * FEATURE_AMOUNT:]
        _lib.check(L.mm_actor_front_prep(wp, bp, _lib.ptr(wq), _lib.ptr(wk), _lib.ptr(wv), _lib.ptr(ws), stream),
                   "mm_actor_front_prep")
        return ws

    ws = x3.cached_value("front_prep", params, prep)
    if h16:
        h = torch.empty((B, FEATURE_AMOUNT * EMBEDDING_DIM), dtype=torch.float16, device=x.device)
        algo = _lib.FRONT_FWD["mfma" if _front_fwd_algo(B) == "mfma" else "row1"]
        _lib.check(L.mm_actor_front_fwd_h16_ex(_lib.ptr(ws), _lib.ptr(x), OBS_SPACE, B, int(parity), _lib.ptr(h),
                                               algo, stream), "mm_actor_front_fwd_h16_ex")
        return ws, h
    h = torch.empty((B, FEATURE_AMOUNT * EMBEDDING_DIM), dtype=torch.float32, device=x.device)
    _lib.check(L.mm_actor_front_fwd_ex(_lib.ptr(ws), _lib.ptr(x), OBS_SPACE, B, int(parity), _lib.ptr(h),
                                       _lib.FRONT_FWD[_front_fwd_algo(B)], stream), "mm_actor_front_fwd_ex")
    return ws, h


def _front_bwd_to(ws, x, parity, dh, grads):
    """The fused front-end backward writing the parameter gradients into ``grads``
    (front_params order; each in its module layout) -- mm_actor_front_bwd_to."""
    from . import _lib

    L = _lib.lib()
    B = x.shape[0]
    dh = dh.contiguous()
    grid = _front_bwd_grid(B, x.device)
    plen = L.mm_actor_front_partial_len()
    partial = torch.empty((grid, plen), dtype=torch.float32, device=x.device)
    red = torch.empty(plen, dtype=torch.float64, device=x.device)  # the fp64 sums
    assert all(g.is_contiguous() for g in grads)
    ptrs = [g.data_ptr() for g in grads]
    gw = (ctypes.c_void_p * FEATURE_AMOUNT)(*ptrs[:FEATURE_AMOUNT])
    gb = (ctypes.c_void_p * FEATURE_AMOUNT)(*ptrs[FEATURE_AMOUNT:2 * FEATURE_AMOUNT])
    gq, gk, gv = grads[2 * FEATURE_AMOUNT:]
    _lib.check(L.mm_actor_front_bwd_to(_lib.ptr(ws), _lib.ptr(x), OBS_SPACE, B, int(parity), _lib.ptr(dh),
                                       _lib.ptr(partial), grid, _lib.ptr(red), gw, gb, _lib.ptr(gq), _lib.ptr(gk),
                                       _lib.ptr(gv), _lib.FRONT_BWD[FRONT_BWD_ALGO], _lib.stream_ptr()),
               "mm_actor_front_bwd_to")


class Critic(nn.Module):
    """networks.py:84-106.  forward(x [.., agents, 65]) -> V [B, 1]."""

    def __init__(self, agent_amount, hidden_sizes=(128, 128), activation=nn.ReLU, gemm_prec=None):
        super().__init__()
        hidden_sizes = list(hidden_sizes)
        gemm_prec = FP32_GEMM if gemm_prec is None else gemm_prec
        assert gemm_prec in GEMM_PRECISIONS
        self.gemm_prec = gemm_prec  # the GEMMs' precision on the GPU
        self.layers = nn.ModuleList()
        self.activation = activation
        self.agent_amount = agent_amount
        self.layers.append(nn.Linear(agent_amount * OBS_SPACE, hidden_sizes[0]))
        for a, b in zip(hidden_sizes[:-1], hidden_sizes[1:]):
            self.layers.append(nn.Linear(a, b))
        self.layers.append(nn.Linear(hidden_sizes[-1], 1))
        self.initialize_weights()

    def initialize_weights(self):  # networks.py:104-106
        for layer in self.layers:
            nn.init.orthogonal_(layer.weight)

    def _params(self):
        return [t for lin in self.layers for t in (lin.weight, lin.bias)]

    def _engine(self, x):
        # the engine's critic: three layers, hidden widths <= 64 (the 8-byte-row A source of the [M, 130] input)
        ok = (len(self.layers) == 3 and self.activation is nn.ReLU and x.shape[1] % 2 == 0
              and all(lin.weight.shape[0] <= 64 for lin in self.layers)
              and _engine_ok(x, [lin.weight.shape[0] for lin in self.layers]))
        if x.is_cuda and not ok:
            _warn_torch_path("this Critic")
        return ok

    def forward(self, x):
        x = torch.as_tensor(x, dtype=torch.float32, device=self.layers[0].weight.device)
        x = x.reshape(-1, self.agent_amount * OBS_SPACE)
        if self._engine(x):
            x = x.contiguous()
            params = self._params()
            if torch.is_grad_enabled() and any(p.requires_grad for p in params):
                return _EngineCritic.apply(self.gemm_prec, x, *params)
            with torch.no_grad():
                return _critic_fwd(x, params, self.gemm_prec, False)[0]
        act = self.activation()
        for lin in self.layers[:-1]:
            x = act(F.linear(x, lin.weight, lin.bias))
        return F.linear(x, self.layers[-1].weight, self.layers[-1].bias)

    # ---- the update's explicit forward / backward (no autograd; GPU) ----
    @torch.no_grad()
    def value_into(self, x, out):
        """V(x) written into out ([M] or [M, 1] fp32, contiguous) -- the rollout's per-step values without a
        copy (GPU engine shapes only)."""
        from . import _lib

        x = x.reshape(-1, self.agent_amount * OBS_SPACE)  # as forward(): a mismatched input fails here
        if not self._engine(x):
            out.copy_(self(x).reshape(out.shape))
            return out
        w0, b0, w1, b1, w2, b2 = self._params()
        # the kernel takes x's width as w0's row stride: the fused path only where they agree
        if (len(self.layers) == 3 and w0.shape[0] == 64 and w0.shape[1] == x.shape[1] and w1.shape == (64, 64)
                and w2.shape == (1, 64) and x.shape[1] <= 132 and out.is_contiguous()):
            # the three layers in one launch on the fp32 MFMA (mm_critic_value; also for the fp16 networks: the
            # rollout's values are then fp32-class, the update's critic runs in fp16)
            _lib.check(_lib.lib().mm_critic_value(_lib.ptr(x), x.stride(0), x.shape[1], x.shape[0], 64, 64,
                                                   *(_lib.ptr(t) for t in (w0, b0, w1, b1, w2, b2)), _lib.ptr(out),
                                                   _lib.stream_ptr()), "mm_critic_value")
            return out
        _critic_fwd(x, self._params(), self.gemm_prec, False, out=out.view(-1, 1))
        return out

    def train_forward(self, x):
        """x [M, agents * 65] f32 on the GPU -> (V [M, 1], saved state)."""
        x = x.reshape(-1, self.agent_amount * OBS_SPACE).contiguous()
        assert x.is_cuda and self._engine(x)
        v, hs, bits = _critic_fwd(x, self._params(), self.gemm_prec, True)
        return v, (hs, bits)

    def pack_specs(self):
        """The weight packs (x3.pack_many specs) of one train_forward + train_backward."""
        ws = [lin.weight for lin in self.layers]
        return [(w, False, self.gemm_prec) for w in ws] + [(w, True, self.gemm_prec) for w in ws[1:-1]]

    def train_backward(self, saved, dv):
        """Every parameter's gradient for d loss / d V (dv [M, 1]) into .grad."""
        hs, bits = saved
        params = self._params()
        _critic_bwd(hs, bits, params, dv.reshape(-1, 1).contiguous(), self.gemm_prec,
                    outs=[_grad_of(p) for p in params])
