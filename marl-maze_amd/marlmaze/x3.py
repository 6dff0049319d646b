"""Python side of the actor/critic GEMMs (csrc/x3mlp.hip, include/marlmaze.h).

A TP tensor is the int16 buffer holding an fp32 [R, C] matrix as three exact
bf16 planes (precision "x3") or one fp16 plane ("f16") in MFMA fragment order
(R padded to 256, C to 32).  ``TP`` carries its logical shape and precision.
"""
import weakref

import torch

from . import _lib


PRECS = {"x3": _lib.PREC_X3, "f16": _lib.PREC_F16, "x2": _lib.PREC_X2}


class TP:
    __slots__ = ("buf", "R", "C", "prec", "src")

    def __init__(self, R, C, device, buf=None, prec="x3"):
        self.R, self.C, self.prec = int(R), int(C), prec
        self.src = None  # (fp32 tensor, trans) it was packed from: gemm(checked=True) repacks it at x3
        n = _lib.lib().mm_gemm_tp_len(PRECS[prec], self.R, self.C)
        self.buf = buf if buf is not None else torch.empty(n, dtype=torch.int16, device=device)
        assert self.buf.numel() >= n

    def ptr(self):
        return _lib.ptr(self.buf)


# packed weights reused inside a ``cached_packs()`` scope (the rollout: the actor/critic weights are
# fixed while it runs, and every step packs them): id(x) -> {(trans, prec, shape, stride): (weakref to
# x, data_ptr, x._version, generation, TP)}.  An entry is stale when the tensor's version counter moved
# (torch in-place ops) or the generation did: the hand-written optimizer (marlmaze.update) and parameter
# loads call ``invalidate_packs()``, because they write parameters without touching the version counter.
_PACK_CACHE = {}
_CACHE_DEPTH = [0]
_GENERATION = [0]


def invalidate_packs():
    """Parameters were written outside torch's version tracking: cached packs are stale."""
    _GENERATION[0] += 1


class cached_packs:
    """with x3.cached_packs(): ... -- pack() reuses the TP of an unchanged tensor within the scope
    (scopes nest; the cache is dropped when the outermost one ends)."""

    def __enter__(self):
        if _CACHE_DEPTH[0] == 0:
            _PACK_CACHE.clear()
            _DERIVED.clear()
        _CACHE_DEPTH[0] += 1
        return self

    def __exit__(self, *exc):
        _CACHE_DEPTH[0] -= 1
        if _CACHE_DEPTH[0] == 0:
            _PACK_CACHE.clear()
            _DERIVED.clear()
        return False


_DERIVED = {}  # cached_value(): (tag, keys of the inputs, generation) -> result, dropped with the scope


def cached_value(tag, tensors, make):
    """make() once per cached_packs() scope for unchanged ``tensors`` (data_ptr, version counter and the
    invalidate_packs() generation all equal), e.g. the actor front-end's folded-map workspace, which depends
    only on the weights; outside a scope, make() every call."""
    if _CACHE_DEPTH[0] == 0:
        return make()
    key = (tag, tuple((id(t), t.data_ptr(), t._version) for t in tensors), _GENERATION[0])
    hit = _DERIVED.get(key)
    if hit is None:
        hit = _DERIVED[key] = make()
    return hit


def _cache_get(x, key):
    ent = _PACK_CACHE.get(id(x), {}).get(key)
    if (ent is not None and ent[0]() is x and ent[1] == x.data_ptr() and ent[2] == x._version
            and ent[3] == _GENERATION[0]):
        return ent[4]
    return None


def _cache_put(x, key, res):
    if len(_PACK_CACHE) > 256:  # drop entries of tensors that are gone
        for k in [k for k, v in _PACK_CACHE.items() if all(e[0]() is None for e in v.values())]:
            del _PACK_CACHE[k]
    d = _PACK_CACHE.get(id(x))
    if d is None or any(e[0]() is not x for e in d.values()):  # a new tensor at a reused id
        d = _PACK_CACHE[id(x)] = {}
    d[key] = (weakref.ref(x), x.data_ptr(), x._version, _GENERATION[0], res)


def _pack_shape(x, trans):
    assert x.dtype == torch.float32 and x.is_cuda and x.dim() == 2 and x.stride(1) == 1
    R, C = (x.shape[1], x.shape[0]) if trans else (x.shape[0], x.shape[1])
    return R, C, (bool(trans), tuple(x.shape), x.stride(0))


def pack(x, out=None, trans=False, prec="x3"):
    """fp32 [R, C] (or its transpose when trans=True, reading x as [C, R]) -> TP (reused inside a
    ``cached_packs()`` scope while the tensor is unchanged)."""
    R, C, key = _pack_shape(x, trans)
    key = (prec,) + key
    cache = out is None and _CACHE_DEPTH[0] > 0
    if cache:
        hit = _cache_get(x, key)
        if hit is not None:
            return hit
    res = out if out is not None else TP(R, C, x.device, prec=prec)
    assert (res.R, res.C, res.prec) == (R, C, prec)
    _lib.check(_lib.lib().mm_gemm_tp_pack(PRECS[prec], _lib.ptr(x), R, C, x.stride(0), int(trans), res.ptr(),
                                          _lib.stream_ptr()), "mm_gemm_tp_pack")
    res.src = (x, bool(trans))
    if cache:
        _cache_put(x, key, res)
    return res


def pack_many(specs):
    """Pack several weights at once -- specs: (x, trans, prec) -- in one launch per precision
    (mm_gemm_tp_pack_multi, <= 16 a launch) into the ``cached_packs()`` cache, so that the pack() calls
    of a forward and backward that follow find them.  Tensors already cached are skipped.  Returns the
    TPs in spec order."""
    assert _CACHE_DEPTH[0] > 0, "pack_many fills the cache of a cached_packs() scope"
    res, todo = [], {}
    for x, trans, prec in specs:
        R, C, key = _pack_shape(x, trans)
        key = (prec,) + key
        tp = _cache_get(x, key)
        if tp is None:
            tp = TP(R, C, x.device, prec=prec)
            todo.setdefault(prec, []).append(_lib.PackSeg(_lib.ptr(x), R, C, x.stride(0), int(trans), tp.ptr()))
            _cache_put(x, key, tp)
        res.append(tp)
    L = _lib.lib()
    for prec, segs in todo.items():
        for i in range(0, len(segs), 16):
            chunk = segs[i:i + 16]
            arr = (_lib.PackSeg * len(chunk))(*chunk)
            _lib.check(L.mm_gemm_tp_pack_multi(PRECS[prec], arr, len(chunk), _lib.stream_ptr()),
                       "mm_gemm_tp_pack_multi")
    return res


# Reductions deferred to the end of a backward: inside a ``deferred()`` scope, colsum(x, out) and
# wgrad(..., out) launch their per-slab / per-slice partials only, and the final sums of all of them run
# together when the scope ends (mm_colsum_multi / mm_wsum_multi: two + one launches for up to 16 each,
# bit-identical to the per-call forms).  The outputs are valid after the scope.
_DEFER = []


class deferred:
    def __enter__(self):
        self.cols, self.sums, self.keep = [], [], []
        _DEFER.append(self)
        return self

    def __exit__(self, exc_type, *exc):
        _DEFER.remove(self)
        if exc_type is None:
            self.flush()
        return False

    def flush(self):
        L, st = _lib.lib(), _lib.stream_ptr()
        cur = torch.cuda.current_stream(self.keep[0].device) if self.keep and self.keep[0].is_cuda else None
        for t in self.keep:  # partials a side stream made (networks.wgrad_stream): read here, on this stream
            if cur is not None:
                t.record_stream(cur)
        for i in range(0, len(self.cols), 16):
            chunk = self.cols[i:i + 16]
            arr = (_lib.ColsumSeg * len(chunk))(*chunk)
            n = L.mm_colsum_multi_ws_len(arr, len(chunk))
            _lib.check(n if n < 0 else 0, "mm_colsum_multi_ws_len")
            dev = self.keep[0].device
            ws = torch.empty(max(1, n), dtype=torch.float32, device=dev)
            self.keep.append(ws)
            _lib.check(L.mm_colsum_multi(arr, len(chunk), _lib.ptr(ws), st), "mm_colsum_multi")
        for i in range(0, len(self.sums), 16):
            chunk = self.sums[i:i + 16]
            arr = (_lib.WsumSeg * len(chunk))(*chunk)
            _lib.check(L.mm_wsum_multi(arr, len(chunk), st), "mm_wsum_multi")
        # the scratch is freed to torch's caching allocator on this stream: reuse is stream-ordered
        self.cols, self.sums, self.keep = [], [], []


def gemm(a, b, bias=None, relu=False, mbits_in=None, mbits_out=None, colsum=None, ascale=1.0, out=None,
         checked=False, cscale=None, oscale=1.0):
    """out = (1/ascale) ((ascale A) B^T) (+bias)(ReLU) in B's precision (mm_gemm_nt):
    A fp32 [M, K] row-major (16-byte rows, or 8-byte rows for N <= 64), B = TP
    [N, K].  mbits_out records the ReLU mask; mbits_in applies one (the input
    gradient through the ReLU below) with colsum its per-tile column sums.
    ascale: a power of two for fp16 operands (1 for x3); cscale (default 1 / ascale): the output's scale.
    fp16 a / out (f16 only, mm_gemm_nt_h): the f16 networks' stored activations and pre-scaled input gradients
    (an fp16 input-gradient out holds fp16(out * oscale)).
    checked (x2 / f16): read the range flag after the call (a synchronisation) and, when an operand left
    the fp16 range, redo the GEMM at x3 from B's source tensor (pack() records it)."""
    if checked and b.prec != "x3":
        assert b.src is not None, "checked=True needs a TP made by pack()"
        if a.dtype == torch.float16 or (out is not None and out.dtype == torch.float16) or cscale is not None:
            # the x3 redo reads fp32 A, writes fp32 and has no output scale: it could not reproduce these
            raise ValueError("gemm(checked=True) takes fp32 A and output without cscale (the x3 redo's forms)")
        range_flag(clear=True)
        res = gemm(a, b, bias, relu, mbits_in, mbits_out, colsum, ascale, out)
        if int(range_flag(clear=True).item()):
            src, trans = b.src
            res = gemm(a, pack(src, trans=trans, prec="x3"), bias, relu, mbits_in, mbits_out, colsum, 1.0, out)
        return res
    N, K = b.R, b.C
    assert a.dtype in (torch.float32, torch.float16) and a.dim() == 2 and a.stride(1) == 1 and a.shape[1] == K, \
        (a.dtype, a.shape, K)
    M = a.shape[0]
    if out is None:
        out = torch.empty((M, N), dtype=torch.float32, device=a.device)
    if a.dtype == torch.float16 or out.dtype == torch.float16:  # fp16 activations (f16 only: mm_gemm_nt_h)
        assert b.prec == "f16" and out.dtype in (torch.float32, torch.float16), (b.prec, out.dtype)
        flags = ((_lib.GEMM_A_F16 if a.dtype == torch.float16 else 0)
                 | (_lib.GEMM_C_F16 if out.dtype == torch.float16 else 0))
        cs = 1.0 / float(ascale) if cscale is None else float(cscale)
        _lib.check(_lib.lib().mm_gemm_nt_h(PRECS[b.prec], flags, _lib.ptr(a), a.stride(0), float(ascale), b.ptr(),
                                           M, N, K, _lib.ptr(bias), int(relu), _lib.ptr(mbits_in),
                                           _lib.ptr(mbits_out), _lib.ptr(colsum), cs, float(oscale), _lib.ptr(out),
                                           out.stride(0), _lib.stream_ptr()), "mm_gemm_nt_h")
        return out
    assert cscale is None or cscale == 1.0 / float(ascale), "cscale: fp16 operands only"
    _lib.check(_lib.lib().mm_gemm_nt(PRECS[b.prec], _lib.ptr(a), a.stride(0), float(ascale), b.ptr(), M, N, K,
                                     _lib.ptr(bias), int(relu), _lib.ptr(mbits_in), _lib.ptr(mbits_out),
                                     _lib.ptr(colsum), 1.0 / float(ascale), _lib.ptr(out), out.stride(0),
                                     _lib.stream_ptr()), "mm_gemm_nt")
    return out


def trunk3_ok(M, h0, packs, prec):
    """Whether three ReLU layers of these packs (TP [N_l, K_l], one precision) at M rows run as one
    mm_trunk3 launch."""
    L = _lib.lib()
    if not hasattr(L, "mm_trunk3") or len(packs) != 3 or any(p.prec != prec for p in packs):
        return False
    if packs[1].C != packs[0].R or packs[2].C != packs[1].R or h0.shape[1] != packs[0].C:
        return False
    return bool(L.mm_trunk3_ok(PRECS[prec], int(M), packs[0].C, packs[0].R, packs[1].R, packs[2].R,
                               h0.stride(0)))


def trunk3(h0, packs, biases, out=None):
    """relu(relu(relu(h0 W0^T + b0) W1^T + b1) W2^T + b2) in one launch (mm_trunk3; bit-identical to three
    gemm(..., bias, relu=True) calls): h0 fp32 [M, K0], packs the TPs of W0..W2."""
    assert h0.dtype == torch.float32 and h0.dim() == 2 and h0.stride(1) == 1
    M = h0.shape[0]
    if out is None:
        out = torch.empty((M, packs[2].R), dtype=torch.float32, device=h0.device)
    _lib.check(_lib.lib().mm_trunk3(PRECS[packs[0].prec], _lib.ptr(h0), h0.stride(0), M, packs[0].C, packs[0].ptr(),
                                    _lib.ptr(biases[0]), packs[0].R, packs[1].ptr(), _lib.ptr(biases[1]), packs[1].R,
                                    packs[2].ptr(), _lib.ptr(biases[2]), packs[2].R, _lib.ptr(out), out.stride(0),
                                    _lib.stream_ptr()), "mm_trunk3")
    return out


def trunk3_head_sample_ok(M, h0, packs, prec):
    """Whether the trunk + heads + sampler of these packs run as one mm_trunk3_head_sample launch."""
    L = _lib.lib()
    return (trunk3_ok(M, h0, packs, prec) and hasattr(L, "mm_trunk3_head_sample")
            and bool(L.mm_trunk3_head_sample_ok(PRECS[prec], int(M), packs[0].C, packs[0].R, packs[1].R, packs[2].R,
                                                h0.stride(0))))


def trunk3_head_sample(h0, packs, biases, head_w, head_b, masks, seed, offset, actions, logp=None, joint_logp=None,
                       logits=None, offset_dev=None, h3=None):
    """trunk3 + the actor heads + PPO.get_action in one launch (mm_trunk3_head_sample): the same actions,
    log-probs and logits as trunk3 followed by ops.head_sample, bit for bit.  masks [M, 6] u8, actions
    [M, 2] i8 (written); h3 (optional) receives the trunk's output."""
    assert h0.dtype == torch.float32 and h0.dim() == 2 and h0.stride(1) == 1
    M = h0.shape[0]
    assert masks.dtype == torch.uint8 and masks.is_contiguous() and actions.is_contiguous()
    _lib.check(_lib.lib().mm_trunk3_head_sample(
        PRECS[packs[0].prec], _lib.ptr(h0), h0.stride(0), M, packs[0].C, packs[0].ptr(), _lib.ptr(biases[0]),
        packs[0].R, packs[1].ptr(), _lib.ptr(biases[1]), packs[1].R, packs[2].ptr(), _lib.ptr(biases[2]),
        packs[2].R, _lib.ptr(head_w), _lib.ptr(head_b), _lib.ptr(masks), int(seed) & (2**64 - 1),
        int(offset) & (2**64 - 1), _lib.ptr(offset_dev), _lib.ptr(actions), _lib.ptr(logp), _lib.ptr(joint_logp),
        _lib.ptr(logits), _lib.ptr(h3), h3.stride(0) if h3 is not None else 0, _lib.stream_ptr()),
        "mm_trunk3_head_sample")
    return actions, logp, joint_logp


def a16_ok(M, N, K):
    """Whether an f16 GEMM of that shape takes fp16 A (mm_gemm_a16_ok: the B-resident kernel's shapes)."""
    return bool(_lib.lib().mm_gemm_a16_ok(int(M), int(N), int(K), int(K), int(N)))


def range_flag(out=None, clear=True):
    """The library's range flag of the fp16-plane precisions (mm_gemm_range_flag): a device int32 [1],
    nonzero when an x2 / f16 operand converted since the last clear had |x s| >= 2^15 (its GEMM's result
    is not to be used: redo it at x3).  Stream-ordered; clears the flag unless clear=False."""
    if out is None:
        out = torch.empty(1, dtype=torch.int32, device="cuda")
    _lib.check(_lib.lib().mm_gemm_range_flag(_lib.ptr(out), int(bool(clear)), _lib.stream_ptr()),
               "mm_gemm_range_flag")
    return out


def set_algo(name):
    """The kernel gemm() runs (mm_gemm_nt_algo, process-wide): "auto" = B resident in LDS where the
    shape fits, "stream" = B streamed per k-step.  Returns the previous setting's name."""
    prev = _lib.lib().mm_gemm_nt_algo(_lib.GEMM_ALGO[name])
    return {v: k for k, v in _lib.GEMM_ALGO.items()}[prev]


WGRAD_ALGO = {"dma": 0, "reg": 1}  # MM_WGRAD_DMA, MM_WGRAD_REG


def set_wgrad_algo(name):
    """The kernel of the x2 trunk weight gradients (mm_gemm_wgrad_algo, process-wide): "dma" = raw rows
    staged by LDS-DMA into a two-stage ring (k_wgrad_dma), "reg" = staged through registers (k_wgrad_rect).
    Bit-identical results.  Returns the previous setting's name."""
    prev = _lib.lib().mm_gemm_wgrad_algo(WGRAD_ALGO[name])
    return {v: k for k, v in WGRAD_ALGO.items()}[prev]


def wgrad(dy, x, prec="x3", dscale=1.0, out=None, checked=False, cscale=None):
    """dW [N, K] = dY^T X summed over the M rows (mm_gemm_wgrad), dY [M, N] and
    X [M, K] fp32 row-major; fp16 operands take dY * dscale (a power of two).
    Inside a ``deferred()`` scope with ``out`` given, the row-slice partials'
    sum runs when the scope ends.  checked (x2 / f16): as gemm()'s -- redone at
    x3 when an operand left the fp16 range."""
    if checked and prec != "x3":
        if dy.dtype == torch.float16 or x.dtype == torch.float16 or cscale is not None:
            # the x3 redo reads fp32 operands and has no output scale: a pre-scaled fp16 dY would come back
            # scaled by its s
            raise ValueError("wgrad(checked=True) takes fp32 dY and X without cscale (the x3 redo's forms)")
        range_flag(clear=True)
        res = wgrad(dy, x, prec, dscale, out)
        if int(range_flag(clear=True).item()):
            res = wgrad(dy, x, "x3", 1.0, out)
        return res
    M, N = dy.shape
    K = x.shape[1]
    assert x.shape[0] == M and dy.stride(1) == 1 and x.stride(1) == 1
    assert x.dtype in (torch.float32, torch.float16) and dy.dtype in (torch.float32, torch.float16), (x.dtype, dy.dtype)
    # fp16 X: f16 activations (x3 / f16); fp16 dY: f16's pre-scaled input gradients (dscale 1, cscale the inverse)
    flags = ((_lib.GEMM_B_F16 if x.dtype == torch.float16 else 0)
             | (_lib.GEMM_A_F16 if dy.dtype == torch.float16 else 0))
    cs = 1.0 / float(dscale) if cscale is None else float(cscale)
    defer = bool(_DEFER) and out is not None and M > 0  # a result the caller reads now is never deferred
    if out is None:
        out = torch.empty((N, K), dtype=torch.float32, device=dy.device)
    L = _lib.lib()
    if defer:
        assert out.is_contiguous()
        S = L.mm_gemm_wgrad_slices(PRECS[prec], M, N, K)
        _lib.check(S if S < 0 else 0, "mm_gemm_wgrad_slices")
        ws = torch.empty(S * N * K, dtype=torch.float32, device=dy.device)
        args = (_lib.ptr(dy), dy.stride(0), float(dscale), _lib.ptr(x), x.stride(0), M, N, K, cs,
                _lib.ptr(ws), _lib.stream_ptr())
        _lib.check(L.mm_gemm_wgrad_partials_h(PRECS[prec], flags, *args) if flags
                   else L.mm_gemm_wgrad_partials(PRECS[prec], *args), "mm_gemm_wgrad_partials")
        d = _DEFER[-1]
        d.sums.append(_lib.WsumSeg(_lib.ptr(ws), N * K, S, _lib.ptr(out)))
        d.keep += [ws, out]
        return out
    ws = torch.empty(max(1, L.mm_gemm_wgrad_ws_len(M, N, K)), dtype=torch.float32, device=dy.device)
    args = (_lib.ptr(dy), dy.stride(0), float(dscale), _lib.ptr(x), x.stride(0), M, N, K, cs,
            _lib.ptr(ws), _lib.ptr(out), _lib.stream_ptr())
    _lib.check(L.mm_gemm_wgrad_h(PRECS[prec], flags, *args) if flags else L.mm_gemm_wgrad(PRECS[prec], *args),
               "mm_gemm_wgrad")
    return out


def mbits(M, device):
    """Buffer for a ReLU bit mask of an [M, N <= 272] GEMM output (accumulator order)."""
    return torch.empty(_lib.lib().mm_x3_mbits_len(int(M)), dtype=torch.int32, device=device)


def nt(a, b, bias=None, relu=False, mask=None, out=None, out_tp=None, want_f32=True, mbits_in=None,
       mbits_out=None, colsum=None):
    """C = A B^T (+bias)(ReLU)(* (mask > 0)) with B = TP [N, K] and A either a TP
    [M, K] or an fp32 row-major [M, K] tensor (split inside the GEMM).  mask: fp32
    [M, N] (the ReLU output of the layer below).  Returns (fp32 C or None, TP C or None)."""
    N, K = b.R, b.C
    if isinstance(a, TP):
        assert a.C == K, (a.C, K)
        M, dev = a.R, a.buf.device
    else:
        assert a.dtype == torch.float32 and a.dim() == 2 and a.stride(1) == 1 and a.shape[1] == K, (a.shape, K)
        M, dev = a.shape[0], a.device
    if want_f32 and out is None:
        out = torch.empty((M, N), dtype=torch.float32, device=dev)
    if mask is not None:
        assert mask.shape == (M, N) and mask.stride(1) == 1
    ldc = out.stride(0) if out is not None else 0
    ldm = mask.stride(0) if mask is not None else 0
    L = _lib.lib()
    head = (_lib.ptr(bias), int(relu), _lib.ptr(mask), ldm)
    tail = (_lib.ptr(out), ldc, out_tp.ptr() if out_tp is not None else None, _lib.stream_ptr())
    if isinstance(a, TP):
        assert mbits_in is None and mbits_out is None
        rc = L.mm_x3_nt(a.ptr(), b.ptr(), M, N, K, *head, *tail)
    else:
        rc = L.mm_x3_nt_f32a(_lib.ptr(a), a.stride(0), b.ptr(), M, N, K, *head, _lib.ptr(mbits_in),
                             _lib.ptr(mbits_out), _lib.ptr(colsum), *tail)
    _lib.check(rc, "mm_x3_nt")
    return out, out_tp


def colsum_buf(M, N, device):
    """Per-16-row-tile column sums [ceil(M / 16), N] (bias-gradient partials)."""
    return torch.empty(((int(M) + 15) // 16, int(N)), dtype=torch.float32, device=device)


def colsum(x, out=None, slabs=256):
    """x [R, N] f32 -> column sums [N] (mm_colsum: two passes in a fixed order) -- the bias gradients,
    from the GEMM epilogues' per-tile sums or straight from dY.  Inside a ``deferred()`` scope with
    ``out`` given (and the default slabs), the sum runs when the scope ends."""
    x = x.contiguous()
    R, N = x.shape
    defer = bool(_DEFER) and out is not None and slabs == 256  # a result the caller reads now is never deferred
    if out is None:
        out = torch.empty(N, dtype=torch.float32, device=x.device)
    if R == 0:
        return out.zero_()
    if defer:
        assert out.is_contiguous() and out.numel() == N
        d = _DEFER[-1]
        d.cols.append(_lib.ColsumSeg(_lib.ptr(x), int(R), int(N), _lib.ptr(out)))
        d.keep += [x, out]
        return out
    G = max(1, min(int(slabs), int(R) // 8))  # slabs of >= 8 rows
    part = torch.empty((G, N), dtype=torch.float32, device=x.device) if G > 1 else None
    _lib.check(_lib.lib().mm_colsum(_lib.ptr(x), int(R), int(N), _lib.ptr(part), G, _lib.ptr(out),
                                    _lib.stream_ptr()), "mm_colsum")
    return out


def heads_bwd(dz, w, bits, oscale=None):
    """dY = (dz [M, J] @ w [J, N]) * bits, and its per-tile column sums.  oscale: dY stored fp16 as
    fp16(dY * oscale) (the f16 networks' pre-scaled input gradients, mm_x3_heads_bwd_h16)."""
    M, J = dz.shape
    N = w.shape[1]
    dz, w = dz.contiguous(), w.contiguous()
    cs = colsum_buf(M, N, dz.device)
    if oscale is not None:
        dy = torch.empty((M, N), dtype=torch.float16, device=dz.device)
        _lib.check(_lib.lib().mm_x3_heads_bwd_h16(_lib.ptr(dz), J, _lib.ptr(w), _lib.ptr(bits), M, N, _lib.ptr(dy),
                                                  _lib.ptr(cs), float(oscale), _lib.stream_ptr()), "mm_x3_heads_bwd_h16")
        return dy, cs
    dy = torch.empty((M, N), dtype=torch.float32, device=dz.device)
    _lib.check(_lib.lib().mm_x3_heads_bwd(_lib.ptr(dz), J, _lib.ptr(w), _lib.ptr(bits), M, N, _lib.ptr(dy),
                                          _lib.ptr(cs), _lib.stream_ptr()), "mm_x3_heads_bwd")
    return dy, cs


def unpack(tp):
    """TP -> fp32 [R, C] (hi + mid + lo), with torch ops: for tests and debugging."""
    Rp, Cp = (tp.R + 255) // 256 * 256, (tp.C + 31) // 32 * 32
    b = tp.buf[:Rp * Cp * 3].view(Rp // 16, Cp // 32, 3, 4, 16, 8).to(torch.int32) & 0xFFFF
    f = (b << 16).view(torch.float32)
    x = f[:, :, 2] + f[:, :, 1] + f[:, :, 0]  # small terms first: exact for a split of an fp32
    # [rt, ks, chunk c, row, j] -> column 32 ks + kcol(c, j), kcol = 4c + j (j < 4) or 16 + 4c + (j - 4)
    x = x.view(Rp // 16, Cp // 32, 4, 16, 2, 4).permute(0, 3, 1, 4, 2, 5)  # [rt, row, ks, half, c, q]
    return x.reshape(Rp, Cp)[:tp.R, :tp.C]
