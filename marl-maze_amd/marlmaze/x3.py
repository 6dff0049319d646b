"""Python side of the actor/critic GEMMs (csrc/x3mlp.hip, include/marlmaze.h).

A TP tensor is the int16 buffer holding an fp32 [R, C] matrix as three exact
bf16 planes (precision "x3") or one fp16 plane ("f16") in MFMA fragment order
(R padded to 256, C to 32).  ``TP`` carries its logical shape and precision.
"""
import weakref

import torch

from . import _lib


PRECS = {"x3": _lib.PREC_X3, "f16": _lib.PREC_F16}


class TP:
    __slots__ = ("buf", "R", "C", "prec")

    def __init__(self, R, C, device, buf=None, prec="x3"):
        self.R, self.C, self.prec = int(R), int(C), prec
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
        _CACHE_DEPTH[0] += 1
        return self

    def __exit__(self, *exc):
        _CACHE_DEPTH[0] -= 1
        if _CACHE_DEPTH[0] == 0:
            _PACK_CACHE.clear()
        return False


def pack(x, out=None, trans=False, prec="x3"):
    """fp32 [R, C] (or its transpose when trans=True, reading x as [C, R]) -> TP (reused inside a
    ``cached_packs()`` scope while the tensor is unchanged)."""
    assert x.dtype == torch.float32 and x.is_cuda and x.dim() == 2 and x.stride(1) == 1
    R, C = (x.shape[1], x.shape[0]) if trans else (x.shape[0], x.shape[1])
    key = (bool(trans), prec, tuple(x.shape), x.stride(0))
    cache = out is None and _CACHE_DEPTH[0] > 0
    if cache:
        ent = _PACK_CACHE.get(id(x), {}).get(key)
        if (ent is not None and ent[0]() is x and ent[1] == x.data_ptr() and ent[2] == x._version
                and ent[3] == _GENERATION[0]):
            return ent[4]
    res = out if out is not None else TP(R, C, x.device, prec=prec)
    assert (res.R, res.C, res.prec) == (R, C, prec)
    _lib.check(_lib.lib().mm_gemm_tp_pack(PRECS[prec], _lib.ptr(x), R, C, x.stride(0), int(trans), res.ptr(),
                                          _lib.stream_ptr()), "mm_gemm_tp_pack")
    if cache:
        if len(_PACK_CACHE) > 256:  # drop entries of tensors that are gone
            for k in [k for k, v in _PACK_CACHE.items() if all(e[0]() is None for e in v.values())]:
                del _PACK_CACHE[k]
        d = _PACK_CACHE.get(id(x))
        if d is None or any(e[0]() is not x for e in d.values()):  # a new tensor at a reused id
            d = _PACK_CACHE[id(x)] = {}
        d[key] = (weakref.ref(x), x.data_ptr(), x._version, _GENERATION[0], res)
    return res


def gemm(a, b, bias=None, relu=False, mbits_in=None, mbits_out=None, colsum=None, ascale=1.0, out=None):
    """out = (1/ascale) ((ascale A) B^T) (+bias)(ReLU) in B's precision (mm_gemm_nt):
    A fp32 [M, K] row-major (16-byte rows, or 8-byte rows for N <= 64), B = TP
    [N, K].  mbits_out records the ReLU mask; mbits_in applies one (the input
    gradient through the ReLU below) with colsum its per-tile column sums.
    ascale: a power of two for fp16 operands (1 for x3)."""
    N, K = b.R, b.C
    assert a.dtype == torch.float32 and a.dim() == 2 and a.stride(1) == 1 and a.shape[1] == K, (a.shape, K)
    M = a.shape[0]
    if out is None:
        out = torch.empty((M, N), dtype=torch.float32, device=a.device)
    _lib.check(_lib.lib().mm_gemm_nt(PRECS[b.prec], _lib.ptr(a), a.stride(0), float(ascale), b.ptr(), M, N, K,
                                     _lib.ptr(bias), int(relu), _lib.ptr(mbits_in), _lib.ptr(mbits_out),
                                     _lib.ptr(colsum), 1.0 / float(ascale), _lib.ptr(out), out.stride(0),
                                     _lib.stream_ptr()), "mm_gemm_nt")
    return out


def set_algo(name):
    """The kernel gemm() runs (mm_gemm_nt_algo, process-wide): "auto" = B resident in LDS where the
    shape fits, "stream" = B streamed per k-step.  Returns the previous setting's name."""
    prev = _lib.lib().mm_gemm_nt_algo(_lib.GEMM_ALGO[name])
    return {v: k for k, v in _lib.GEMM_ALGO.items()}[prev]


def wgrad(dy, x, prec="x3", dscale=1.0, out=None):
    """dW [N, K] = dY^T X summed over the M rows (mm_gemm_wgrad), dY [M, N] and
    X [M, K] fp32 row-major; fp16 operands take dY * dscale (a power of two)."""
    M, N = dy.shape
    K = x.shape[1]
    assert x.shape[0] == M and dy.stride(1) == 1 and x.stride(1) == 1
    if out is None:
        out = torch.empty((N, K), dtype=torch.float32, device=dy.device)
    L = _lib.lib()
    ws = torch.empty(max(1, L.mm_gemm_wgrad_ws_len(M, N, K)), dtype=torch.float32, device=dy.device)
    _lib.check(L.mm_gemm_wgrad(PRECS[prec], _lib.ptr(dy), dy.stride(0), float(dscale), _lib.ptr(x), x.stride(0), M,
                               N, K, 1.0 / float(dscale), _lib.ptr(ws), _lib.ptr(out), _lib.stream_ptr()),
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
    from the GEMM epilogues' per-tile sums or straight from dY."""
    x = x.contiguous()
    R, N = x.shape
    if out is None:
        out = torch.empty(N, dtype=torch.float32, device=x.device)
    if R == 0:
        return out.zero_()
    G = max(1, min(int(slabs), int(R) // 8))  # slabs of >= 8 rows
    part = torch.empty((G, N), dtype=torch.float32, device=x.device) if G > 1 else None
    _lib.check(_lib.lib().mm_colsum(_lib.ptr(x), int(R), int(N), _lib.ptr(part), G, _lib.ptr(out),
                                    _lib.stream_ptr()), "mm_colsum")
    return out


def heads_bwd(dz, w, bits):
    """dY = (dz [M, J] @ w [J, N]) * bits, and its per-tile column sums."""
    M, J = dz.shape
    N = w.shape[1]
    dz, w = dz.contiguous(), w.contiguous()
    dy = torch.empty((M, N), dtype=torch.float32, device=dz.device)
    cs = colsum_buf(M, N, dz.device)
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
