"""Flat parameter storage and the hand-written optimizer step of the PPO update.

The reference steps two ``torch.optim.Adam`` optimizers after
``clip_grad_norm_`` (PPO.py:18-19, 74-85).  On the GPU that is ~10 framework
launches per minibatch (foreach norms, stack, clamp, scale, fused Adam x2) plus
copies.  Here:

* ``FlatParams`` lays the parameters of the actor AND the critic out in ONE
  flat fp32 buffer (every parameter's ``.data`` becomes a view of it) and their
  gradients in a second one (``.grad`` views), one segment per network.  The
  explicit backward (``Actor.train_backward``) writes straight into those
  views, the data-parallel all-reduce is one collective on the gradient
  buffer, and the two heads sit back to back so ``Actor.heads()`` is a view.
* ``FlatAdam`` keeps ``torch.optim.Adam``'s interface -- ``param_groups``
  (``decay_lr`` edits ``lr`` there, PPO.py:216-220), ``state_dict`` /
  ``load_state_dict`` in torch's own format (``PPO.pth`` files move both ways)
  -- with the moments in flat buffers.
* ``clip_adam`` is clip_grad_norm_ + Adam for both networks in two launches
  (``mm_clip_adam``, csrc/update_kernels.hip).
"""
import math

import torch

from . import _lib, x3

_ALIGN = 4  # floats: every parameter starts 16-byte aligned (the GEMM engine's fp32 operands)


class FlatParams:
    """One flat fp32 buffer for the parameters of several modules and one for their gradients.

    ``segments``: a list (one entry per network) of parameter lists, in the order to lay them out.
    ``adjacent``: groups of parameters placed back to back with no alignment padding between them
    (e.g. the two heads' weights, so [move; mark] is one [6, K] view).  Padding elements stay zero in
    all buffers (no gradient, no update)."""

    def __init__(self, segments, adjacent=()):
        glued = {id(p): i for i, grp in enumerate(adjacent) for p in grp[1:]}
        dev = segments[0][0].device
        self.segs = []  # (offset, length) per segment
        self.offsets = {}  # id(param) -> element offset
        off = 0
        for params in segments:
            start = off
            for p in params:
                if id(p) not in glued:
                    off = (off + _ALIGN - 1) // _ALIGN * _ALIGN
                self.offsets[id(p)] = off
                off += p.numel()
            off = (off + _ALIGN - 1) // _ALIGN * _ALIGN
            self.segs.append((start, off - start))
        self.numel = off
        self.data = torch.zeros(off, dtype=torch.float32, device=dev)
        self.grad = torch.zeros(off, dtype=torch.float32, device=dev)
        self.params = [p for params in segments for p in params]
        with torch.no_grad():
            for p in self.params:
                o = self.offsets[id(p)]
                v = self.data[o:o + p.numel()].view_as(p)
                v.copy_(p.data)
                p.data = v
                p.grad = self.grad[o:o + p.numel()].view_as(p)
                p._mm_flat_grad = p.grad  # networks._grad_of re-binds .grad to it if anything replaced it

    def seg_view(self, buf, k):
        o, n = self.segs[k]
        return buf[o:o + n]

    def moment_view(self, buf, p):
        """The view of a flat moment buffer that belongs to parameter p."""
        o = self.offsets[id(p)]
        return buf[o:o + p.numel()].view_as(p)


class FlatAdam:
    """torch.optim.Adam over one segment of a FlatParams (PPO.py:18-19).

    Interface: ``param_groups`` (one group; its ``lr`` is read at every step),
    ``state_dict()`` / ``load_state_dict()`` in torch.optim.Adam's format,
    ``zero_grad()``, ``step()`` (this network alone, optional clipping).  The
    update steps the actor and critic together through ``clip_adam``.  The
    moments live in flat buffers shared by the segments (``exp_avg`` /
    ``exp_avg_sq`` of the FlatParams' layout); one step counter per optimizer
    (the reference's parameters all step together)."""

    def __init__(self, flat, seg, params, lr, betas=(0.9, 0.999), eps=1e-8, moments=None):
        self.flat, self.seg = flat, seg
        self.params = list(params)
        # a real Adam only as the holder of the hyper-parameters (its param_groups define torch's
        # state_dict format); it is never stepped
        self._fmt = torch.optim.Adam(self.params, lr=lr, betas=betas, eps=eps)
        self.param_groups = self._fmt.param_groups
        if moments is None:
            moments = (torch.zeros_like(flat.data), torch.zeros_like(flat.data))
        self.exp_avg, self.exp_avg_sq = moments
        self.t = 0

    # ---- torch.optim.Adam's interface ----
    def zero_grad(self, set_to_none=False):
        """Zero this network's gradient segment (the .grad views stay in place: set_to_none is ignored)."""
        self.flat.seg_view(self.flat.grad, self.seg).zero_()

    def state_dict(self):
        sd = self._fmt.state_dict()
        if self.t > 0:
            sd["state"] = {i: {"step": torch.tensor(float(self.t)),
                               "exp_avg": self.flat.moment_view(self.exp_avg, p).detach().clone(),
                               "exp_avg_sq": self.flat.moment_view(self.exp_avg_sq, p).detach().clone()}
                           for i, p in enumerate(self.params)}
        return sd

    def load_state_dict(self, sd):
        groups = sd["param_groups"]
        if len(groups) != 1 or len(groups[0]["params"]) != len(self.params):
            raise ValueError("optimizer state does not match this network's parameters")
        g = groups[0]
        if g.get("weight_decay", 0) or g.get("amsgrad", False) or g.get("maximize", False):
            raise NotImplementedError("FlatAdam implements Adam without weight decay / amsgrad / maximize")
        for k, v in g.items():
            if k != "params":
                self.param_groups[0][k] = v
        steps = set()
        with torch.no_grad():
            for i, p in enumerate(self.params):
                st = sd["state"].get(i, sd["state"].get(str(i)))
                m, v = self.flat.moment_view(self.exp_avg, p), self.flat.moment_view(self.exp_avg_sq, p)
                if st is None:
                    m.zero_()
                    v.zero_()
                    steps.add(0)
                    continue
                m.copy_(torch.as_tensor(st["exp_avg"]).reshape(p.shape))
                v.copy_(torch.as_tensor(st["exp_avg_sq"]).reshape(p.shape))
                steps.add(int(float(st["step"])))
        if len(steps - {0}) > 1:
            raise ValueError(f"parameters at different Adam steps {sorted(steps)}: not supported")
        self.t = max(steps) if steps else 0

    def step(self, max_norm=0.0):
        clip_adam([self], max_norm)

    # ---- the kernel's view ----
    def segment(self, max_norm, grad_scale=1.0):
        """The mm_adam_seg_t of the NEXT step, t + 1 (the caller advances ``t`` once the step is queued)."""
        t = self.t + 1
        g = self.param_groups[0]
        b1, b2 = g["betas"]
        lr = float(g["lr"])
        f = self.flat
        o, n = f.segs[self.seg]
        s = _lib.AdamSeg()
        s.param = f.data.data_ptr() + 4 * o
        s.grad = f.grad.data_ptr() + 4 * o
        s.exp_avg = self.exp_avg.data_ptr() + 4 * o
        s.exp_avg_sq = self.exp_avg_sq.data_ptr() + 4 * o
        s.n = n
        s.max_norm = float(max_norm)
        s.step_size = lr / (1.0 - b1 ** t)  # as the single-tensor Adam forms them (python floats)
        s.bc2_sqrt = math.sqrt(1.0 - b2 ** t)
        s.grad_scale = float(grad_scale)
        return s


def clip_adam(opts, max_norm, norms=None, grad_scale=1.0):
    """clip_grad_norm_(params of each optimizer, max_norm) + each optimizer's Adam step in two launches
    (mm_clip_adam).  norms: optional f32 [len(opts)] device tensor receiving the unclipped norms.
    grad_scale multiplies the gradients first (1 / world under data parallelism: the all-reduce sums).

    Where this differs from clip_grad_norm_ + Adam.step (PPO.py:74-85), none of which the update reads:
    the clipped (and, under DP, averaged) gradient lives only inside the kernel, so ``.grad`` keeps the
    gradient as the backward (and the all-reduce: a SUM over ranks) left it; max_norm <= 0 means no
    clipping (torch would scale every gradient to ~0; the reference always clips at 0.5).  The step
    counters advance only once the launch is queued without error."""
    L = _lib.lib()
    f = opts[0].flat
    g0 = opts[0].param_groups[0]
    for o in opts:
        g = o.param_groups[0]
        if tuple(g["betas"]) != tuple(g0["betas"]) or g["eps"] != g0["eps"] or o.flat is not f:
            raise ValueError("clip_adam steps optimizers with the same betas / eps over one FlatParams")
    segs = (_lib.AdamSeg * len(opts))(*[o.segment(max_norm, grad_scale) for o in opts])
    ws = _workspace(f.data.device, L.mm_clip_adam_ws_len(len(opts)))
    b1, b2 = g0["betas"]
    _lib.check(L.mm_clip_adam(segs, len(opts), float(b1), float(b2), float(g0["eps"]), _lib.ptr(ws),
                              _lib.ptr(norms), _lib.stream_ptr()), "mm_clip_adam")
    for o in opts:
        o.t += 1
    x3.invalidate_packs()  # parameters changed behind torch's version counters


_WS = {}


def _workspace(dev, n):
    key = (str(dev), int(n))
    if key not in _WS:
        _WS[key] = torch.empty(int(n), dtype=torch.float32, device=dev)
    return _WS[key]


def mse_loss(v, rtg, dv=None):
    """nn.MSELoss()(V, rtg) partial sums and its gradient (mm_mse_loss).  Returns (partials, dv)."""
    L = _lib.lib()
    M = v.numel()
    v, rtg = v.reshape(M).contiguous(), rtg.reshape(M).contiguous()
    if dv is None:
        dv = torch.empty(M, dtype=torch.float32, device=v.device)
    part = torch.empty(L.mm_mse_loss_partials(M), dtype=torch.float32, device=v.device)
    _lib.check(L.mm_mse_loss(_lib.ptr(v), _lib.ptr(rtg), M, _lib.ptr(dv), _lib.ptr(part), _lib.stream_ptr()),
               "mm_mse_loss")
    return part, dv


def losses_final(ppo_part, mse_part, M, out):
    """out[0] = the actor loss, out[1] = the critic loss (mm_losses_final)."""
    _lib.check(_lib.lib().mm_losses_final(_lib.ptr(ppo_part), ppo_part.numel(), _lib.ptr(mse_part),
                                          mse_part.numel(), int(M), _lib.ptr(out), _lib.stream_ptr()),
               "mm_losses_final")
    return out
