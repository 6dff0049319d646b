"""Tensor-level wrappers of the rollout kernels (GAE scan, action sampler).

Every tensor handed to the C ABI is held in a local variable until the call
returns: a temporary (e.g. ``x.contiguous()`` inside the argument list) would
be released at once, and torch's caching allocator could hand its block to
the next temporary before the enqueued kernel has read it.
"""
import numpy as np
import torch

from . import _lib

GAMMA_F32 = float(np.float32(0.99))


_GAE_ALGOS = {"auto": 0, "column": 1, "walk": 2, "scan": 3}


def gae(reward, value, done, last_value=None, gamma=0.99, lam=0.95, adv=None, rtg=None, algo="auto"):
    """PPO.get_GAEs (PPO.py:193-203) over time-major [T, N] tensors.

    reward, value: f32 [T, N]; done: u8/bool [T, N]; last_value: f32 [N] or
    None (every segment end is an episode end).  Returns (adv, rtg) with
    rtg = adv + value (PPO.py:46).  Bit-exact with the reference's fp32 order
    for algo "auto" / "column" / "walk" (mm_gae_ex); "scan" reassociates the
    recursion (parallel inside episodes, ~1e-7 relative).
    """
    T, N = value.shape
    r = reward.contiguous()
    v = value.contiguous()
    d = done.to(torch.uint8).contiguous()
    lv = last_value.contiguous() if last_value is not None else None
    if adv is None:
        adv = torch.empty_like(v)
    if rtg is None:
        rtg = torch.empty_like(v)
    g = float(np.float32(gamma))
    gl = float(np.float32(gamma * lam))  # python float product, cast once (PPO.py:201)
    _lib.check(_lib.lib().mm_gae_ex(_lib.ptr(r), _lib.ptr(v), _lib.ptr(d), _lib.ptr(lv), int(T), int(N), g, gl,
                                    _lib.ptr(adv), _lib.ptr(rtg), _GAE_ALGOS[algo], _lib.stream_ptr()), "mm_gae_ex")
    return adv, rtg


def sample(move_logits, mark_logits, masks, seed, offset, actions=None, logp=None, joint_logp=None):
    """PPO.get_action (PPO.py:170-186) for every (maze, agent) row.

    move_logits [M, 5] f32, mark_logits [M] or [M, 1] f32, masks [M, 6] u8.
    Returns actions [M, 2] int8, per-row logp [M] f32, joint logp [M/2] f32.
    """
    M = move_logits.shape[0]
    dev = move_logits.device
    ml = move_logits.contiguous()
    kl = mark_logits.contiguous()
    mk = masks.to(torch.uint8).contiguous()
    if actions is None:
        actions = torch.empty((M, 2), dtype=torch.int8, device=dev)
    if logp is None:
        logp = torch.empty(M, dtype=torch.float32, device=dev)
    if joint_logp is None:
        joint_logp = torch.empty((M + 1) // 2, dtype=torch.float32, device=dev)
    _lib.check(_lib.lib().mm_sample(_lib.ptr(ml), _lib.ptr(kl), _lib.ptr(mk), int(M), int(seed) & (2**64 - 1),
                                    int(offset) & (2**64 - 1), _lib.ptr(actions), _lib.ptr(logp),
                                    _lib.ptr(joint_logp), _lib.stream_ptr()), "mm_sample")
    return actions, logp, joint_logp


def head_sample(h, head_w, head_b, masks, seed, offset, actions=None, logp=None, joint_logp=None, logits=None,
                offset_dev=None):
    """Actor heads + PPO.get_action in one kernel (csrc/rl_kernels.hip k_head_sample).

    h [M, K] f32 (last hidden layer), head_w [6, K] = [move_head.weight;
    mark_head.weight], head_b [6], masks [M, 6] u8.  Same draws as ``sample``
    on the same (seed, offset, row); offset_dev (a device int64 [1], optional)
    adds a device-side base to ``offset`` (HIP-graph replays).  Returns
    actions, logp, joint_logp.
    """
    M, K = h.shape
    dev = h.device
    hc = h.contiguous()
    w = head_w.contiguous()
    b = head_b.contiguous()
    mk = masks.to(torch.uint8).contiguous()
    if actions is None:
        actions = torch.empty((M, 2), dtype=torch.int8, device=dev)
    if logp is None:
        logp = torch.empty(M, dtype=torch.float32, device=dev)
    if joint_logp is None:
        joint_logp = torch.empty((M + 1) // 2, dtype=torch.float32, device=dev)
    _lib.check(_lib.lib().mm_head_sample_ex(_lib.ptr(hc), int(hc.stride(0)), int(K), _lib.ptr(w), _lib.ptr(b),
                                            _lib.ptr(mk), int(M), int(seed) & (2**64 - 1), int(offset) & (2**64 - 1),
                                            _lib.ptr(offset_dev), _lib.ptr(actions), _lib.ptr(logp),
                                            _lib.ptr(joint_logp), _lib.ptr(logits), _lib.stream_ptr()),
               "mm_head_sample_ex")
    return actions, logp, joint_logp
