"""ctypes binding of libmarlmaze.so (the C ABI declared in include/marlmaze.h).

The library is the product: there is no CPU fallback.  Importing this module
on a machine without the built library raises immediately, and every call
checks the returned status code.
"""
import ctypes
import os

import torch  # noqa: F401  (load torch's HIP runtime first: the .so binds to it)

PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# MARLMAZE_LIB: an alternative build of the same library (instrumented builds under tools/)
LIB_PATH = os.environ.get("MARLMAZE_LIB") or os.path.join(PKG_ROOT, "libmarlmaze.so")

OBS_DIM = 65
MASK_DIM = 6
RNG_WORDS = 625
MAX_SIDE = 41
MAZES_PER_BLOCK = 32

ST_GEN_FAIL = 1  # MM_ST_* (maze status word)
ST_BAD_MOVE = 2

GAE_AUTO, GAE_COLUMN, GAE_WALK, GAE_SCAN = 0, 1, 2, 3  # mm_gae_ex algorithms

AF_KNOWS_END = 1
AF_SEES_END = 2
AF_OTHER_KNOWS = 4
AF_HAS_KEY = 8
AF_SEES_KEY = 16
AF_TEAM_KEY = 32
AF_HAS_MARK = 64

# exported symbols (tests check every one of them is present)
EXPORTS = ("mm_version", "mm_env_desc_size", "mm_layout_stride", "mm_env_seed", "mm_env_reset",
           "mm_env_step", "mm_env_step_timed", "mm_env_reset_done", "mm_env_pregen", "mm_gae", "mm_gae_ex", "mm_sample", "mm_head_sample", "mm_head_sample_ex", "mm_heads_fwd",
           "mm_actor_front_ws_len", "mm_actor_front_prep", "mm_actor_front_fwd", "mm_actor_front_fwd_ex",
           "mm_actor_front_grad_len", "mm_actor_front_partial_len", "mm_actor_front_bwd", "mm_actor_front_bwd_ex",
           "mm_actor_front_bwd_to", "mm_actor_front_bwd_grid",
           "mm_x3_tp_len", "mm_x3_tp_pack", "mm_x3_nt", "mm_x3_nt_f32a", "mm_x3_mbits_len",
           "mm_x3_heads_bwd", "mm_ppo_loss_partials", "mm_ppo_loss", "mm_ppo_loss_bwd",
           "mm_gemm_tp_len", "mm_gemm_tp_pack", "mm_gemm_nt", "mm_gemm_nt_algo", "mm_gemm_wgrad_algo", "mm_gemm_wgrad_ws_len",
           "mm_gemm_wgrad", "mm_colsum", "mm_mse_loss_partials", "mm_mse_loss", "mm_losses_final",
           "mm_clip_adam_ws_len", "mm_clip_adam", "mm_gemm_tp_pack_multi", "mm_gemm_wgrad_slices",
           "mm_gemm_wgrad_partials", "mm_colsum_multi_ws_len", "mm_colsum_multi", "mm_wsum_multi", "mm_critic_value",
           "mm_gemm_range_flag", "mm_gemm_nt_h", "mm_gemm_a16_ok", "mm_gemm_wgrad_h", "mm_gemm_wgrad_partials_h",
           "mm_heads_fwd_h16", "mm_x3_heads_bwd_h16", "mm_trunk3_ok", "mm_trunk3",
           "mm_trunk3_head_sample_ok", "mm_trunk3_head_sample", "mm_actor_front_fwd_h16",
           "mm_actor_front_fwd_h16_ex")
VERSION = 307  # mm_version() this binding is written for

PREC_X3, PREC_F16, PREC_X2 = 0, 1, 2  # MM_PREC_*
FRONT_BWD = {"mfma": 0, "valu": 1}  # MM_FRONT_BWD_*
FRONT_FWD = {"row1": 0, "row2": 1, "mfma": 2}  # MM_FRONT_FWD_*
GEMM_ALGO = {"auto": 0, "stream": 1}  # MM_GEMM_*
GEMM_A_F16, GEMM_C_F16, GEMM_B_F16 = 1, 2, 4  # MM_GEMM_A_F16 / _C_F16 / _B_F16


class EnvDesc(ctypes.Structure):
    """mirror of mm_env_t"""
    _fields_ = [
        ("n", ctypes.c_int32), ("size_w", ctypes.c_int32), ("size_h", ctypes.c_int32),
        ("max_timestep", ctypes.c_int32), ("difficulty", ctypes.c_int32),
        ("rand_start", ctypes.c_int32), ("rand_sizes", ctypes.c_int32),
        ("rand_lo", ctypes.c_int32), ("rand_hi", ctypes.c_int32),
        ("layout_stride", ctypes.c_int32),
        ("layout", ctypes.c_void_p), ("agents", ctypes.c_void_p), ("mazes", ctypes.c_void_p),
        ("rng", ctypes.c_void_p), ("work", ctypes.c_void_p),
        ("next_layout", ctypes.c_void_p), ("next_mazes", ctypes.c_void_p), ("next_rng", ctypes.c_void_p),
        ("gen_state", ctypes.c_void_p),
    ]


class AdamSeg(ctypes.Structure):
    """mirror of mm_adam_seg_t"""
    _fields_ = [
        ("param", ctypes.c_void_p), ("grad", ctypes.c_void_p), ("exp_avg", ctypes.c_void_p),
        ("exp_avg_sq", ctypes.c_void_p), ("n", ctypes.c_long), ("max_norm", ctypes.c_float),
        ("step_size", ctypes.c_float), ("bc2_sqrt", ctypes.c_float), ("grad_scale", ctypes.c_float),
    ]


class PackSeg(ctypes.Structure):
    """mirror of mm_pack_seg_t"""
    _fields_ = [("X", ctypes.c_void_p), ("R", ctypes.c_int), ("C", ctypes.c_int), ("ld", ctypes.c_int),
                ("trans", ctypes.c_int), ("tp", ctypes.c_void_p)]


class ColsumSeg(ctypes.Structure):
    """mirror of mm_colsum_seg_t"""
    _fields_ = [("x", ctypes.c_void_p), ("R", ctypes.c_long), ("N", ctypes.c_int), ("out", ctypes.c_void_p)]


class WsumSeg(ctypes.Structure):
    """mirror of mm_wsum_seg_t"""
    _fields_ = [("x", ctypes.c_void_p), ("n", ctypes.c_long), ("S", ctypes.c_int), ("out", ctypes.c_void_p)]


_LIB = None


class MMError(RuntimeError):
    pass


def lib():
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            raise MMError(
                f"libmarlmaze.so not found at {LIB_PATH}: build it with "
                "`python -c 'import __graft_entry__ as g; g.build()'` (hipcc, gfx950). "
                "There is no CPU fallback.")
        if not os.environ.get("MARLMAZE_LIB"):  # the in-tree build must be of the sources in this tree
            from . import _build

            if _build.stored_hash() != _build.source_hash():
                raise MMError(
                    f"{LIB_PATH} was not built from the sources in this tree (its {os.path.basename(_build.HASH_FILE)} "
                    "is missing or differs from the sha256 of csrc/ + include/): rebuild it with "
                    "`python -c 'import __graft_entry__ as g; g.build()'`")
        L = ctypes.CDLL(LIB_PATH)
        P, i32, u64, f32 = ctypes.c_void_p, ctypes.c_int, ctypes.c_uint64, ctypes.c_float
        L.mm_version.restype = i32
        L.mm_layout_stride.argtypes = [i32] * 5
        L.mm_layout_stride.restype = i32
        L.mm_env_seed.argtypes = [ctypes.POINTER(EnvDesc), P, P]
        L.mm_env_seed.restype = i32
        L.mm_env_reset.argtypes = [ctypes.POINTER(EnvDesc), P, P, P, P]
        L.mm_env_reset.restype = i32
        L.mm_env_step.argtypes = [ctypes.POINTER(EnvDesc), P, P, P, P, P, P, i32, P]
        L.mm_env_step.restype = i32
        L.mm_env_step_timed.argtypes = [ctypes.POINTER(EnvDesc), P, P, P, P, P, P, i32, P, P, P]
        L.mm_env_step_timed.restype = i32
        L.mm_env_reset_done.argtypes = [ctypes.POINTER(EnvDesc), P, P, P]
        L.mm_env_reset_done.restype = i32
        L.mm_env_pregen.argtypes = [ctypes.POINTER(EnvDesc), P]
        L.mm_env_pregen.restype = i32
        L.mm_gae.argtypes = [P, P, P, P, i32, i32, f32, f32, P, P, P]
        L.mm_gae.restype = i32
        L.mm_gae_ex.argtypes = [P, P, P, P, i32, i32, f32, f32, P, P, i32, P]
        L.mm_gae_ex.restype = i32
        L.mm_sample.argtypes = [P, P, P, i32, u64, u64, P, P, P, P]
        L.mm_sample.restype = i32
        L.mm_head_sample.argtypes = [P, i32, i32, P, P, P, i32, u64, u64, P, P, P, P, P]
        L.mm_head_sample.restype = i32
        L.mm_heads_fwd.argtypes = [P, i32, i32, P, P, i32, P, P]
        L.mm_heads_fwd.restype = i32
        L.mm_critic_value.argtypes = [P, i32, i32, i32, i32, i32, P, P, P, P, P, P, P, P]
        L.mm_critic_value.restype = i32
        L.mm_head_sample_ex.argtypes = [P, i32, i32, P, P, P, i32, u64, u64, P, P, P, P, P, P]
        L.mm_head_sample_ex.restype = i32
        L.mm_x3_tp_len.argtypes = [i32, i32]
        L.mm_x3_tp_len.restype = ctypes.c_long
        L.mm_x3_tp_pack.argtypes = [P, i32, i32, i32, i32, P, P]
        L.mm_x3_tp_pack.restype = i32
        L.mm_x3_nt.argtypes = [P, P, i32, i32, i32, P, i32, P, i32, P, i32, P, P]
        L.mm_x3_nt.restype = i32
        L.mm_x3_nt_f32a.argtypes = [P, i32, P, i32, i32, i32, P, i32, P, i32, P, P, P, P, i32, P, P]
        L.mm_x3_heads_bwd.argtypes = [P, i32, P, P, i32, i32, P, P, P]
        L.mm_x3_heads_bwd.restype = i32
        L.mm_ppo_loss_partials.argtypes = [i32]
        L.mm_ppo_loss_partials.restype = i32
        L.mm_ppo_loss.argtypes = [P, P, P, P, P, i32, f32, P, P, P]
        L.mm_ppo_loss.restype = i32
        L.mm_ppo_loss_bwd.argtypes = [P, P, P, P, P, i32, P, P]
        L.mm_ppo_loss_bwd.restype = i32
        L.mm_colsum.argtypes = [P, ctypes.c_long, i32, P, i32, P, P]
        L.mm_colsum.restype = i32
        L.mm_mse_loss_partials.argtypes = [i32]
        L.mm_mse_loss_partials.restype = i32
        L.mm_mse_loss.argtypes = [P, P, i32, P, P, P]
        L.mm_mse_loss.restype = i32
        L.mm_losses_final.argtypes = [P, i32, P, i32, i32, P, P]
        L.mm_losses_final.restype = i32
        L.mm_clip_adam_ws_len.argtypes = [i32]
        L.mm_clip_adam_ws_len.restype = ctypes.c_long
        L.mm_clip_adam.argtypes = [ctypes.POINTER(AdamSeg), i32, f32, f32, f32, P, P, P]
        L.mm_clip_adam.restype = i32
        L.mm_actor_front_bwd_to.argtypes = [P, P, i32, i32, i32, P, P, i32, P, ctypes.POINTER(P), ctypes.POINTER(P),
                                            P, P, P, i32, P]
        L.mm_actor_front_bwd_to.restype = i32
        L.mm_env_desc_size.restype = i32
        L.mm_gemm_tp_len.argtypes = [i32, i32, i32]
        L.mm_gemm_tp_len.restype = ctypes.c_long
        L.mm_gemm_tp_pack.argtypes = [i32, P, i32, i32, i32, i32, P, P]
        L.mm_gemm_tp_pack.restype = i32
        L.mm_gemm_nt.argtypes = [i32, P, i32, f32, P, i32, i32, i32, P, i32, P, P, P, f32, P, i32, P]
        L.mm_gemm_nt.restype = i32
        L.mm_gemm_nt_algo.argtypes = [i32]
        L.mm_gemm_nt_algo.restype = i32
        L.mm_gemm_wgrad_algo.argtypes = [i32]
        L.mm_gemm_wgrad_algo.restype = i32
        L.mm_gemm_wgrad_ws_len.argtypes = [i32, i32, i32]
        L.mm_gemm_wgrad_ws_len.restype = ctypes.c_long
        L.mm_gemm_wgrad.argtypes = [i32, P, i32, f32, P, i32, i32, i32, i32, f32, P, P, P]
        L.mm_gemm_wgrad.restype = i32
        L.mm_gemm_tp_pack_multi.argtypes = [i32, ctypes.POINTER(PackSeg), i32, P]
        L.mm_gemm_tp_pack_multi.restype = i32
        L.mm_gemm_wgrad_slices.argtypes = [i32, i32, i32, i32]
        L.mm_gemm_wgrad_slices.restype = i32
        L.mm_gemm_wgrad_partials.argtypes = [i32, P, i32, f32, P, i32, i32, i32, i32, f32, P, P]
        L.mm_gemm_wgrad_partials.restype = i32
        L.mm_gemm_range_flag.argtypes = [P, i32, P]
        L.mm_gemm_range_flag.restype = i32
        # (library 305's fp16-activation entry points; bound when present, so that tools/ab_libs.py can time
        # an older build beside this one -- the product's build has them, tests/test_cpu_host.py checks)
        for name, args in (("mm_gemm_nt_h", [i32, i32, P, i32, f32, P, i32, i32, i32, P, i32, P, P, P, f32, f32, P, i32,
                                             P]),
                           ("mm_x3_heads_bwd_h16", [P, i32, P, P, i32, i32, P, P, f32, P]),
                           ("mm_gemm_a16_ok", [i32, i32, i32, i32, i32]),
                           ("mm_gemm_wgrad_h", [i32, i32, P, i32, f32, P, i32, i32, i32, i32, f32, P, P, P]),
                           ("mm_gemm_wgrad_partials_h", [i32, i32, P, i32, f32, P, i32, i32, i32, i32, f32, P, P]),
                           ("mm_heads_fwd_h16", [P, i32, i32, P, P, i32, P, P]),
                           ("mm_trunk3_ok", [i32, i32, i32, i32, i32, i32, i32]),
                           ("mm_trunk3", [i32, P, i32, i32, i32, P, P, i32, P, P, i32, P, P, i32, P, i32, P]),
                           ("mm_trunk3_head_sample_ok", [i32, i32, i32, i32, i32, i32, i32]),
                           ("mm_actor_front_fwd_h16", [P, P, i32, i32, i32, P, P]),
                           ("mm_actor_front_fwd_h16_ex", [P, P, i32, i32, i32, P, i32, P]),
                           ("mm_trunk3_head_sample", [i32, P, i32, i32, i32, P, P, i32, P, P, i32, P, P, i32, P, P, P,
                                                      u64, u64, P, P, P, P, P, P, i32, P])):
            if hasattr(L, name):
                getattr(L, name).argtypes = args
                getattr(L, name).restype = i32
        L.mm_colsum_multi_ws_len.argtypes = [ctypes.POINTER(ColsumSeg), i32]
        L.mm_colsum_multi_ws_len.restype = ctypes.c_long
        L.mm_colsum_multi.argtypes = [ctypes.POINTER(ColsumSeg), i32, P, P]
        L.mm_colsum_multi.restype = i32
        L.mm_wsum_multi.argtypes = [ctypes.POINTER(WsumSeg), i32, P]
        L.mm_wsum_multi.restype = i32
        L.mm_x3_mbits_len.argtypes = [i32]
        L.mm_x3_mbits_len.restype = ctypes.c_long
        L.mm_x3_nt_f32a.restype = i32
        L.mm_actor_front_ws_len.restype = i32
        L.mm_actor_front_prep.argtypes = [ctypes.POINTER(P), ctypes.POINTER(P), P, P, P, P, P]
        L.mm_actor_front_prep.restype = i32
        L.mm_actor_front_fwd.argtypes = [P, P, i32, i32, i32, P, P]
        L.mm_actor_front_fwd.restype = i32
        L.mm_actor_front_fwd_ex.argtypes = [P, P, i32, i32, i32, P, i32, P]
        L.mm_actor_front_fwd_ex.restype = i32
        L.mm_actor_front_grad_len.restype = i32
        L.mm_actor_front_partial_len.restype = i32
        L.mm_actor_front_bwd_grid.argtypes = [i32, i32]
        L.mm_actor_front_bwd_grid.restype = i32
        L.mm_actor_front_bwd.argtypes = [P, P, i32, i32, i32, P, P, i32, P, P, P]
        L.mm_actor_front_bwd.restype = i32
        L.mm_actor_front_bwd_ex.argtypes = [P, P, i32, i32, i32, P, P, i32, P, P, i32, P]
        L.mm_actor_front_bwd_ex.restype = i32
        # the structs this module mirrors must match the library's (a short mm_env_t mirror would make
        # the library read past the caller's struct)
        if L.mm_version() // 100 != VERSION // 100 or L.mm_env_desc_size() != ctypes.sizeof(EnvDesc):
            raise MMError(f"{LIB_PATH}: ABI {L.mm_version()} / mm_env_t of {L.mm_env_desc_size()} bytes, "
                          f"this binding expects {VERSION} / {ctypes.sizeof(EnvDesc)}: rebuild the library")
        _LIB = L
    return _LIB


def check(rc, what):
    if rc != 0:
        raise MMError(f"{what} failed with status {rc}")


def ptr(t):
    """Device pointer of a tensor (None -> NULL)."""
    if t is None:
        return None
    return ctypes.c_void_p(t.data_ptr())


def stream_ptr(stream=None):
    s = stream if stream is not None else torch.cuda.current_stream()
    return ctypes.c_void_p(s.cuda_stream)
