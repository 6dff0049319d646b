"""PPO over N parallel mazes on one or more MI355X -- the reference's PPO API.

Mirrors ``PPO`` of the reference (PPO.py:11-238): same constructor arguments,
same methods (train, get_batch, get_action, get_log_probs, get_state_values,
get_GAEs, get_rtgs, decay_lr, save/load_parameters), same checkpoint dict
(``actor``, ``critic``, ``actor_optim``, ``critic_optim``) so ``PPO.pth`` files
move both ways.  What changes is where the work runs:

* rollout: ``n_envs`` mazes step together in HBM (VecMaze, HIP kernels); per
  step one critic call on all [N, 130] observations, one actor call on all
  [2N, 65] agent rows, one sampler kernel (masked Categorical + Bernoulli,
  PPO.py:170-186) and one env-step kernel.  No host synchronisation inside
  the rollout.
* GAE: one HIP scan over the time-major [T, N] buffers (PPO.get_GAEs,
  PPO.py:193-203, bit-exact fp32).
* update: the clipped-surrogate + value-MSE minibatch loop of PPO.py:46-85,
  both losses in one backward, one flat gradient all-reduce under data
  parallelism (marlmaze.dist), clip_grad_norm_ per network, Adam.

Rollout semantics: the reference collects whole episodes from ONE maze until
more than ``batch_size`` steps are stored (PPO.py:108-141).  Here every maze
advances ``horizon`` steps per batch and episodes continue across batches; a
segment that ends mid-episode is bootstrapped with V(s_T) (``bootstrap=True``)
or treated as an episode end exactly like the reference's last step
(``bootstrap=False``).  The minibatch loop keeps the reference's quirk Q8
(it spans ``batch_size``, not the number of samples collected).
"""
import math
import os
import random
import warnings

import numpy as np
import torch

from . import networks, ops, update, x3
from .dist import DP
from .networks import Actor, Critic
from .vecmaze import VecMaze

MODEL_PATH = "PPO.pth"  # PPO.py:9 (CWD-relative)
# the captured rollout's critic on a side stream (a parallel branch of the graph): MARLMAZE_ROLLOUT_SIDE=0 keeps
# it on the main stream (A/B)
ROLLOUT_SIDE_STREAM = os.environ.get("MARLMAZE_ROLLOUT_SIDE", "1") != "0"
# the rollout's critic values in ONE launch over all T (+1) steps' observations after the env loop (they depend on
# the observations only, and the weights do not change during a rollout): no critic launch and no cross-stream
# hand-off per step.  MARLMAZE_ROLLOUT_CRITIC=step keeps the per-step form (A/B)
ROLLOUT_BATCHED_CRITIC = os.environ.get("MARLMAZE_ROLLOUT_CRITIC", "batched") != "step"
# the update's critic (forward, value loss, backward) on a side stream beside the actor's kernels: the two
# networks share nothing until the loss values and the optimizer step.  At small minibatches (BASELINE
# configs[1]: 26,214 samples) the kernels of either network leave most CUs idle, and at the headline's 209,715
# the critic's kernels still fill the actor's tails: measured (same box, alternating) configs[1] 5.25M ->
# 5.38M env-steps/s, headline 6.96M -> 7.07M, f16 share 8.76M -> 8.95M.  MARLMAZE_CRITIC_STREAM=on (default)
# / off / auto (side stream up to CRITIC_STREAM_MAX_SAMPLES samples per minibatch)
CRITIC_STREAM = os.environ.get("MARLMAZE_CRITIC_STREAM", "on")
CRITIC_STREAM_MAX_SAMPLES = int(os.environ.get("MARLMAZE_CRITIC_STREAM_MAX", "65536"))


def _ppo_loss_fwd(heads, mk, a8, old_logp, adv, clip):
    """mm_ppo_loss: (coef [M] = d loss / d logp, per-workgroup partial sums of the surrogate)."""
    from . import _lib

    L = _lib.lib()
    M = old_logp.shape[0]
    old_logp, adv = old_logp.contiguous(), adv.contiguous()
    coef = torch.empty(M, dtype=torch.float32, device=heads.device)
    part = torch.empty(L.mm_ppo_loss_partials(M), dtype=torch.float32, device=heads.device)
    _lib.check(L.mm_ppo_loss(_lib.ptr(heads), _lib.ptr(mk), _lib.ptr(a8), _lib.ptr(old_logp), _lib.ptr(adv), M,
                             float(clip), _lib.ptr(coef), _lib.ptr(part), _lib.stream_ptr()), "mm_ppo_loss")
    return coef, part


def _ppo_loss_bwd(heads, mk, a8, coef, dloss):
    """mm_ppo_loss_bwd: d loss / d heads [2M, 6] (dloss: a 1-element device tensor)."""
    from . import _lib

    dz = torch.empty_like(heads)
    _lib.check(_lib.lib().mm_ppo_loss_bwd(_lib.ptr(heads), _lib.ptr(mk), _lib.ptr(a8), _lib.ptr(coef),
                                          _lib.ptr(dloss), coef.shape[0], _lib.ptr(dz), _lib.stream_ptr()),
               "mm_ppo_loss_bwd")
    return dz


def _u8(masks):
    masks = masks.contiguous()
    return masks.view(torch.uint8) if masks.dtype == torch.bool else masks.to(torch.uint8)


class _PolicyLoss(torch.autograd.Function):
    """-mean(min(r A, clamp(r, 1-clip, 1+clip) A)), r = exp(logp - old_logp),
    logp = sum over the two agents of get_log_probs (PPO.py:62-72, 154-168),
    straight from the [2M, 6] head logits (mm_ppo_loss, mm_ppo_loss_bwd), with
    autograd (the update itself runs the kernels without it)."""

    @staticmethod
    def forward(ctx, heads, masks, act, old_logp, adv, clip):
        heads = heads.contiguous()
        mk = _u8(masks)
        a8 = act.to(torch.int8).contiguous()
        coef, part = _ppo_loss_fwd(heads, mk, a8, old_logp, adv, clip)
        ctx.save_for_backward(heads, mk, a8, coef)
        return -part.sum() / old_logp.shape[0]

    @staticmethod
    def backward(ctx, dloss):
        heads, mk, a8, coef = ctx.saved_tensors
        dz = _ppo_loss_bwd(heads, mk, a8, coef, dloss.reshape(1).to(torch.float32).contiguous())
        return dz, None, None, None, None, None


class PPO:
    def __init__(self, agent_amount, epochs=500, batch_size=15000, lr=0.0002, discount_rate=0.99, lam=0.95,
                 updates_per_batch=5, clip=0.2, max_grad=0.5, *, n_envs=4096, horizon=None, env_config=None,
                 seed=3234, sample_seed=None, device=None, model_path=MODEL_PATH, load=True, parity_mode=True,
                 bootstrap=True, dp=None, verbose=True, save=True, episode_batches=False,
                 episode_chunk=64, dtype="f32", graph_rollout=False):
        self.maze = None  # wired by Maze.__init__ (maze.py:39-42), as in the reference
        self.dp = dp if dp is not None else DP.single()
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device())
        self.device = torch.device(device)
        # networks are built on the CPU right after the seed, like PPO.py:7,16-17; only the CPU
        # generator is seeded (torch.manual_seed would also reset the caller's CUDA streams) and
        # its state is restored afterwards
        g = torch.random.get_rng_state()
        torch.default_generator.manual_seed(seed)
        # dtype "f32": the networks' GEMMs at fp32-class accuracy (x2 by default: two fp16 planes per operand,
        # three f16 MFMAs per product, range-guarded; x3 = bf16x3 on request); "f16": fp16 MFMA operands with
        # fp32 accumulation, storage and Adam (BASELINE configs[4]); the parameters are fp32 either way
        if dtype not in ("f32", "f16"):
            raise ValueError(f"dtype must be 'f32' or 'f16', not {dtype!r}")
        self.dtype = dtype
        # the fp32-class GEMM arithmetic: networks.FP32_GEMM, "x2" (two fp16 planes, three MFMAs per product)
        # unless MARLMAZE_FP32_GEMM=x3 (three bf16 planes, six)
        prec = networks.FP32_GEMM if dtype == "f32" else "f16"
        self.gemm_prec = prec
        self.actor = Actor([264, 264, 264], parity_mode=parity_mode, gemm_prec=prec).to(self.device)
        self.critic = Critic(agent_amount, hidden_sizes=[64, 64], gemm_prec=prec).to(self.device)
        torch.random.set_rng_state(g)
        # Adam (PPO.py:18-19)
        self.flat = None
        if self.device.type == "cuda":
            # both networks in one flat parameter buffer (marlmaze.update): the explicit backward writes
            # into its gradient twin, one all-reduce under DP, clip + Adam for both in two launches
            a = self.actor
            order = [p for n, p in a.named_parameters() if not n.startswith(("move_head", "mark_head"))]
            order += [a.move_head.weight, a.mark_head.weight, a.move_head.bias, a.mark_head.bias]
            self.flat = update.FlatParams([order, list(self.critic.parameters())],
                                          adjacent=[(a.move_head.weight, a.mark_head.weight),
                                                    (a.move_head.bias, a.mark_head.bias)])
            self.dp.broadcast_tensor(self.flat.data)
            mom = (torch.zeros_like(self.flat.data), torch.zeros_like(self.flat.data))
            self.actor_optim = update.FlatAdam(self.flat, 0, self.actor.parameters(), lr=lr, moments=mom)
            self.critic_optim = update.FlatAdam(self.flat, 1, self.critic.parameters(), lr=lr, moments=mom)
        else:  # the host (CPU torch) form, for CPU runs and tests
            self.dp.broadcast_params([self.actor, self.critic])
            self.actor_optim = torch.optim.Adam(self.actor.parameters(), lr=lr)
            self.critic_optim = torch.optim.Adam(self.critic.parameters(), lr=lr)
        self._one = torch.ones(1, dtype=torch.float32, device=self.device)  # d loss / d loss

        self.agent_amount = agent_amount
        self.epochs = epochs
        self.batch_size = batch_size
        self.lr = lr
        self.discount_rate = discount_rate
        self.lam = lam
        self.updates_per_batch = updates_per_batch
        self.mbatch_size = self.batch_size // 5
        self.clip = clip
        self.max_grad = max_grad

        self.n_envs = int(n_envs)
        self.horizon = int(horizon) if horizon else max(1, math.ceil(batch_size / (self.n_envs * self.dp.world)))
        self.env_config = env_config
        self.bootstrap = bootstrap
        self.episode_batches = bool(episode_batches)  # the reference's whole-episode batches (_episode_batch)
        self.episode_chunk = int(episode_chunk)
        self._fresh = False  # the env was just reset (its first batch needs no reset of its own)
        self.sample_seed = (sample_seed if sample_seed is not None else random.getrandbits(63)) + 7919 * self.dp.rank
        self._sample_offset = 0
        self._shuffle_gen = None
        self.model_path = model_path
        self.verbose = verbose and self.dp.rank == 0
        self.save = save
        self.venv = None
        self._bufs = None
        self.history = []
        self.step_events = None  # list -> rollout records (start, end) events around each env step
        # capture the fixed-horizon rollout (every step's critic, actor trunk, head + sampler, env step and
        # the GAE) in one HIP graph and replay it: at a few thousand mazes the ~15 launches per step are
        # host-bound, a replay is one launch
        self.graph_rollout = bool(graph_rollout)
        self._graph = None
        self.range_redos = 0  # updates redone at x3 by the range guard (_range_guarded)
        self.range_switched = False  # the rollout's operands left the fp16 range: the networks now run x3
        self.batches_discarded = 0  # batches the range guard threw away (their rollout left the fp16 range)
        self.last_update_discarded = False
        self._flag_armed = False  # a rollout cleared the range flag at its start: the next update reads its flag
        self._graph_key = None
        self._graph_warm = False
        self._ctr = None  # device base of the sampler's Philox offset in graph replays
        self._ctr_val = None
        if load:
            self.load_parameters()

    # ------------------------------------------------------------------
    # environment + buffers
    # ------------------------------------------------------------------
    def _env_kwargs(self):
        if self.env_config is not None:
            return dict(self.env_config)
        m = self.maze
        if m is None:
            return dict(default_size=(10, 10), max_timestep=1200)
        return dict(default_size=tuple(m.default_size), max_timestep=m.max_timestep, difficulty=m.difficulty,
                    rand_start=m.rand_start, rand_sizes=m.rand_sizes, rand_range=tuple(m.rand_range))

    def _ensure_env(self):
        if self.venv is not None:
            return
        n = self.n_envs
        base = int(self.env_config.get("seed_base", 0)) if self.env_config else random.getrandbits(32)
        kw = {k: v for k, v in self._env_kwargs().items() if k != "seed_base"}
        seeds = np.arange(n, dtype=np.uint64) + np.uint64(base) + np.uint64(self.dp.rank * n)
        self.venv = VecMaze(n, seeds=seeds, device=self.device, **kw)
        T, d = self.horizon, self.device
        self._bufs = dict(
            obs=torch.zeros((T + 1, n, 2, 65), dtype=torch.float32, device=d),
            masks=torch.zeros((T + 1, n, 2, 6), dtype=torch.uint8, device=d),
            act=torch.zeros((T, n, 2, 2), dtype=torch.int8, device=d),
            logp=torch.zeros((T, n), dtype=torch.float32, device=d),
            rowlogp=torch.zeros((T, 2 * n), dtype=torch.float32, device=d),
            val_all=torch.zeros((T + 1, n), dtype=torch.float32, device=d),  # [T] values + the bootstrap row
            rew=torch.zeros((T, n), dtype=torch.float32, device=d),
            done=torch.zeros((T, n), dtype=torch.uint8, device=d),
            stats=torch.zeros((T, n, 2), dtype=torch.int32, device=d),
            adv=torch.zeros((T, n), dtype=torch.float32, device=d),
            rtg=torch.zeros((T, n), dtype=torch.float32, device=d),
        )
        self._bufs["val"] = self._bufs["val_all"][:T]
        self._bufs["last_val"] = self._bufs["val_all"][T]
        self.venv.reset(obs=self._bufs["obs"][0], masks=self._bufs["masks"][0])
        self._fresh = True

    # ------------------------------------------------------------------
    # rollout (PPO.get_batch, PPO.py:89-152)
    # ------------------------------------------------------------------
    def _arm_range_flag(self):
        """A rollout starts: clear the library's range flag, so that what the next update reads as the
        rollout's flag (``pre``, _range_guarded) covers this batch's GEMMs and nothing older."""
        if self.flat is not None and self.gemm_prec != "x3":
            x3.range_flag(clear=True)
            self._flag_armed = True

    @torch.no_grad()
    def rollout(self):
        """Advance every maze ``horizon`` steps; fills the [T, N] buffers."""
        self._arm_range_flag()
        self._ensure_env()
        b, n, T = self._bufs, self.n_envs, self.horizon
        if self.graph_rollout and self.step_events is None and self.device.type == "cuda":
            return self._rollout_graph(b, n, T)
        with x3.cached_packs():  # the weights are fixed during the rollout: pack them once, not per step
            return self._rollout_steps_deferred(b, n, T)

    def _rollout_steps_deferred(self, b, n, T):
        """_rollout_steps with the side-stream maze pre-generation queued once, after the last step
        (VecMaze.defer_pregen): the steps' kernels get the GPU to themselves."""
        self.venv.defer_pregen = True
        try:
            return self._rollout_steps(b, n, T)
        finally:
            self.venv.defer_pregen = False
            self.venv.flush_pregen()

    def _rollout_graph(self, b, n, T):
        """The rollout as a replay of a captured HIP graph (same kernels, same
        draws: the sampler reads its Philox base offset from the device)."""
        # everything the captured launches hold by value: a change re-captures
        key = (id(self.venv), self.flat.data.data_ptr() if self.flat is not None else None, T, id(b["obs"]),
               self.sample_seed, float(self.discount_rate), float(self.lam), bool(self.bootstrap))
        if self._graph is None or self._graph_key != key:
            if not self._graph_warm:  # the first rollout runs uncaptured (one-time host work: kernel attributes)
                self._graph_warm = True
                with x3.cached_packs():
                    return self._rollout_steps_deferred(b, n, T)
            self._graph = torch.cuda.CUDAGraph()
            self._ctr = torch.tensor([self._sample_offset], dtype=torch.int64, device=self.device)
            self._ctr_val = self._sample_offset
            torch.cuda.synchronize(self.device)
            self.venv.capturing = True
            try:
                with torch.cuda.graph(self._graph):
                    with x3.cached_packs():
                        self._rollout_steps(b, n, T, offset_dev=self._ctr)
                    self._ctr += T
            finally:
                self.venv.capturing = False
            self._graph_key = key
        if self._ctr_val != self._sample_offset:  # an uncaptured rollout ran in between
            self._ctr.fill_(self._sample_offset)
        self._graph.replay()
        self._sample_offset += T
        self._ctr_val = self._sample_offset
        self.venv._kick_pregen()  # refill the next mazes the replay's resets consumed
        return b

    def _rollout_steps(self, b, n, T, offset_dev=None):
        head_w, head_b = self.actor.heads()
        cur = torch.cuda.current_stream(self.device) if self.device.type == "cuda" else None
        # the critic reads only the observations, which stay in the [T + 1] buffer: by default its values for
        # every step come from one launch after the loop (ROLLOUT_BATCHED_CRITIC); the per-step form runs it on
        # a side stream beside the actor when the rollout is captured (two branches of the graph)
        batched = ROLLOUT_BATCHED_CRITIC and cur is not None
        side = (self._critic_stream() if (self.graph_rollout and cur is not None and ROLLOUT_SIDE_STREAM
                                          and not batched) else None)
        for t in range(T):
            obs_t = b["obs"][t]
            if batched:
                pass
            elif side is not None:
                side.wait_stream(cur)  # obs[t] written by the previous step's env kernel
                with torch.cuda.stream(side):
                    self.critic.value_into(obs_t, b["val"][t])
            elif cur is not None:
                self.critic.value_into(obs_t, b["val"][t])
            else:
                b["val"][t] = self.critic(obs_t).view(n)
            # actor trunk, heads and sampling (PPO.py:170-186): one launch after the front-end at small N
            # (Actor.sample_actions), else the trunk's GEMMs + ops.head_sample
            self.actor.sample_actions(obs_t.view(2 * n, 65), head_w, head_b, b["masks"][t].view(2 * n, 6),
                                      self.sample_seed, t if offset_dev is not None else self._sample_offset,
                                      actions=b["act"][t].view(2 * n, 2), logp=b["rowlogp"][t],
                                      joint_logp=b["logp"][t], offset_dev=offset_dev)
            if offset_dev is None:
                self._sample_offset += 1
            ev = self.step_events
            if ev is None:
                self.venv.step(b["act"][t], auto_reset=True, obs=b["obs"][t + 1], masks=b["masks"][t + 1],
                               reward=b["rew"][t], done=b["done"][t], ep_stats=b["stats"][t])
            else:  # instrumented: HIP events stamped at the env-step kernel's own start / end
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()  # materialise the events; the launch re-stamps them
                e1.record()
                self.venv.step(b["act"][t], auto_reset=2, obs=b["obs"][t + 1], masks=b["masks"][t + 1],
                               reward=b["rew"][t], done=b["done"][t], ep_stats=b["stats"][t], events=(e0, e1))
                self.venv.reset_done(obs=b["obs"][t + 1], masks=b["masks"][t + 1])
                ev.append((e0, e1))
        if side is not None:
            cur.wait_stream(side)  # every value written before the GAE reads them
        last = None
        if batched:  # V(s_0 .. s_T-1) (and V(s_T) for the bootstrap) in one launch
            rows = T + 1 if self.bootstrap else T
            self.critic.value_into(b["obs"][:rows].reshape(rows * n, -1), b["val_all"][:rows].reshape(rows * n))
            last = b["last_val"] if self.bootstrap else None
        elif self.bootstrap:  # (the per-step values' arithmetic for V(s_T) too)
            if cur is not None:
                self.critic.value_into(b["obs"][T], b["last_val"])
            else:
                b["last_val"].copy_(self.critic(b["obs"][T]).view(n))
            last = b["last_val"]
        ops.gae(b["rew"], b["val"], b["done"], last_value=last, gamma=self.discount_rate, lam=self.lam,
                adv=b["adv"], rtg=b["rtg"])
        return b

    def _critic_stream(self):
        if getattr(self, "_cstream", None) is None:
            self._cstream = torch.cuda.Stream(device=self.device)
        return self._cstream

    def _carry_over(self):
        """The next batch starts from the last observation (episodes continue)."""
        b = self._bufs
        b["obs"][0].copy_(b["obs"][self.horizon])
        b["masks"][0].copy_(b["masks"][self.horizon])

    @torch.no_grad()
    def _episode_batch(self):
        """PPO.get_batch (PPO.py:89-152) over ``n_envs`` mazes, whole episodes only.

        Every maze is reset (PPO.py:104) and all step together.  The batch ends
        at the first step t* after which the steps of completed episodes (all
        mazes) exceed ``batch_size`` (per rank under DP) -- with one maze that is
        the reference's rule, the first episode end after more than
        ``batch_size`` steps (PPO.py:126-141).  Episodes still running at t* are
        dropped (the reference keeps only complete episodes).  Samples are
        ordered maze by maze, each maze's episodes in time order (one maze: the
        reference's order), and GAE runs on whole episodes (PPO.py:133; the
        episode-parallel walk of mm_gae_ex, bit-exact).  No step past t* may
        leave a trace (a maze finishing there would draw its next maze from its
        RNG stream, which the reference never does): after step t at most n (t + 1) steps
        can belong to completed episodes, so the steps before
        t_min = batch_size // n run in chunks of ``episode_chunk`` with one host
        synchronisation per chunk.  From t_min on the chunks grow geometrically
        (1, 2, 4, ... up to ``episode_chunk`` steps) from an environment
        snapshot: when the stop step falls inside a chunk, the environment is
        rewound to the chunk's start and only the steps up to t* are replayed
        with the recorded actions, so neither the MT19937 streams nor the
        sampler's Philox offset carry any trace of the overshoot into the next
        batch.
        """
        self._arm_range_flag()
        self._ensure_env()
        n, dev = self.n_envs, self.device
        limit = self.batch_size // self.dp.world
        if self._fresh:  # the state at the batch's first step
            obs0, masks0 = self._bufs["obs"][0].clone(), self._bufs["masks"][0].clone()
        else:
            obs0 = torch.empty((n, 2, 65), dtype=torch.float32, device=dev)
            masks0 = torch.empty((n, 2, 6), dtype=torch.uint8, device=dev)
            self.venv.reset(obs=obs0, masks=masks0)  # PPO.py:104
        self._fresh = False
        head_w, head_b = self.actor.heads()
        chunks = []
        last_end = torch.full((n,), -1, dtype=torch.int64, device=dev)
        t0, t_stop, end_at_stop = 0, None, None
        t_min = limit // n  # the first step after which the batch can be full
        tail = 1  # the next chunk length past t_min
        self._episode_replayed = 0
        with x3.cached_packs():  # the weights are fixed during the batch: packed once, not per step
            while t_stop is None:
                if t0 < t_min:
                    C, snap = min(self.episode_chunk, t_min - t0), None
                else:
                    C, tail = tail, min(2 * tail, self.episode_chunk)
                    snap, off0 = self.venv.snapshot(), self._sample_offset
                ch = dict(obs=torch.empty((C + 1, n, 2, 65), dtype=torch.float32, device=dev),
                          masks=torch.empty((C + 1, n, 2, 6), dtype=torch.uint8, device=dev),
                          act=torch.empty((C, n, 2, 2), dtype=torch.int8, device=dev),
                          logp=torch.empty((C, n), dtype=torch.float32, device=dev),
                          rowlogp=torch.empty((C, 2 * n), dtype=torch.float32, device=dev),
                          val=torch.empty((C, n), dtype=torch.float32, device=dev),
                          rew=torch.empty((C, n), dtype=torch.float32, device=dev),
                          done=torch.empty((C, n), dtype=torch.uint8, device=dev),
                          stats=torch.empty((C, n, 2), dtype=torch.int32, device=dev))
                ch["obs"][0].copy_(obs0)
                ch["masks"][0].copy_(masks0)
                for t in range(C):
                    # the fixed-horizon rollout's value arithmetic (value_into: the fused fp32 kernel), so a
                    # network's stored values do not depend on the batch mode
                    self.critic.value_into(ch["obs"][t], ch["val"][t])
                    self.actor.sample_actions(ch["obs"][t].view(2 * n, 65), head_w, head_b,
                                              ch["masks"][t].view(2 * n, 6), self.sample_seed, self._sample_offset,
                                              actions=ch["act"][t].view(2 * n, 2), logp=ch["rowlogp"][t],
                                              joint_logp=ch["logp"][t])
                    self._sample_offset += 1
                    self.venv.step(ch["act"][t], auto_reset=True, obs=ch["obs"][t + 1], masks=ch["masks"][t + 1],
                                   reward=ch["rew"][t], done=ch["done"][t], ep_stats=ch["stats"][t])
                chunks.append(ch)
                obs0, masks0 = ch["obs"][C], ch["masks"][C]
                # completed-episode steps after each step of the chunk: sum over mazes of (last end + 1)
                tt = torch.arange(t0, t0 + C, device=dev).view(C, 1)
                ends = torch.where(ch["done"].bool(), tt, torch.full_like(tt, -1))
                ends = torch.maximum(torch.cummax(ends, 0).values, last_end.view(1, n))
                filled = (ends + 1).sum(1)
                hit = torch.nonzero(filled > limit)
                if hit.numel():  # one host synchronisation per chunk; only a tail chunk can hit
                    k = int(hit[0, 0])
                    t_stop, end_at_stop = t0 + k, ends[k]
                    if k + 1 < C:  # overshoot: rewind to the chunk's start, replay steps t0 .. t* only
                        self.venv.restore(snap)
                        for t in range(k + 1):
                            self.venv.step(ch["act"][t], auto_reset=True, obs=ch["obs"][t + 1],
                                           masks=ch["masks"][t + 1], reward=ch["rew"][t], done=ch["done"][t],
                                           ep_stats=ch["stats"][t])
                        self._sample_offset = off0 + k + 1
                        self._episode_replayed = k + 1
                else:
                    last_end = ends[-1]
                    t0 += C
        Ts = t_stop + 1  # == the steps kept (the last chunk may hold discarded steps past t_stop)
        cat = {k: torch.cat([c[k][:c["act"].shape[0]] for c in chunks], 0)[:Ts]
               for k in ("obs", "masks", "act", "logp", "val", "rew", "done", "stats")}
        adv, rtg = ops.gae(cat["rew"], cat["val"], cat["done"], gamma=self.discount_rate, lam=self.lam)
        keep = torch.arange(Ts, device=dev).view(Ts, 1) <= end_at_stop.view(1, n)
        nt = torch.nonzero(keep.t())  # (maze, t), maze-major, t ascending
        flat = nt[:, 1] * n + nt[:, 0]
        B = flat.numel()
        pick = lambda x, *shape: x.reshape(Ts * n, *shape)[flat]  # noqa: E731
        st = pick(cat["stats"], 2)
        fin = st[:, 0] > 0
        out = (pick(cat["obs"], 2, 65), pick(cat["act"], 2, 2).float(), pick(cat["logp"]),
               st[fin, 1].tolist(), st[fin, 0].tolist(), pick(cat["masks"], 2, 6).bool(), pick(adv), pick(cat["val"]))
        self._episode_info = dict(t_stop=t_stop, samples=B, rtg=pick(rtg), act=cat["act"], done=cat["done"])
        return out

    def get_batch(self):
        """Reference 8-tuple (PPO.py:151-152).  Default: every maze advances
        ``horizon`` steps, samples flattened time-major.  ``episode_batches``:
        whole episodes only (_episode_batch)."""
        if self.episode_batches:
            return self._episode_batch()
        b = self.rollout()
        T, n = self.horizon, self.n_envs
        B = T * n
        out = (b["obs"][:T].reshape(B, 2, 65).clone(), b["act"].reshape(B, 2, 2).float(),
               b["logp"].reshape(B).clone(), None, None, b["masks"][:T].reshape(B, 2, 6).bool(),
               b["adv"].reshape(B).clone(), b["val"].reshape(B).clone())
        st = b["stats"].reshape(B, 2)
        fin = st[:, 0] > 0
        ep_lens = st[fin, 0].tolist()
        shortest = st[fin, 1].tolist()
        self._carry_over()
        return out[:3] + (shortest, ep_lens) + out[5:]

    # ------------------------------------------------------------------
    # update (PPO.py:46-85)
    # ------------------------------------------------------------------
    def policy_logp(self, obs, act, masks):
        """Sum over agents of get_log_probs (PPO.py:66-68), one actor call on [2M, 65]."""
        M = obs.shape[0]
        ml, kl = self.actor(obs.reshape(2 * M, 65))
        mk = masks.reshape(2 * M, 6).bool()
        a = act.reshape(2 * M, 2)
        ml = ml.masked_fill(~mk[:, 0:5], float("-inf"))
        lp = torch.log_softmax(ml, dim=-1).gather(1, a[:, 0:1].long()).squeeze(1)
        kl = kl.squeeze(1).masked_fill(~mk[:, 5], float("-inf"))
        p = torch.sigmoid(kl)
        p = torch.where(a[:, 1] != 0, p, 1 - p)
        lp = (lp + torch.log(p)).view(M, 2)
        return lp[:, 0] + lp[:, 1]

    def minibatch_grads(self, obs, act, old_logp, adv, rtg, masks, out=None):
        """Losses of PPO.py:62-80 and their gradients in every parameter's .grad
        (before the all-reduce, the clipping and Adam).  Returns (actor_loss,
        critic_loss) as 0-dim tensors (views of ``out`` [2] when given).

        On the GPU: no autograd.  The critic and actor forwards keep what their
        backwards need; the policy loss (mm_ppo_loss) and the value loss
        (mm_mse_loss) hand d loss / d logits and d loss / dV straight to the
        explicit backwards (Actor / Critic .train_backward), which write into the
        flat gradient buffer."""
        if not obs.is_cuda:
            return self._minibatch_grads_host(obs, act, old_logp, adv, rtg, masks)
        M = obs.shape[0]
        a8 = (act if act.dtype == torch.int8 else act.to(torch.int8)).contiguous()
        mk = _u8(masks)
        if out is None:
            out = torch.empty(2, dtype=torch.float32, device=obs.device)
        side = CRITIC_STREAM == "on" or (CRITIC_STREAM == "auto" and M <= CRITIC_STREAM_MAX_SAMPLES)
        if side:
            return self._minibatch_grads_two_streams(obs, a8, old_logp, adv, rtg, mk, out)
        with x3.cached_packs():
            # every weight pack of both networks' forward and backward in one launch per precision, and
            # the backwards' bias-gradient and weight-gradient reductions together at their end
            x3.pack_many(self.critic.pack_specs() + self.actor.pack_specs())
            V, csaved = self.critic.train_forward(obs.reshape(M, -1))
            mse_part, dv = update.mse_loss(V, rtg)
            heads, asaved = self.actor.train_forward(obs.reshape(2 * M, 65))
            coef, ppo_part = _ppo_loss_fwd(heads, mk, a8, old_logp, adv, self.clip)
            dz = _ppo_loss_bwd(heads, mk, a8, coef, self._one)
            update.losses_final(ppo_part, mse_part, M, out)
            with x3.deferred():
                self.actor.train_backward(asaved, dz)
                self.critic.train_backward(csaved, dv)
        return out[0], out[1]

    def _minibatch_grads_two_streams(self, obs, a8, old_logp, adv, rtg, mk, out):
        """minibatch_grads with the critic's forward, value loss and backward on a side stream, beside the
        actor's (the same kernels and arithmetic: the same results bit for bit).  The side stream waits for
        the weight packs; the main stream waits for the critic before the loss values and the optimizer."""
        M = obs.shape[0]
        cur = torch.cuda.current_stream(obs.device)
        side = self._critic_update_stream()
        with x3.cached_packs():
            x3.pack_many(self.critic.pack_specs() + self.actor.pack_specs())
            side.wait_stream(cur)
            with torch.cuda.stream(side):
                V, csaved = self.critic.train_forward(obs.reshape(M, -1))
                mse_part, dv = update.mse_loss(V, rtg)
                with x3.deferred():
                    self.critic.train_backward(csaved, dv)
            heads, asaved = self.actor.train_forward(obs.reshape(2 * M, 65))
            coef, ppo_part = _ppo_loss_fwd(heads, mk, a8, old_logp, adv, self.clip)
            dz = _ppo_loss_bwd(heads, mk, a8, coef, self._one)
            with x3.deferred():
                self.actor.train_backward(asaved, dz)
            cur.wait_stream(side)
            mse_part.record_stream(cur)  # (allocated on the side stream, read on this one)
            update.losses_final(ppo_part, mse_part, M, out)
        return out[0], out[1]

    def _critic_update_stream(self):
        if getattr(self, "_cupd_stream", None) is None:
            self._cupd_stream = torch.cuda.Stream(device=self.device)
        return self._cupd_stream

    def _minibatch_grads_host(self, obs, act, old_logp, adv, rtg, masks):
        """The CPU torch form (autograd, the reference's formulas)."""
        V = self.critic(obs).view(-1)
        cur = self.policy_logp(obs, act, masks)
        ratio = torch.exp(cur - old_logp)
        s1 = ratio * adv
        s2 = torch.clamp(ratio, 1 - self.clip, 1 + self.clip) * adv
        actor_loss = -torch.mean(torch.min(s1, s2))
        critic_loss = torch.nn.functional.mse_loss(V, rtg)
        self.actor_optim.zero_grad(set_to_none=True)
        self.critic_optim.zero_grad(set_to_none=True)
        (actor_loss + critic_loss).backward()  # disjoint parameters: same grads as two backwards
        return actor_loss.detach(), critic_loss.detach()

    def minibatch_step(self, obs, act, old_logp, adv, rtg, masks, out=None):
        """One iteration of PPO.py:58-85: losses, gradients, all-reduce (DP),
        clip_grad_norm_ per network, Adam.  Returns (aloss, closs, gnorm_a,
        gnorm_c) as 0-dim tensors (views of ``out`` [4] when given).

        On the GPU the step is the minibatch_grads launches, one all-reduce of the
        flat gradient buffer under DP (sums; the 1 / world scale is folded into
        the optimizer kernel), and mm_clip_adam for both networks."""
        if self.flat is None:
            return self._minibatch_step_host(obs, act, old_logp, adv, rtg, masks)
        if out is None:
            out = torch.empty(4, dtype=torch.float32, device=obs.device)
        self.minibatch_grads(obs, act, old_logp, adv, rtg, masks, out=out[0:2])
        scale = 1.0
        if self.dp.active:
            self.dp.allreduce_sum(self.flat.grad)
            scale = 1.0 / self.dp.world
        update.clip_adam([self.actor_optim, self.critic_optim], self.max_grad, norms=out[2:4], grad_scale=scale)
        return out[0], out[1], out[2], out[3]

    def _minibatch_step_host(self, obs, act, old_logp, adv, rtg, masks):
        actor_loss, critic_loss = self._minibatch_grads_host(obs, act, old_logp, adv, rtg, masks)
        params = list(self.actor.parameters()) + list(self.critic.parameters())
        self.dp.allreduce_grads(params)
        gna = torch.nn.utils.clip_grad_norm_(self.actor.parameters(), self.max_grad)
        gnc = torch.nn.utils.clip_grad_norm_(self.critic.parameters(), self.max_grad)
        self.actor_optim.step()
        self.critic_optim.step()
        return actor_loss, critic_loss, gna.detach(), gnc.detach()

    def update(self, b_obs, b_act, b_logp, b_masks, b_advs, b_vals, index_list=None, generator=None):
        """Update body of PPO.train; returns per-minibatch (aloss, closs, gnorm_a, gnorm_c) [K, 4]."""
        b_rtgs = b_advs + b_vals
        mean, std = self.dp.global_mean_std(b_advs)
        b_advs = (b_advs - mean) / (std + 1e-10)
        B = b_obs.shape[0]
        if index_list is None:
            if generator is None:  # a per-rank stream (sample_seed differs by rank), not the global RNG
                if self._shuffle_gen is None or self._shuffle_gen.device != b_obs.device:
                    self._shuffle_gen = torch.Generator(device=b_obs.device)
                    self._shuffle_gen.manual_seed(self.sample_seed ^ 0x5EED)
                generator = self._shuffle_gen
            index_list = torch.randperm(B, device=b_obs.device, generator=generator)
        else:
            index_list = torch.as_tensor(index_list, device=b_obs.device, dtype=torch.long)
        # the reference's minibatch loop spans batch_size (Q8).  Under DP, or for a batch smaller than
        # batch_size (explicit horizon * n_envs < batch_size), the batch is used whole: exactly 5
        # minibatches of local_bs // 5 (a remainder of < 5 samples is left out, as the reference's
        # loop leaves out everything past batch_size)
        local_bs = min(self.batch_size // self.dp.world, B)
        whole = self.dp.active or local_bs < self.batch_size
        mb = local_bs // 5 if whole else self.mbatch_size
        if mb < 1:
            raise ValueError(f"batch of {B} samples per rank is too small for 5 minibatches")
        starts = list(range(0, 5 * mb, mb)) if whole else list(range(0, local_bs, mb))
        # the reference shuffles once per batch (PPO.py:48-49): gather the batch into that order once,
        # so every minibatch is a contiguous slice (same rows, no per-minibatch gathers)
        used = min(B, starts[-1] + mb)
        order = index_list[:used]
        p_obs, p_act, p_logp, p_advs, p_rtgs, p_masks = (t[order] for t in (b_obs, b_act, b_logp, b_advs, b_rtgs,
                                                                          b_masks))
        if p_obs.is_cuda:  # the fused policy-loss kernels take int8 actions and u8 masks: convert once
            p_act = p_act.to(torch.int8)
            p_masks = _u8(p_masks)
        K = self.updates_per_batch * len(starts)
        mbs = [(p_obs[s:s + mb], p_act[s:s + mb], p_logp[s:s + mb], p_advs[s:s + mb], p_rtgs[s:s + mb],
                p_masks[s:s + mb]) for s in starts]

        def passes():
            hist = torch.empty((K, 4), dtype=torch.float32, device=b_obs.device)
            k = 0
            for _ in range(self.updates_per_batch):
                self.decay_lr()
                for args in mbs:
                    row = self.minibatch_step(*args, **({"out": hist[k]} if self.flat is not None else {}))
                    if self.flat is None:
                        hist[k] = torch.stack(row)
                    k += 1
            if self.dp.active:  # local losses -> global-minibatch losses (equal shards); norms are already global
                self.dp.allreduce_sum(hist)
                hist /= self.dp.world
            return hist

        self.last_update_discarded = False
        if self.flat is None or self.gemm_prec == "x3":
            return passes()
        return self._range_guarded(passes)

    # ---- range guard of the fp16-plane GEMMs (x2, f16) ----
    def set_gemm_prec(self, prec):
        """The precision of both networks' GEMMs on the GPU ("x2", "x3" or "f16")."""
        assert prec in networks.GEMM_PRECISIONS
        self.gemm_prec = self.actor.gemm_prec = self.critic.gemm_prec = prec
        self._graph = None  # a captured rollout holds the old precision's kernels

    def _range_flags(self, pre, post):
        """(pre_set, post_set) from this rank's two device flags, decided for ALL ranks: under DP the flags
        are MAX-all-reduced before the one host read, so a range violation on any rank's shard takes every
        rank down the same branch (the same redo, the same collectives, identical parameters after it)."""
        flags = torch.cat([pre, post])
        self.dp.allreduce_max(flags)
        return tuple(int(v) for v in flags.tolist())  # the synchronisation

    def _range_guarded(self, passes):
        """Run the update passes; if any GEMM operand they converted to fp16 planes had |x s| >= 2^15 (the
        library's range flag, mm_gemm_range_flag) on any rank, restore the parameters and optimizer state and
        run the same passes again with the bf16x3 GEMMs (fp32's range).  A flag raised since the batch's rollout
        began (its actor GEMMs, on any rank) means this batch's actions and old log-probs did not come from the
        fp32 policy (an inf / NaN accumulator can become 0 through a ReLU): the update on it is thrown away
        (parameters and optimizer state restored, hist NaN, ``last_update_discarded``), and both networks run
        their GEMMs at x3 from now on (``train`` then collects a new batch).  One host synchronisation per
        update (the flags' read)."""
        # the flag raised since this agent's last rollout began (its actor GEMMs); a batch that did not come
        # from a rollout of this agent (update() on given tensors) has no rollout flag: a stale one is dropped
        pre = x3.range_flag(clear=True)
        if not self._flag_armed:
            pre.zero_()
        self._flag_armed = False
        flat = self.flat
        opts = (self.actor_optim, self.critic_optim)
        moments = {id(t): t for o in opts for t in (o.exp_avg, o.exp_avg_sq)}
        snap = (flat.data.clone(), {k: t.clone() for k, t in moments.items()}, [o.t for o in opts],
                [[g["lr"] for g in o.param_groups] for o in opts])

        def restore():
            with torch.no_grad():
                flat.data.copy_(snap[0])
                for k, t in moments.items():
                    t.copy_(snap[1][k])
            for o, t, lrs in zip(opts, snap[2], snap[3]):
                o.t = t
                for g, lr in zip(o.param_groups, lrs):
                    g["lr"] = lr
            x3.invalidate_packs()

        hist = passes()
        post = x3.range_flag(clear=True)
        pre_set, post_set = self._range_flags(pre, post)
        self.last_update_discarded = bool(pre_set)
        if pre_set:
            restore()
            warnings.warn(f"marlmaze: a {self.gemm_prec} GEMM operand of the rollout reached |x| >= 2^15 (fp16 "
                          "planes): the update on this batch is discarded, and both networks run their GEMMs at "
                          "x3 (bf16x3, fp32 range) from now on")
            self.set_gemm_prec("x3")
            self.range_switched = True
            self.batches_discarded += 1
            hist.fill_(float("nan"))
            return hist
        if post_set:
            restore()
            prec = self.gemm_prec
            self.set_gemm_prec("x3")
            try:
                hist = passes()
            finally:
                self.set_gemm_prec(prec)
            self.range_redos += 1
        return hist

    def train(self):
        for epoch in range(self.epochs):
            b_obs, b_act, b_lp, b_sp, ep_lens, b_masks, b_advs, b_vals = self.get_batch()
            hist = self.update(b_obs, b_act, b_lp, b_masks, b_advs, b_vals)
            if self.last_update_discarded:  # the range guard threw the batch away (now at x3): collect another
                b_obs, b_act, b_lp, b_sp, ep_lens, b_masks, b_advs, b_vals = self.get_batch()
                hist = self.update(b_obs, b_act, b_lp, b_masks, b_advs, b_vals)
            episodes, mean_len, mean_short = self.dp.episode_stats(ep_lens, b_sp)  # all ranks' episodes
            stats = dict(epoch=epoch, episodes=episodes, mean_len=mean_len, mean_shortest=mean_short,
                         actor_loss=float(hist[-1, 0]), critic_loss=float(hist[-1, 1]))
            self.history.append(stats)
            if self.verbose:  # PPO.py:37-44, condensed
                print(f"-------------------- Epoch #{epoch} --------------------")
                print(f"Mazes solved in current epoch: {stats['episodes']}")
                print(f"Average Exit Time: {stats['mean_len']}")
                print(f"Average Length of Shortest Path: {stats['mean_shortest']}", flush=True)
            if self.save and self.dp.rank == 0:
                self.save_parameters()

    # ------------------------------------------------------------------
    # single-sample API of the reference
    # ------------------------------------------------------------------
    @torch.no_grad()
    def get_action(self, obs, action_mask):
        """PPO.get_action (PPO.py:170-186): ([move, mark], log_prob (1,1))."""
        ml, kl = self.actor(obs)
        mk = torch.as_tensor(np.asarray(action_mask, dtype=np.uint8), device=self.device).view(1, 6)
        a, lp, _ = ops.sample(ml, kl.reshape(-1), mk, self.sample_seed, self._sample_offset)
        self._sample_offset += 1
        a = a.cpu().tolist()[0]
        return [a[0], a[1]], lp.view(1, 1)

    def get_log_probs(self, i, batch_obs, batch_actions, batch_masks):
        """PPO.get_log_probs (PPO.py:154-168)."""
        moves, marks = batch_actions[:, i, 0], batch_actions[:, i, 1]
        ml, kl = self.actor(batch_obs[:, i, :])
        ml = ml.masked_fill(~batch_masks[:, i, 0:5], float("-inf"))
        lp = torch.log_softmax(ml, dim=-1).gather(1, moves.long().view(-1, 1)).squeeze(1)
        kl = kl.squeeze(1).masked_fill(~batch_masks[:, i, 5], float("-inf"))
        p = torch.sigmoid(kl)
        p = torch.where(marks.to(torch.bool), p, 1 - p)
        return lp + torch.log(p)

    def get_state_values(self, batch_obs):
        return self.critic(batch_obs).squeeze()

    def get_GAEs(self, ep_rew, ep_values, ep_dones):
        """PPO.get_GAEs (PPO.py:193-203) on the GPU scan; returns a float64 array like the reference."""
        L = len(ep_rew)
        r = torch.as_tensor(np.asarray(ep_rew, np.float32), device=self.device).view(L, 1)
        v = torch.as_tensor(np.asarray([float(x) for x in ep_values], np.float32), device=self.device).view(L, 1)
        d = torch.as_tensor(np.asarray(ep_dones, np.uint8), device=self.device).view(L, 1)
        d[-1] = 1  # the reference's t+1 == L branch ends the episode
        adv, _ = ops.gae(r, v, d, gamma=self.discount_rate, lam=self.lam)
        return adv.view(L).cpu().numpy().astype(np.float64)

    def get_rtgs(self, batch_rew):
        """PPO.get_rtgs (PPO.py:205-214): logging helper, 0.995 discount."""
        rtgs = []
        for episode_rew in reversed(batch_rew):
            acc = 0
            for rew in reversed(episode_rew):
                acc = rew + 0.995 * acc
                rtgs.append(acc)
        rtgs.reverse()
        return rtgs

    def decay_lr(self):
        for opt in (self.actor_optim, self.critic_optim):  # PPO.py:216-220
            for group in opt.param_groups:
                group["lr"] *= 0.997

    def save_parameters(self):
        """PPO.py:222-230: the same four entries; tensors are saved on the CPU so
        the reference (CPU torch) can load the file as it loads its own."""
        def cpu(o):
            if torch.is_tensor(o):
                return o.detach().cpu()
            if isinstance(o, dict):
                return {k: cpu(v) for k, v in o.items()}
            if isinstance(o, (list, tuple)):
                return type(o)(cpu(v) for v in o)
            return o

        torch.save(cpu({"actor": self.actor.state_dict(), "critic": self.critic.state_dict(),
                        "actor_optim": self.actor_optim.state_dict(),
                        "critic_optim": self.critic_optim.state_dict()}), self.model_path)

    def load_optim_state(self, opt, state):
        """Adam.load_state_dict, keeping this build's Adam: a state dict written
        by the reference (CPU torch.optim.Adam) loads into the flat GPU optimizer
        (marlmaze.update.FlatAdam) and back."""
        opt.load_state_dict(state)
        if self.flat is not None:
            x3.invalidate_packs()

    def load_parameters(self):
        if os.path.exists(self.model_path):
            sd = torch.load(self.model_path, weights_only=True, map_location=self.device)
            self.actor.load_state_dict(sd["actor"])
            self.critic.load_state_dict(sd["critic"])
            self.load_optim_state(self.actor_optim, sd["actor_optim"])
            self.load_optim_state(self.critic_optim, sd["critic_optim"])
            if self.verbose:
                print("successfuly loaded existing parameters")
            return True
        return False

