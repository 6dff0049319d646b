"""Data parallelism for the PPO hot path: one process per GPU, torch.distributed.

The reference is single-process (no collectives).  Mazes are
independent, so rollout and GAE need no communication; the exchange steps are
(SURVEY §8(e)):

1. advantage normalisation (PPO.py:47): one all-reduce of {sum A, sum A^2, n}
   in fp64, so mean and the unbiased std are global;
2. one all-reduce of a single flat fp32 bucket holding every actor AND critic
   gradient per minibatch step (278,383 params = 1.11 MB) before clipping, so
   the clipped global norm is identical on every rank.  On the GPU the bucket IS
   the gradient storage (marlmaze.update.FlatParams: no gather or scatter) and
   the 1 / world average is applied inside the optimizer kernel;
3. per-epoch statistics (episodes finished, their lengths and shortest
   paths: three fp64 sums, ``episode_stats``);
4. the x2 / f16 range guard's two flags per update (``allreduce_max``), so the
   decision to redo an update at x3, or to discard a batch, is the same on
   every rank.

Backend "nccl" is RCCL on ROCm (xGMI inside the node); "gloo" for CPU tests.
"""
import os

import torch
import torch.distributed as dist


class DP:
    """World handle.  ``DP.single()`` is the no-communication case."""

    def __init__(self, rank=0, world=1, group=None):
        self.rank = rank
        self.world = world
        self.group = group
        self._flat = None

    @staticmethod
    def single():
        return DP(0, 1)

    @staticmethod
    def from_env(backend=None):
        """torchrun-style env (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR /
        MASTER_PORT).  Binds the process to GPU ``LOCAL_RANK`` (modulo the
        visible devices, so a gloo rehearsal may put several ranks on one GPU)
        BEFORE the process group exists, and hands that device to RCCL, so the
        communicator, ``PPO``'s default device and every barrier agree."""
        world = int(os.environ.get("WORLD_SIZE", "1"))
        if world <= 1:
            return DP.single()
        local = int(os.environ.get("LOCAL_RANK", os.environ.get("RANK", "0")))
        dev = None
        if torch.cuda.is_available():
            dev = torch.device("cuda", local % torch.cuda.device_count())
            torch.cuda.set_device(dev)
        if not dist.is_initialized():
            if backend is None:
                backend = "nccl" if dev is not None else "gloo"
            if backend == "nccl":
                dist.init_process_group(backend=backend, device_id=dev)
            else:
                dist.init_process_group(backend=backend)
        return DP(dist.get_rank(), dist.get_world_size())

    @property
    def active(self):
        return self.world > 1

    def broadcast_params(self, modules):
        if not self.active:
            return
        with torch.no_grad():
            for m in modules:
                for p in m.parameters():
                    dist.broadcast(p.data, src=0)

    def broadcast_tensor(self, t):
        """Rank 0's t on every rank (the flat parameter buffer: one collective)."""
        if self.active:
            dist.broadcast(t, src=0)

    def allreduce_grads(self, params):
        """Average the gradients of ``params`` across ranks in ONE flat bucket."""
        if not self.active:
            return
        grads = [p.grad for p in params]
        n = sum(g.numel() for g in grads)
        if self._flat is None or self._flat.numel() != n or self._flat.device != grads[0].device:
            self._flat = torch.empty(n, dtype=grads[0].dtype, device=grads[0].device)
        flat = self._flat
        torch.cat([g.reshape(-1) for g in grads], out=flat)
        dist.all_reduce(flat, op=dist.ReduceOp.SUM)
        flat.mul_(1.0 / self.world)
        off = 0  # the averaged gradients ARE the bucket: each .grad becomes a view of it (no copy back)
        for p, g in zip(params, grads):
            k = g.numel()
            p.grad = flat[off:off + k].view_as(g)
            off += k

    def global_mean_std(self, x):
        """torch.mean / unbiased torch.std over the union of every rank's x (PPO.py:47)."""
        if not self.active:
            return torch.mean(x), torch.std(x)
        xd = x.double()
        s = torch.stack([xd.sum(), (xd * xd).sum(), torch.tensor(float(x.numel()), dtype=torch.float64,
                                                                  device=x.device)])
        dist.all_reduce(s, op=dist.ReduceOp.SUM)
        tot, sq, n = s[0], s[1], s[2]
        mean = tot / n
        var = (sq - n * mean * mean) / (n - 1)
        return mean.to(x.dtype), var.clamp_min(0).sqrt().to(x.dtype)

    def episode_stats(self, ep_lens, shortest):
        """(episodes, mean exit time, mean shortest path) over every rank's
        finished episodes (the figures PPO.py:37-44 prints)."""
        s = torch.tensor([float(len(ep_lens)), float(sum(ep_lens)), float(sum(shortest))], dtype=torch.float64)
        if self.active:
            dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" else "cpu"
            s = s.to(dev)
            dist.all_reduce(s, op=dist.ReduceOp.SUM)
            s = s.cpu()
        n = int(s[0])
        return n, (float(s[1]) / n if n else 0.0), (float(s[2]) / n if n else 0.0)

    def allreduce_sum(self, t):
        if self.active:
            dist.all_reduce(t, op=dist.ReduceOp.SUM)
        return t

    def allreduce_max(self, t):
        """In place: the element-wise maximum over ranks (the x2 range guard's flags: a flag raised on any
        rank is raised on every rank, so all ranks take the same branch and issue the same collectives)."""
        if self.active:
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return t

    def barrier(self):
        if self.active:
            dist.barrier()
