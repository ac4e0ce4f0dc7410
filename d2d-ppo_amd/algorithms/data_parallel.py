"""Data parallelism over env shards (one process per GPU, torch.distributed;
backend "nccl" = RCCL over xGMI on MI355X).

The reference is single-process (no collectives).  Here each
rank owns a contiguous shard of the env batch (its own Philox counter range,
env_base = rank * n_envs) and runs rollouts with no communication.  The only
exchanges per PPO epoch are:
  1. the normalisation statistics of advantages / returns (column sums, then
     centred sums of squares; float64, <= a few KB) so every rank normalises
     with the GLOBAL mean/std, exactly as one big rollout would;
  2. ONE flattened fp32 gradient bucket per optimizer (all N actors, all
     critics): all-reduce SUM / world.  Shards are equal-sized and every loss
     is a per-agent batch mean, so the averaged gradient is the full-batch
     gradient (up to summation order).  Gradient clipping (D2D, norm 20) runs
     after the all-reduce, identically on every rank.
  3. D2D's agent permutation is broadcast from rank 0 (every rank normally
     draws the same one from identically seeded numpy streams anyway).
Initial weights are broadcast from rank 0 once.
"""
import numpy as np
import torch
import torch.distributed as dist
from torch._utils import _flatten_dense_tensors, _unflatten_dense_tensors


def world():
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def allreduce_grads_(params, group=None):
    """Average the .grad of `params` over ranks with one bucketed all-reduce."""
    params = [p for p in params if p.grad is not None]
    if not params:
        return
    ws = dist.get_world_size(group)
    grads = [p.grad for p in params]
    flat = _flatten_dense_tensors(grads)
    dist.all_reduce(flat, group=group)
    flat.div_(ws)
    for g, r in zip(grads, _unflatten_dense_tensors(flat, grads)):
        g.copy_(r)


def broadcast_params_(params, src=0, group=None):
    with torch.no_grad():
        for p in params:
            dist.broadcast(p.data, src=src, group=group)


def broadcast_perm(perm, device, src=0, group=None):
    t = torch.as_tensor(np.asarray(perm, dtype=np.int64), device=device)
    dist.broadcast(t, src=src, group=group)
    return t.cpu().numpy()


def allreduce_mean_scalar(x, device, group=None):
    t = torch.tensor([float(x)], dtype=torch.float64, device=device)
    dist.all_reduce(t, group=group)
    return float(t.item()) / dist.get_world_size(group)


class DataParallelMixin:
    """Hooks used by BatchedLearnerBase when torch.distributed is initialised."""

    def _setup_data_parallel(self, params):
        self.rank, self.world_size = world()
        if self.world_size == 1:
            return
        self.process_group = dist.group.WORLD
        env = self.env
        want = self.rank * env.n_envs
        err = None
        if getattr(env, "_batch", None) is None:
            if getattr(env, "env_base", 0) not in (0, want):
                err = f"env was sharded with env_base {env.env_base}, expected {want} (= rank * n_envs)"
            else:
                env.shard(self.rank, self.world_size)
        elif env._batch.desc.env_base != want:
            # an env batch built before the learner (e.g. by env.reset()) draws the Philox streams of
            # envs [env_base, env_base + n_envs): unsharded, every rank would roll out identical
            # episodes and the all-reduced gradient would be one rank's gradient
            err = (f"the env batch already exists with env_base {env._batch.desc.env_base}; call "
                   f"env.shard({self.rank}, {self.world_size}) before the first reset, or build the "
                   f"learner before using the env")
        # every rank learns whether any rank is misconfigured, so all of them raise (no rank is left
        # waiting in the weight broadcast below)
        bad = torch.tensor([0 if err is None else 1], dtype=torch.int64,
                           device=self.device if dist.get_backend(self.process_group) == "nccl" else "cpu")
        dist.all_reduce(bad, group=self.process_group)
        if int(bad.item()):
            raise RuntimeError(f"rank {self.rank}: " + (err or "another rank's env is not sharded for it"))
        broadcast_params_(params, 0, self.process_group)

    def _reduce_grads(self, params):
        if getattr(self, "world_size", 1) > 1:
            allreduce_grads_(params, self.process_group)

    def _last_shard(self):
        return getattr(self, "rank", 0) == getattr(self, "world_size", 1) - 1

    def _n_envs_total(self):
        ws = getattr(self, "world_size", 1)
        return None if ws == 1 else self.env.n_envs * ws

    def _sync_perm(self, perm):
        if getattr(self, "world_size", 1) > 1:
            return broadcast_perm(perm, self.device, 0, self.process_group)
        return perm
