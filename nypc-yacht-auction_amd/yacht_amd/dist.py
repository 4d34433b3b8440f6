"""Multi-GPU Coach: one process per GPU, games sharded by global env id, one RCCL all-gather
of the fixed-size trajectory records into every rank's replay buffer, DDP gradient averaging
for the train step and a summed tally for the gating arena.

Self-play has no cross-game dependency, so the data path needs no collective; the exchanges
are pooling the finished trajectories, the gradient all-reduce of the train step
and three arena counters.  Backend "nccl" is RCCL on ROCm (over xGMI within a node); "gloo"
is used for CPU tests and for rehearsals with ranks sharing one GPU.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist


def setup(backend: str = None):
    """Initialise torch.distributed from torchrun's env (RANK/WORLD_SIZE/LOCAL_RANK/MASTER_*)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and not dist.is_initialized():
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        if backend == "nccl":
            torch.cuda.set_device(local)
        dist.init_process_group(backend=backend)
    return rank, world, local


def rank_world():
    """(rank, world) of the initialised process group, (0, 1) without one."""
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def _group():
    """True when a process group is initialised.  The collectives below short-circuit only
    without one: a group of world size 1 still issues its RCCL call (the one-GPU box's test of
    the code path the 8-GPU run takes)."""
    return dist.is_available() and dist.is_initialized()


def barrier():
    if rank_world()[1] > 1:
        dist.barrier()


def device_index(local: int) -> int:
    """GPU of this rank: one per rank; ranks share the visible GPUs only in gloo rehearsals."""
    n = torch.cuda.device_count()
    return local % n if n else 0


def shard(n_total: int, rank: int, world: int):
    """Equal-size shards of n_total items (the all-gather needs equal images): every rank gets
    c = ceil(n_total / world) slots; rank r owns items [r*c, min(n_total, (r+1)*c))."""
    c = max(-(-n_total // world), 1)
    lo = min(rank * c, n_total)
    return c, lo, min(lo + c, n_total)


def allgather_records(buf: torch.Tensor) -> torch.Tensor:
    """Every rank contributes an equal-size uint8 record image -> [world, nbytes] on all ranks."""
    if not _group():
        return buf.reshape(1, -1)
    world = dist.get_world_size()
    out = torch.empty((world, buf.numel()), dtype=buf.dtype, device=buf.device)
    if dist.get_backend() == "nccl":
        dist.all_gather_into_tensor(out, buf.contiguous())
    else:  # gloo moves host tensors
        host = torch.empty((world, buf.numel()), dtype=buf.dtype)
        dist.all_gather(list(host.unbind(0)), buf.contiguous().cpu())
        out = host.to(buf.device) if buf.is_cuda else host
    return out


def allreduce_grads(trainer, weight: float = None) -> None:
    """DDP gradient averaging for the native trainer: one all-reduce of the flat
    gradient buffer (state_dict order) between yk_trainer_backward and yk_trainer_apply, so
    every rank clips and steps on the same gradient, as torch DDP does.  weight=None: the mean
    of the ranks' gradients; else each rank's gradient is scaled by `weight` (its share of the
    minibatch) and the results summed - the gradient of the whole minibatch when the shares
    are unequal.  RCCL works on the device buffer in place; gloo goes through a host copy."""
    if not _group():
        return
    g = trainer.grads()
    w = dist.get_world_size()
    scale = (1.0 / w) if weight is None else None
    if weight is not None:
        g.mul_(float(weight))
    if dist.get_backend() == "nccl":
        dist.all_reduce(g)
        if scale is not None:
            g.mul_(scale)
    else:
        h = g.cpu()
        dist.all_reduce(h)
        g.copy_(h.mul_(scale) if scale is not None else h)


def allreduce_counts(counts, device=None):
    """Sum of small integer tallies over the ranks (the gating arena's wins / losses / draws)."""
    if not _group():
        return [int(x) for x in counts]
    nccl = dist.get_backend() == "nccl"  # RCCL reduces device tensors only
    t = torch.tensor([int(x) for x in counts], dtype=torch.int64, device=(device or "cuda") if nccl else "cpu")
    dist.all_reduce(t)
    return [int(x) for x in t.cpu().tolist()]


def env_base(rank: int, envs_per_rank: int) -> int:
    """Global env id of this rank's first game: results do not depend on the GPU count."""
    return rank * envs_per_rank


class ReplayBuffer:
    """The pooled replay history (Coach.py:84-101): the last `maxlen_iters` iterations of
    examples, each an ExampleShard built on the device from every rank's record image."""

    def __init__(self, maxlen_iters: int = 5):
        self.shards = []
        self.maxlen = maxlen_iters

    def add_gathered(self, gathered: torch.Tensor, n_envs: int, max_moves: int, sims: int, n_games: int = -1,
                     maxlen_examples: int = None):
        from .replay import examples_from_images
        dev = gathered if gathered.is_cuda else gathered.to("cuda")
        shard = examples_from_images(dev, n_envs, max_moves, sims, n_games=n_games, maxlen=maxlen_examples)
        self.shards.append(shard)
        if len(self.shards) > self.maxlen:
            self.shards.pop(0)
        return shard

    def num_examples(self) -> int:
        return int(sum(len(s) for s in self.shards))

    def device_arrays(self):
        from .replay import as_device_examples
        return as_device_examples(self.shards)
