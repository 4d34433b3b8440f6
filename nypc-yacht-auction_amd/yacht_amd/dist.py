"""Multi-GPU self-play: one process per GPU, games sharded by global env id, one RCCL
all-gather of the fixed-size trajectory records into every rank's replay buffer.

Self-play has no cross-game dependency, so the data path needs no collective; the only
exchange is pooling the finished trajectories.  Backend "nccl" is RCCL on
ROCm (over xGMI within a node); "gloo" is used for CPU tests.
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


def device_index(local: int) -> int:
    """GPU of this rank: one per rank; ranks share the visible GPUs only in gloo rehearsals."""
    n = torch.cuda.device_count()
    return local % n if n else 0


def allgather_records(buf: torch.Tensor) -> torch.Tensor:
    """Every rank contributes an equal-size uint8 record image -> [world, nbytes] on all ranks."""
    if not dist.is_initialized() or dist.get_world_size() == 1:
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


def allreduce_grads(trainer) -> None:
    """DDP gradient averaging for the native trainer: one all-reduce of the flat
    gradient buffer (state_dict order) between yk_trainer_backward and yk_trainer_apply, so
    every rank clips and steps on the same mean gradient, as torch DDP does.  RCCL works on the
    device buffer in place; gloo goes through a host copy."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return
    g = trainer.grads()
    w = dist.get_world_size()
    if dist.get_backend() == "nccl":
        dist.all_reduce(g)
        g.div_(w)
    else:
        h = g.cpu()
        dist.all_reduce(h)
        g.copy_(h.div_(w))


def env_base(rank: int, envs_per_rank: int) -> int:
    """Global env id of this rank's first game: results do not depend on the GPU count."""
    return rank * envs_per_rank


class ReplayBuffer:
    """Rank-local replica of the pooled trajectory records (host memory)."""

    def __init__(self, maxlen_batches: int = 5):
        self.batches = []
        self.maxlen = maxlen_batches

    def add_gathered(self, gathered: torch.Tensor, n_envs: int, max_moves: int, sims: int):
        from .engine import unpack_record_image
        host = gathered.cpu().numpy()
        self.batches.append([unpack_record_image(host[r], n_envs, max_moves, sims) for r in range(host.shape[0])])
        if len(self.batches) > self.maxlen:
            self.batches.pop(0)

    def num_examples(self) -> int:
        return int(sum(int(img["n_moves"].sum()) for b in self.batches for img in b))
