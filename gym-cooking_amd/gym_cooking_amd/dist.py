"""One process per GPU: env-batch sharding and the episode-summary all-gather.

The reference runs one env per OS process and fans experiments out as independent processes
(gym_cooking/runpara.ps1:44-68); it has no collective.  Here envs are independent, so the
global batch is cut into contiguous shards, one per rank (rank r owns global env ids
[r*B, (r+1)*B)), with NO data-path communication.  The only exchange is a tiny all-gather
of per-GPU episode summaries (OC_NSTATS uint64) once per reporting window -- RCCL over xGMI
on the GPU box (backend "nccl"), gloo in the CPU tests.
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from typing import List, Tuple

import torch
import torch.distributed as dist

STAT_NAMES = ("episodes", "successes", "steps", "collisions", "errors")


@dataclass
class Shard:
    rank: int
    world: int
    local_rank: int
    env_offset: int   # first global env id of this rank
    batch: int        # envs on this rank


def world_from_env() -> Tuple[int, int, int]:
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def shard(batch_per_rank: int, rank: int, world: int, local_rank: int = 0) -> Shard:
    """Weak scaling: every rank owns `batch_per_rank` envs, contiguous in global id."""
    return Shard(rank, world, local_rank, rank * batch_per_rank, batch_per_rank)


def shard_global(global_batch: int, rank: int, world: int, local_rank: int = 0) -> Shard:
    """Strong scaling split of a fixed global batch (remainder spread over the first ranks)."""
    base, rem = divmod(global_batch, world)
    off = rank * base + min(rank, rem)
    return Shard(rank, world, local_rank, off, base + (1 if rank < rem else 0))


def init(backend: str = "nccl") -> Shard:
    """Initialise the process group from torchrun's env (MASTER_ADDR/PORT, RANK, WORLD_SIZE)."""
    rank, world, local = world_from_env()
    if world > 1 and not dist.is_initialized():
        if backend == "nccl":
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    return Shard(rank, world, local, 0, 0)


def gather_summaries(totals: torch.Tensor) -> torch.Tensor:
    """All-gather each rank's [OC_NSTATS] totals -> [world, OC_NSTATS] (int64)."""
    t = totals.to(torch.int64).reshape(-1)
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return t.unsqueeze(0)
    out = torch.empty(dist.get_world_size() * t.numel(), dtype=t.dtype, device=t.device)
    dist.all_gather_into_tensor(out, t)
    return out.view(dist.get_world_size(), -1)


def summarize(gathered: torch.Tensor) -> dict:
    g = gathered.cpu().tolist()
    tot = [sum(r[c] for r in g) for c in range(len(STAT_NAMES))]
    out = dict(zip(STAT_NAMES, tot))
    out["per_rank_episodes"] = [r[0] for r in g]
    out["mean_episode_len"] = (tot[2] / tot[0]) if tot[0] else 0.0
    return out


def max_over_ranks(x: float, device) -> float:
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return x
    t = torch.tensor([x], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def barrier() -> None:
    if dist.is_initialized() and dist.get_world_size() > 1:
        dist.barrier()


def ranks_of(world: int) -> List[int]:
    return list(range(world))
