"""One process per GPU: env-batch sharding and the episode-summary all-gather.

The reference runs one env per OS process and fans experiments out as independent processes
(gym_cooking/runpara.ps1:44-68); it has no collective.  Here envs are independent, so the
global batch is cut into contiguous shards, one per rank (rank r owns global env ids
[r*B, (r+1)*B)), with NO data-path communication.  The only exchange is a tiny all-gather
of per-GPU episode summaries (OC_NSTATS uint64) once per reporting window -- RCCL over xGMI
on the GPU box (backend "nccl"), gloo in the CPU tests.
"""
from __future__ import annotations

import ctypes
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
    """Initialise the process group from torchrun's env (MASTER_ADDR/PORT, RANK, WORLD_SIZE).

    With backend "nccl" (RCCL over xGMI) the group is created at EVERY world size, world 1
    included: a single-GPU run then issues the same RCCL all-gather / all-reduce calls as an
    8-GPU one (a world-1 communicator; its rendezvous is an in-process store when torchrun did
    not set MASTER_ADDR/PORT: no port to probe, none to lose).  The direct communicator of the
    window's all-gather (RcclComm) is an optimisation of that path: when librccl cannot be
    loaded or the communicator does not come up, the process group's collectives carry the
    all-gather instead (a warning on stderr).  gloo (the CPU tests) only joins a group for
    world > 1."""
    rank, world, local = world_from_env()
    if not dist.is_initialized():
        if backend == "nccl":
            torch.cuda.set_device(local)
            kw = {}
            if "MASTER_ADDR" not in os.environ or "MASTER_PORT" not in os.environ:
                if world != 1:
                    raise RuntimeError("WORLD_SIZE %d without MASTER_ADDR/MASTER_PORT" % world)
                kw = dict(store=dist.HashStore(), rank=0, world_size=1)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local), **kw)
            global _RCCL
            try:
                _RCCL = RcclComm(torch.device("cuda", local))
            except (OSError, RuntimeError, AttributeError) as exc:
                import sys
                print("dist: direct RCCL communicator unavailable (%s); all-gathers go through the process "
                      "group" % exc, file=sys.stderr)
                _RCCL = None
        elif world > 1:
            dist.init_process_group(backend)
    return Shard(rank, world, local, 0, 0)


def rccl_ranks() -> int:
    """Ranks of the RCCL ("nccl") group this process belongs to, 0 without one."""
    if dist.is_initialized() and dist.get_backend() == "nccl":
        return dist.get_world_size()
    return 0


class _UniqueId(ctypes.Structure):
    _fields_ = [("internal", ctypes.c_char * 128)]  # rccl.h NCCL_UNIQUE_ID_BYTES


_NCCL_INT64 = 4  # rccl.h ncclDataType_t


class RcclComm:
    """An RCCL communicator driven through the librccl C API (the library torch loaded), whose
    collectives are enqueued on the caller's HIP stream -- the stream the step launches run on
    -- so the window's summary all-gather follows the last launch in stream order, without the
    cross-stream event record / wait pair torch's process group puts around each collective
    (tools/rccl_window_ab.py).  The unique id is broadcast over the torch "nccl" group, which
    stays for barriers and host-value reductions."""

    def __init__(self, device):
        self.lib = ctypes.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so"))
        self.rank, self.world = dist.get_rank(), dist.get_world_size()
        uid = _UniqueId()
        if self.rank == 0:
            self._check(self.lib.ncclGetUniqueId(ctypes.byref(uid)), "ncclGetUniqueId")
        t = torch.tensor(list(bytes(uid)), dtype=torch.uint8, device=device)  # 128 raw bytes
        dist.broadcast(t, 0)
        ctypes.memmove(ctypes.byref(uid), bytes(t.cpu().tolist()), ctypes.sizeof(uid))
        self.comm = ctypes.c_void_p()
        self._check(self.lib.ncclCommInitRank(ctypes.byref(self.comm), self.world, uid, self.rank),
                    "ncclCommInitRank")
        self.device = device

    def _check(self, rc, what):
        if rc != 0:
            raise RuntimeError("%s failed: ncclResult %d" % (what, rc))

    def all_gather_rows(self, out: torch.Tensor) -> torch.Tensor:
        """In-place all-gather of int64 rows: out is [world, C] and this rank's row out[rank]
        holds its data (RCCL's in-place form, send = recv + rank * C)."""
        C = out.shape[1]
        base = out.data_ptr()
        stream = ctypes.c_void_p(torch.cuda.current_stream(out.device).cuda_stream)
        self._check(self.lib.ncclAllGather(ctypes.c_void_p(base + self.rank * C * 8), ctypes.c_void_p(base),
                                           ctypes.c_size_t(C), _NCCL_INT64, self.comm, stream), "ncclAllGather")
        return out

    def destroy(self):
        if self.comm:
            self.lib.ncclCommDestroy(self.comm)
            self.comm = ctypes.c_void_p()


_RCCL = None


def rccl() -> "RcclComm | None":
    """The direct RCCL communicator init() created (backend "nccl"), else None."""
    return _RCCL


def summary_rows(columns: int, device) -> Tuple[torch.Tensor, torch.Tensor]:
    """(out [world, columns] int64 zeros, this rank's row out[rank]): the buffer
    gather_summaries fills in place."""
    world = dist.get_world_size() if dist.is_initialized() else 1
    rank = dist.get_rank() if dist.is_initialized() else 0
    out = torch.zeros((world, columns), dtype=torch.int64, device=device)
    return out, out[rank]


def shutdown() -> None:
    """Destroy the direct communicator and the process group."""
    global _RCCL
    if _RCCL is not None:
        _RCCL.destroy()
        _RCCL = None
    if dist.is_initialized():
        dist.destroy_process_group()


def device_ident(device) -> torch.Tensor:
    """[3] int64 (PCI domain, bus, device) of this rank's GPU, so that a gathered summary shows
    that N ranks ran on N distinct devices."""
    p = torch.cuda.get_device_properties(device)
    return torch.tensor([p.pci_domain_id, p.pci_bus_id, p.pci_device_id], dtype=torch.int64)


def gather_summaries(totals: torch.Tensor, out: "torch.Tensor | None" = None) -> torch.Tensor:
    """All-gather each rank's summary row (the OC_NSTATS totals, optionally followed by more
    int64 columns such as device_ident) -> [world, columns] (int64).

    With `out` from summary_rows() and `totals` its row out[rank], the gather is in place:
    through the direct RCCL communicator (ncclAllGather on the current stream) when init()
    made one, else through the process group.  Without `out`, the process group's
    all_gather_into_tensor into a new tensor (RCCL at every world size under "nccl")."""
    if out is not None:
        if _RCCL is not None:
            return _RCCL.all_gather_rows(out)
        if dist.is_initialized() and dist.get_world_size() > 1:
            dist.all_gather_into_tensor(out.view(-1), totals)
        return out
    t = totals.to(torch.int64).reshape(-1)
    if not dist.is_initialized() or (dist.get_world_size() == 1 and dist.get_backend() != "nccl"):
        return t.unsqueeze(0)
    out = torch.empty(dist.get_world_size() * t.numel(), dtype=t.dtype, device=t.device)
    dist.all_gather_into_tensor(out, t)
    return out.view(dist.get_world_size(), -1)


def summarize(gathered: torch.Tensor) -> dict:
    """Sum the OC_NSTATS columns over ranks; extra columns 5..7, when present, are each rank's
    device_ident and are listed as per_rank_pci ("domain:bus:device")."""
    g = gathered.cpu().tolist()
    tot = [sum(r[c] for r in g) for c in range(len(STAT_NAMES))]
    out = dict(zip(STAT_NAMES, tot))
    out["per_rank_episodes"] = [r[0] for r in g]
    out["mean_episode_len"] = (tot[2] / tot[0]) if tot[0] else 0.0
    if g and len(g[0]) >= len(STAT_NAMES) + 3:
        n = len(STAT_NAMES)
        out["per_rank_pci"] = ["%04x:%02x:%02x" % (r[n], r[n + 1], r[n + 2]) for r in g]
        out["distinct_devices"] = len(set(out["per_rank_pci"]))
    return out


def max_over_ranks(x: float, device) -> float:
    """Max of a host float over ranks (an all_reduce; under RCCL also at world 1)."""
    if not dist.is_initialized() or (dist.get_world_size() == 1 and dist.get_backend() != "nccl"):
        return x
    t = torch.tensor([x], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def barrier() -> None:
    if dist.is_initialized() and dist.get_world_size() > 1:
        dist.barrier()


def ranks_of(world: int) -> List[int]:
    return list(range(world))
