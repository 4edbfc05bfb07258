"""Part-wise sharding across GPUs: one process per GPU, contiguous part
ranges, no data exchange.  Only the timing/barrier helpers touch torch.distributed."""
from __future__ import annotations

import os
from typing import Tuple


def dist_env() -> Tuple[int, int, int]:
    """(world_size, rank, local_rank) from the torch.distributed.run environment."""
    return (int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")),
            int(os.environ.get("LOCAL_RANK", "0")))


def part_range(n_parts: int, rank: int, world: int) -> Tuple[int, int]:
    """[start, stop) of the contiguous part range owned by `rank` ([g·N/G, (g+1)·N/G))."""
    return n_parts * rank // world, n_parts * (rank + 1) // world


def collective(world: int) -> bool:
    """Whether the rank helpers below go through torch.distributed: world > 1, or a process group
    was initialised at world 1 (bench.py's CEC_BENCH_PG=1 rehearsal of the RCCL branch on one
    GPU)."""
    if world > 1:
        return True
    import torch.distributed as dist
    return dist.is_available() and dist.is_initialized()


def max_over_ranks(x: float, world: int, device=None) -> float:
    """Max of a per-rank float over all ranks (the step time the bench reports)."""
    if not collective(world):
        return x
    import torch
    import torch.distributed as dist
    t = torch.tensor([x], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def gather_rows(row, world: int, device=None):
    """Every rank's `row` (a list of floats of the same length on every rank), in rank order, on
    every rank (a collective: every rank must call it).  A SUM all-reduce of a [world][k] zero
    tensor with each rank's own row filled in, so it works on gloo and on RCCL alike."""
    if not collective(world):
        return [list(map(float, row))]
    import torch
    import torch.distributed as dist
    t = torch.zeros((world, len(row)), dtype=torch.float64, device=device)
    t[dist.get_rank()] = torch.tensor(list(map(float, row)), dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return t.cpu().tolist()


def all_ranks_ok(ok: bool, world: int, device=None) -> bool:
    """True on every rank iff `ok` holds on every rank (a collective: every rank must call it).
    Lets the ranks skip an optional step together when one of them cannot run it, so no rank is
    left waiting in that step's barriers."""
    return -max_over_ranks(-(1.0 if ok else 0.0), world, device) >= 1.0


def barrier(world: int) -> None:
    if collective(world):
        import torch.distributed as dist
        dist.barrier()


def rank_seed(base: int, rank: int) -> int:
    """Synthetic-data seed of a rank's parts (weak scaling: every rank owns distinct parts)."""
    return base + rank


def cpu_quota():
    """CPUs this process may use: (affinity count, cgroup v2 cpu.max quota in CPUs or None)."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            quota = round(int(q) / int(period), 2)
    except (OSError, ValueError):
        pass
    return aff, quota


def quota_share(world: int):
    """One rank's share of the cgroup CPU quota, or None without a quota.  The quota covers the
    whole job -- every rank of the node runs in the same cgroup -- so N ranks split it N ways,
    whatever each rank's affinity (a NUMA node's 128 CPUs on the 2-socket hosts) says."""
    _, quota = cpu_quota()
    return None if quota is None else quota / max(world, 1)


def rank_threads(world: int) -> int:
    """Host copy threads of one rank's reader (the bench's end-to-end and stream legs): half the
    CPUs its main thread may use, 8 at most, and no more than its quota share less one CPU for the
    rank's main thread and the engine's own threads.  CEC_E2E_THREADS overrides."""
    env = int(os.environ.get("CEC_E2E_THREADS", "0"))
    if env:
        return env
    n = max(1, min(8, len(os.sched_getaffinity(0)) // 2))
    share = quota_share(world)
    if share is not None:
        n = max(1, min(n, int(share) - 1))
    return n


def multi_copy_threads(world: int) -> int:
    """Staging copy threads per cec_multi shard (CEC_MULTI_COPY_THREADS; the engine's default is
    4): at N > 1 under a quota, half the rank's share, so the ranks' reader and staging threads
    together stay within the job's CPUs."""
    env = os.environ.get("CEC_MULTI_COPY_THREADS")
    if env:
        return int(env)
    share = quota_share(world)
    if share is None or world <= 1:
        return 4
    return max(1, min(4, int(share) // 2))
