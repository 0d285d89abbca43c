"""Multi-GPU fit farm: one process per GPU, independent fits, no data collective.

SURVEY.md §8e: the sweep's fits are independent, so the only multi-GPU work
is assigning them to ranks (LPT on the FLOP model) and gathering the small
per-fit result records on the host afterwards.  xGMI/RCCL carry nothing on
the data path; the process group is used for a barrier, a max-reduce of the
elapsed time and an object gather of the records.
"""

from __future__ import annotations

import torch
import torch.distributed as dist

from .engine import lpt_partition


def world() -> tuple:
    if dist.is_available() and dist.is_initialized():
        return dist.get_world_size(), dist.get_rank()
    return 1, 0


def rank_share(costs: list, n_ranks: int, rank: int) -> list:
    """Indices of the fits rank `rank` trains (deterministic on every rank)."""
    if n_ranks <= 1:
        return list(range(len(costs)))
    owner = lpt_partition(costs, n_ranks)
    return [i for i, o in enumerate(owner) if o == rank]


def barrier() -> None:
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    if world()[0] > 1:
        dist.barrier()


def max_over_ranks(x: float) -> float:
    if world()[0] <= 1:
        return float(x)
    dev = "cuda" if dist.get_backend() == "nccl" else "cpu"
    t = torch.tensor([x], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def gather_records(local: dict) -> dict:
    """Union of every rank's {fit index: record} (host-side object gather)."""
    n, _ = world()
    if n <= 1:
        return dict(local)
    parts = [None] * n
    dist.all_gather_object(parts, local)
    out = {}
    for p in parts:
        out.update(p)
    return out
