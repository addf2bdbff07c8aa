"""Multi-GPU plumbing around liblbm (one process per GPU): z-slab planning, RCCL unique-id
hand-out and the max/sum-over-ranks reductions bench.py reports with.  Everything here runs
on a CPU process group (gloo), so the same code is exercised by the CPU tests; the data
path itself (halo exchange, residual all-reduce) is RCCL inside liblbm (lbm_attach_rccl).
"""
from __future__ import annotations

from typing import Callable, Sequence

import torch
import torch.distributed as dist

from .cases import slab_bounds


def slab_plan(nz_global: int, world: int):
    """[(z0, z1)] per rank: an even z split, remainder to the lowest ranks (every rank >= 1 plane)."""
    if world < 1 or nz_global < world:
        raise ValueError(f"cannot split {nz_global} planes over {world} ranks")
    return [slab_bounds(nz_global, world, r) for r in range(world)]


def share_unique_id(rank: int, group, make_id: Callable[[], bytes]) -> bytes:
    """Rank 0 creates the 128-byte communicator id (lbm_rccl_unique_id), everyone receives it."""
    obj = [make_id() if rank == 0 else None]
    dist.broadcast_object_list(obj, src=0, group=group)
    uid = obj[0]
    if not isinstance(uid, (bytes, bytearray)) or len(uid) != 128:
        raise ValueError("unique id must be 128 bytes")
    return bytes(uid)


def max_over_ranks(values: Sequence[float], group) -> list:
    t = torch.tensor(list(values), dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return [float(v) for v in t]


def sum_over_ranks(values: Sequence[float], group) -> list:
    t = torch.tensor(list(values), dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    return [float(v) for v in t]
