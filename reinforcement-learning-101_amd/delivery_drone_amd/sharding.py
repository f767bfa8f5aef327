"""Sharding of one global drone batch over the GPUs of a node.

Drones never interact (game_engine.py:95-138 touches only its own drone and
platform), so the batch splits into contiguous blocks of global env ids, one
block per rank, with no collective on the step path.  Spawn draws are keyed
by the global id, so a drone's episodes do not depend on the world size.
The only optional exchange is gathering observations to one rank
(:func:`gather_obs`), over RCCL (backend ``"nccl"``) on the GPUs or gloo on
the CPU.
"""
from __future__ import annotations

import math
import os
from typing import Dict, List, Optional, Tuple

import torch
import torch.distributed as dist

__all__ = ["shard_bounds", "dist_env", "gather_obs", "gather_state"]


def shard_bounds(total: int, rank: int, world: int) -> Tuple[int, int]:
    """(first global id, count) of ``rank``'s block; the first ``total % world``
    ranks hold one extra drone."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError(f"bad rank/world {rank}/{world}")
    if total < 0:
        raise ValueError("total must be >= 0")
    base, extra = divmod(total, world)
    start = rank * base + min(rank, extra)
    return start, base + (1 if rank < extra else 0)


def dist_env() -> Tuple[int, int, int]:
    """(rank, world_size, local_rank) from the torchrun environment (1 process: 0, 1, 0)."""
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    return rank, world, local


def gather_obs(obs: torch.Tensor, total: int, dst: int = 0, group=None) -> Optional[torch.Tensor]:
    """Gather every rank's observation block ``[count_r, 15]`` into one
    ``[total, 15]`` tensor on rank ``dst`` (None elsewhere).

    Blocks are padded to the largest shard so a single ``gather`` call moves
    them (one xGMI transfer per peer with RCCL)."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    counts = [shard_bounds(total, r, world)[1] for r in range(world)]
    if obs.shape[0] != counts[rank]:
        raise ValueError(f"rank {rank} holds {obs.shape[0]} rows, its shard is {counts[rank]}")
    width = max(counts) if counts else 0
    padded = obs.new_zeros((width,) + tuple(obs.shape[1:]))
    padded[: obs.shape[0]] = obs
    gathered: Optional[List[torch.Tensor]] = None
    if rank == dst:
        gathered = [torch.empty_like(padded) for _ in range(world)]
    dist.gather(padded, gather_list=gathered, dst=dst, group=group)
    if rank != dst:
        return None
    return torch.cat([g[:c] for g, c in zip(gathered, counts)], dim=0)


def gather_state(fields: Dict[str, torch.Tensor], total: int, dst: int = 0, group=None) -> Optional[Dict[str, torch.Tensor]]:
    """Gather per-drone tensors (each ``[count_r]`` or ``[count_r, k]``: the
    SoA state fields, a frame's reward / done) from every rank to rank
    ``dst`` as ``[total, ...]`` tensors in global env-id order (None on the
    other ranks).  Fields of one dtype travel packed as the columns of one
    block, so the exchange is one :func:`gather_obs` per dtype, not per
    field: the consumer-side twin of the step path's shards (checkpoints,
    a learner that needs the whole batch)."""
    groups: Dict[torch.dtype, List[str]] = {}
    for name in sorted(fields):  # the same column order on every rank, whatever the dict order
        groups.setdefault(fields[name].dtype, []).append(name)
    out: Dict[str, torch.Tensor] = {}
    for dtype in sorted(groups, key=str):
        names = groups[dtype]
        # reshape(count, prod(rest)), not (count, -1): a rank may hold zero rows
        cols = [fields[n].reshape(fields[n].shape[0], math.prod(fields[n].shape[1:])) for n in names]
        widths = [c.shape[1] for c in cols]
        g = gather_obs(torch.cat(cols, dim=1), total, dst=dst, group=group)
        if g is None:
            continue
        for n, piece in zip(names, torch.split(g, widths, dim=1)):
            out[n] = piece.reshape((total,) + tuple(fields[n].shape[1:]))
    return out if dist.get_rank(group) == dst else None
