"""Multi-GPU sharding of the valuation path (one process per GPU).

VAEP features / labels / formula are independent per game: games are split into
contiguous ranges balanced by action count and each rank values its own range with no
collective. xT fit has one exchange step: every rank bins its shard, then the
shot/goal/move vectors and the C x C transition counts are summed with an all-reduce
(RCCL over xGMI with the ``nccl`` backend; ``gloo`` on CPU in tests) and every rank
solves the identical system.
"""
from __future__ import annotations

from typing import List, Tuple

import numpy as np
import torch


def partition_games(game_off: np.ndarray, world: int) -> List[Tuple[int, int]]:
    """Contiguous game ranges [g0, g1) per rank, split at multiples of n / world actions."""
    game_off = np.asarray(game_off, dtype=np.int64)
    G = len(game_off) - 1
    n = int(game_off[-1])
    cuts = [0]
    for r in range(1, world):
        target = n * r // world
        g = int(np.searchsorted(game_off, target, side='left'))
        g = min(max(g, cuts[-1]), G)
        cuts.append(g)
    cuts.append(G)
    return [(cuts[r], cuts[r + 1]) for r in range(world)]


def allreduce_xt_counts(shot: torch.Tensor, goal: torch.Tensor, move: torch.Tensor,
                        trans: torch.Tensor, err: torch.Tensor, group=None) -> None:
    """Sum the xT count buffers over the ranks of ``group`` in place (2 all-reduces + 1 max)."""
    import torch.distributed as dist
    C = shot.numel()
    vec = torch.cat([shot, goal, move])
    dist.all_reduce(vec, group=group)
    dist.all_reduce(trans, group=group)
    dist.all_reduce(err, op=dist.ReduceOp.MAX, group=group)
    shot.copy_(vec[:C])
    goal.copy_(vec[C:2 * C])
    move.copy_(vec[2 * C:])
