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


def allreduce_xt_counts(acc, group=None) -> None:
    """Sum the xT count buffers of ``acc`` (``ops.xt_zero_counts``) over the ranks of ``group``
    in place with ONE all-reduce: the whole allocation -- shot / goal / move (int64), the error
    flags and the C x C transition counts (int32) -- summed as int32 words.  Exact while every
    summed count is below 2**31 (the bound the int32 transition counts already carry, SURVEY
    §8(e)): the int64 counts' high words stay 0 and their low words cannot carry; the error
    flags are one byte each (``ops.XT_ERR_*``), so up to 255 ranks' flags add without
    overlapping.  No staging copy, no ``torch.cat``."""
    _check_world(group)
    _all_reduce(acc.buf.view(torch.int32), group=group)


def _check_world(group) -> None:
    """The counts' int32-word sum keeps the error bytes apart for at most 255 ranks."""
    import torch.distributed as dist
    if dist.get_world_size(group) > 255:
        raise ValueError('the xT count all-reduce sums one error byte per flag: at most 255 ranks')


# ----------------------------------------------------------------------------- collectives
def _on_device(group) -> bool:
    import torch.distributed as dist
    return dist.get_backend(group) == 'nccl'


def _all_reduce(t: torch.Tensor, op=None, group=None) -> None:
    """In-place all-reduce of a device tensor (RCCL; gloo stages through host memory)."""
    import torch.distributed as dist
    op = dist.ReduceOp.SUM if op is None else op
    if _on_device(group):
        dist.all_reduce(t, op=op, group=group)
    else:
        h = t.cpu()
        dist.all_reduce(h, op=op, group=group)
        t.copy_(h)


def _reduce_scatter(out: torch.Tensor, inp: torch.Tensor, group=None) -> None:
    """out = this rank's equal slice of the sum of ``inp`` over ranks."""
    import torch.distributed as dist
    if _on_device(group):
        dist.reduce_scatter_tensor(out, inp, group=group)
    else:  # gloo has no reduce-scatter: all-reduce on the host and keep the slice
        h = inp.cpu()
        dist.all_reduce(h, group=group)
        r = dist.get_rank(group)
        out.copy_(h[r * out.numel():(r + 1) * out.numel()])


def _all_gather(out: torch.Tensor, inp: torch.Tensor, group=None) -> None:
    """out = concatenation of every rank's equal-size ``inp`` (rank order)."""
    import torch.distributed as dist
    if _on_device(group):
        dist.all_gather_into_tensor(out, inp, group=group)
    else:
        parts = [torch.empty_like(inp, device='cpu') for _ in range(dist.get_world_size(group))]
        dist.all_gather(parts, inp.cpu(), group=group)
        out.copy_(torch.cat(parts))


def xt_solve_sharded(acc, eps: float = 1e-5, max_iter: int = 1000, group=None, batch: int = 8):
    """Row-sharded xT fit over the ranks of ``group``: each rank passes
    its OWN shard's counts (``ops.xt_zero_counts(..., row_blocks=world)`` + ``ops.xt_count``).

    1. one all-reduce of the shot / goal / move vectors (3 x C int64) and the error flags (the
       head of the count allocation, summed as int32 words like ``allreduce_xt_counts``);
    2. reduce-scatter of the C x C transition counts by row blocks: rank r keeps the summed
       count rows [r*B, (r+1)*B), B = ceil(C / world) (half the traffic of an all-reduce);
    3. per iteration, each rank updates its B rows (``sa_xt_iterate_compact`` over the compact
       form of its rows built once, ``sa_xt_iterate_rows`` above 10240 cells; the reference's
       summation order, so every value is bit-identical to the single-GPU solve) into one
       persistent B-row buffer, and one all-gather of those buffers rebuilds the full x on
       every rank;
    4. convergence flags are combined (max) every ``batch`` iterations; iterations past the
       first converged one are computed and discarded.

    Returns ``(mats [4, C] = scoring | shot | move | xT, heatmaps [n_iter + 1, C], n_iter)``;
    the normalised C x C transition matrix is never materialised on this path.
    """
    import ctypes

    import torch.distributed as dist

    from . import _native
    from .batch import stream_handle
    _check_world(group)
    W = dist.get_world_size(group)
    r = dist.get_rank(group)
    C = acc.C
    B = -(-C // W)
    dev = acc.shot.device
    if acc.trans_padded.numel() != W * B * C:
        raise ValueError('counts must be allocated with xt_zero_counts(..., row_blocks=world)')
    _all_reduce(acc.head.view(torch.int32), group=group)  # the vectors + flags: one all-reduce
    shot, goal, move = acc.shot, acc.goal, acc.move
    rows = torch.empty(B * C, dtype=torch.int32, device=dev)
    _reduce_scatter(rows, acc.trans_padded, group=group)
    lib = _native.lib()
    mats = torch.empty((4, C), dtype=torch.float64, device=dev)
    gp = torch.empty((2, C), dtype=torch.float64, device=dev)
    ptr = lambda t: t.data_ptr()  # noqa: E731
    _native.check(lib.sa_xt_probabilities(ptr(shot), ptr(goal), ptr(move), C, ptr(mats),
                                           ptr(gp[0]), ptr(gp[1]), stream_handle()))
    heat = torch.zeros((max_iter + 1, W * B), dtype=torch.float64, device=dev)
    flags = torch.zeros(max_iter + 1, dtype=torch.int32, device=dev)
    r0 = r * B
    nrows = max(0, min(B, C - r0))
    mine = torch.zeros(B, dtype=torch.float64, device=dev)  # this rank's rows, all-gathered
    # the compact form of this rank's count rows, built once (sa_xt_compact_rows)
    compact = C <= _native.SA_XT_COMPACT_MAX_C
    if compact:
        ell = torch.empty(max(int(lib.sa_xt_compact_bytes(C, nrows)) // 4, 4), dtype=torch.int32,
                          device=dev)
        slen = torch.empty(max(-(-nrows // 32), 1), dtype=torch.int32, device=dev)
        _native.check(lib.sa_xt_compact_rows(ptr(rows), C, nrows, ptr(ell), ptr(slen),
                                             stream_handle()))
    iters = -1
    it0 = 0
    while it0 < max_iter and iters < 0:
        it1 = min(it0 + batch, max_iter)
        for it in range(it0, it1):
            if compact:
                _native.check(lib.sa_xt_iterate_compact(
                    ptr(ell), ptr(slen), ptr(rows), ptr(move), ptr(gp[0]), ptr(gp[1]), C,
                    min(r0, C), nrows, ptr(heat[it]), float(eps), ptr(mine), None,
                    ptr(flags[it:]), stream_handle()))
            else:
                _native.check(lib.sa_xt_iterate_rows(
                    ptr(rows), ptr(move), ptr(gp[0]), ptr(gp[1]), C, min(r0, C), nrows,
                    ptr(heat[it]), float(eps), ptr(mine), None, ptr(flags[it:]),
                    stream_handle()))
            _all_gather(heat[it + 1], mine, group=group)
        f = flags[it0:it1]
        _all_reduce(f, dist.ReduceOp.MAX, group=group)
        hf = f.cpu().numpy()
        done = np.flatnonzero(hf == 0)
        if len(done):
            iters = it0 + int(done[0]) + 1
        it0 = it1
    if iters < 0:
        raise RuntimeError(f'xT value iteration did not converge within {max_iter} iterations')
    mats[3].copy_(heat[iters, :C])
    return mats, heat[:iters + 1, :C], iters
