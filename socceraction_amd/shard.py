"""Multi-GPU sharding of the valuation path (one process per GPU).

VAEP features / labels / formula are independent per game: games are split into
contiguous ranges balanced by action count and each rank values its own range with no
collective. xT fit has one exchange step: every rank bins its shard, then the
shot/goal/move vectors and the C x C transition counts are summed with an all-reduce
(RCCL over xGMI with the ``nccl`` backend; ``gloo`` on CPU in tests) and every rank
solves the identical system.
"""
from __future__ import annotations

import contextlib
import time
from typing import List, Tuple

import numpy as np
import torch


class PhaseTimes:
    """Per-phase times of a multi-rank fit (its exchange steps and kernels): a HIP event pair on
    torch's current stream around each phase on a GPU (the collectives' device work is ordered
    on that stream: RCCL's calls make it wait for them), the wall clock on the host otherwise
    (gloo on CPU tensors).  ``ms()`` synchronises once and sums each phase's pairs."""

    def __init__(self, device=None):
        dev = torch.device(device) if device is not None else None
        self.cuda = dev is not None and dev.type == 'cuda'
        self.ev = {}
        self.wall = {}

    @contextlib.contextmanager
    def phase(self, name: str):
        if self.cuda:
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            yield
            b.record()
            self.ev.setdefault(name, []).append((a, b))
        else:
            t0 = time.perf_counter()
            yield
            self.wall[name] = self.wall.get(name, 0.0) + (time.perf_counter() - t0) * 1e3

    def ms(self) -> dict:
        if self.cuda:
            torch.cuda.synchronize()
        out = {k: sum(a.elapsed_time(b) for a, b in v) for k, v in self.ev.items()}
        out.update(self.wall)
        return {k: round(v, 3) for k, v in out.items()}


def _phase(stats, name: str):
    """``stats['timer'].phase(name)`` when the caller passed a :class:`PhaseTimes`, else a no-op."""
    t = stats.get('timer') if stats is not None else None
    return t.phase(name) if t is not None else contextlib.nullcontext()


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
    if not getattr(acc, 'dense', True):  # every rank would raise alike (the same call on each)
        acc.require_dense('allreduce_xt_counts')
    _flag_count_range(acc, group)
    acc.compact = None  # this rank's compact rows no longer describe the summed counts
    _all_reduce(acc.buf.view(torch.int32), group=group)


def _flag_count_range(acc, group) -> None:
    """The int32-word sum is exact while every summed count stays below 2**31: each rank's shot
    and move counts below 2**31 // world guarantee it (a transition count never exceeds its
    row's move count, a goal count its shot count).  A rank over that bound sets the overflow
    byte of the error word (``ops.XT_ERR_OVERFLOW``, raised by ``ops.xt_check_errors``) on the
    device, before the all-reduce: no host round trip."""
    import torch.distributed as dist

    from .ops import XT_ERR_OVERFLOW
    bound = (2 ** 31) // dist.get_world_size(group)
    big = torch.maximum(acc.shot.max(), acc.move.max()) >= bound
    acc.err.add_(big.to(torch.int32) * (XT_ERR_OVERFLOW & -XT_ERR_OVERFLOW))


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


def _all_to_all(out: torch.Tensor, inp: torch.Tensor, out_splits=None, in_splits=None,
                group=None) -> None:
    """out = the concatenation over ranks q of the part of q's ``inp`` meant for this rank
    (``in_splits`` / ``out_splits``: element counts per rank; None: equal parts)."""
    import torch.distributed as dist
    if out.dtype == torch.int16:  # neither RCCL nor gloo takes int16: move the bytes
        sz = lambda sp: None if sp is None else [2 * int(x) for x in sp]  # noqa: E731
        return _all_to_all(out.view(torch.uint8), inp.contiguous().view(torch.uint8),
                           sz(out_splits), sz(in_splits), group)
    if _on_device(group):
        dist.all_to_all_single(out, inp, out_splits, in_splits, group=group)
    else:
        h = torch.empty(out.shape, dtype=out.dtype)
        dist.all_to_all_single(h, inp.cpu(), out_splits, in_splits, group=group)
        out.copy_(h)


def _to_host(t: torch.Tensor, stats=None) -> np.ndarray:
    """The one place the exchange reads device values on the host (a stream synchronisation);
    ``stats['host_reads']`` counts them."""
    if stats is not None:
        stats['host_reads'] = stats.get('host_reads', 0) + 1
    return t.cpu().numpy()


def band_ranges(n_bands: int, world: int) -> List[Tuple[int, int]]:
    """Bands [b0, b1) owned by each rank in the band-sharded fit: ceil(NB / world) consecutive
    bands per rank (the last ranks may own fewer, or none)."""
    per = -(-n_bands // world)
    return [(min(n_bands, q * per), min(n_bands, (q + 1) * per)) for q in range(world)]


def xt_solve_sharded(acc, eps: float = 1e-5, max_iter: int = 1000, group=None, batch: int = 8):
    """Row-sharded xT fit over the ranks of ``group``: each rank passes
    its OWN shard's counts (``ops.xt_zero_counts(..., row_blocks=world)`` + ``ops.xt_count``).

    1. one all-reduce of the shot / goal / move vectors (3 x C int64) and the error flags (the
       head of the count allocation, summed as int32 words like ``allreduce_xt_counts``);
    2. reduce-scatter of the C x C transition counts by row blocks: rank r keeps the summed
       count rows [r*B, (r+1)*B), B = ceil(C / world) (half the traffic of an all-reduce);
    3. per iteration, each rank updates its B rows (``sa_xt_iterate_compact`` over the compact
       form of its rows built once, ``sa_xt_iterate_rows`` above 9472 cells; the reference's
       summation order, so every value is bit-identical to the single-GPU solve) into one
       persistent B-row buffer, and one all-gather of those buffers rebuilds the full x on
       every rank;
    4. convergence flags are combined (max) every ``batch`` iterations; iterations past the
       first converged one are computed and discarded.

    Returns ``(mats [4, C] = scoring | shot | move | xT, heatmaps [n_iter + 1, C], n_iter)``;
    the normalised C x C transition matrix is never materialised on this path.
    """
    import torch.distributed as dist
    _check_world(group)
    W = dist.get_world_size(group)
    r = dist.get_rank(group)
    C = acc.C
    B = -(-C // W)
    dev = acc.shot.device
    if acc.trans_padded.numel() != W * B * C:
        raise ValueError('counts must be allocated with xt_zero_counts(..., row_blocks=world)')
    _flag_count_range(acc, group)
    _all_reduce(acc.head.view(torch.int32), group=group)  # the vectors + flags: one all-reduce
    shot, goal, move = acc.shot, acc.goal, acc.move
    rows = torch.empty(B * C, dtype=torch.int32, device=dev)
    _reduce_scatter(rows, acc.trans_padded, group=group)
    return _solve_row_block(rows, shot, goal, move, C, B, eps, max_iter, group, batch)


def _solve_row_block(rows, shot, goal, move, C: int, B: int, eps: float, max_iter: int, group,
                     batch: int):
    """The row-sharded value iteration: this rank holds the summed count rows [r B, r B + B)
    (``rows``, B x C int32) and the full shot / goal / move vectors."""
    import torch.distributed as dist

    from . import _native
    from .batch import stream_handle
    W = dist.get_world_size(group)
    r = dist.get_rank(group)
    dev = rows.device
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
        slen = torch.empty(max(nrows, 1), dtype=torch.int32, device=dev)  # row lengths
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


def xt_fit_bands_sharded(batches, l: int, w: int, eps: float = 1e-5, max_iter: int = 1000,
                         group=None, batch: int = 8, interp_codes=None, solve: str = 'compact',
                         exact_order: bool = False, stats=None):
    """Band-sharded xT fit (cfg5 over several GPUs) for grids the band-owned count holds
    (``ops.xt_band_shape``, e.g. 105 x 68): the ranks exchange their COUNTED ACTIONS, not count
    tables.  Rank r owns the start-cell bands [b0, b1) = ``band_ranges(NB, world)[r]``, i.e.
    the count rows [b0 R, b1 R).

    1. every rank buckets its own batches (``sa_xt_count_bucket``: one 16-bit key per counted
       action -- its bin in its band's histogram -- sorted by band, so each destination's keys
       are one contiguous range);
    2. one all-to-all of the keys (about 1.7 B per action: ~19 MB per rank at 1e8 actions over 8
       ranks, against 204 MB x 2 (W-1) / W for the table's all-reduce) and one of the band offsets;
    3. each rank counts its own bands from every rank's keys (``sa_xt_count_band_rows``: the B x C
       rows written once from LDS, no global atomics) -- the same row block the reduce-scatter of
       ``xt_solve_sharded`` would leave it;
    4. one all-gather of the shot / goal / move counts of every rank's rows and a max all-reduce
       of the error flags;
    5. ``solve='compact'`` (default): each rank builds the compact form of its rows
       (``sa_xt_compact_rows``), one all-gather of those rows' non-zero entries (62.5 MB in all at
       cfg5) gives every rank the whole compact form, and every rank iterates all rows with no
       further exchange (``_solve_compact_exchange``: the single-GPU fit's own solve,
       ``sa_xt_solve_compact``, reordered sums under the error bound unless ``exact_order``;
       falls back to 'rows' when some count reaches 65535: escaped entries are read from the
       dense row, which only its owner holds); ``solve='rows'``: the row-sharded value
       iteration of ``xt_solve_sharded`` (the reference's order, one all-gather of x per
       iteration).  Either way every value is bit-identical to the single-GPU fit of all ranks'
       actions with the same ``exact_order`` ('rows': ``exact_order=True``).

    ``interp_codes``: one ``ops.xt_interp_codes_buffer`` per batch, filled for the rate.
    ``stats`` (dict, optional) receives the exchange's kind, bytes and host reads.
    Returns ``(mats [4, C], heatmaps [n_iter + 1, C], n_iter, err)``; ``err`` is the error-flag
    word of ``sa_xt_count`` (check with ``ops.xt_check_errors(types.SimpleNamespace(err=err))``).
    """
    import ctypes

    import torch.distributed as dist

    from . import _native, ops
    from .batch import stream_handle
    _check_world(group)
    shape = ops.xt_band_shape(l, w)
    if shape is None:
        raise ValueError(f'the band-owned count does not take a {l} x {w} grid')
    R, NB = shape
    C = l * w
    W = dist.get_world_size(group)
    r = dist.get_rank(group)
    ranges = band_ranges(NB, W)
    per = -(-NB // W)  # bands per rank (equal row blocks for the iteration's all-gather)
    B = per * R
    b0, b1 = ranges[r]
    dev = batches[0].device if batches else torch.device('cuda', torch.cuda.current_device())
    err = torch.zeros(1, dtype=torch.int32, device=dev)
    ic = list(interp_codes) if interp_codes is not None else [None] * len(batches)
    with _phase(stats, 'bucket'):  # K1 - K3 of this rank's batches
        parts = [ops.xt_bucket(b, l, w, err, interp_codes=c) for b, c in zip(batches, ic)]
    with _phase(stats, 'key_all_to_all'):  # headers (one host read), keys, band offsets
        sets_keys, sets_off = exchange_band_keys([(p.keys, p.band_off) for p in parts], NB, group,
                                                 dev, stats)
    nb = b1 - b0
    with _phase(stats, 'band_count'):  # K4 of this rank's bands
        rows = torch.zeros(B * C, dtype=torch.int32, device=dev)
        vec = torch.zeros((3, B), dtype=torch.int64, device=dev)
        kp = (ctypes.c_void_p * len(sets_keys))(*[t.data_ptr() for t in sets_keys])
        op = (ctypes.c_void_p * len(sets_off))(*[t.data_ptr() for t in sets_off])
        _native.check(_native.lib().sa_xt_count_band_rows(
            len(sets_keys), kp, op, l, w, b0, nb, vec[0].data_ptr(), vec[1].data_ptr(),
            vec[2].data_ptr(), rows.data_ptr(), _native.SA_XT_COUNT_OVERWRITE, stream_handle()))
    with _phase(stats, 'vector_all_gather'):  # shot / goal / move of every row, the error word
        allv = torch.empty((W, 3, B), dtype=torch.int64, device=dev)
        _all_gather(allv.reshape(-1), vec.reshape(-1), group=group)
        full = allv.permute(1, 0, 2).reshape(3, W * B)[:, :C].contiguous()
        # the error bytes of every rank: summed, one byte per flag, like allreduce_xt_counts (a
        # MAX of whole words would drop one rank's lower-byte flag behind another's higher one)
        _all_reduce(err, group=group)
    if solve not in ('compact', 'rows'):
        raise ValueError("solve must be 'compact' or 'rows'")
    res = None
    if solve == 'compact' and C <= _native.SA_XT_COMPACT_MAX_C:
        res = _solve_compact_exchange(rows, full[0], full[1], full[2], C, B, eps, max_iter, group,
                                      exact_order, stats)
        if stats is not None:
            stats['exchange'] = ('all-to-all of counted actions + all-gather of compact rows'
                                 if res is not None else
                                 'all-to-all of counted actions (escaped counts: row-sharded '
                                 'iteration, all-gather of x per iteration)')
    if res is None:
        if stats is not None:
            stats['solve_path'] = 'sequential'
        if stats is not None and solve == 'rows':
            stats['exchange'] = 'all-to-all of counted actions + all-gather of x per iteration'
        with _phase(stats, 'row_sharded_solve'):  # incl. an all-gather of x per iteration
            res = _solve_row_block(rows, full[0], full[1], full[2], C, B, eps, max_iter, group,
                                   batch)
    mats, heat, iters = res
    return mats, heat, iters, err


def pack_compact_rows(ell: torch.Tensor, row_chunks: torch.Tensor, pe: int,
                      total: int) -> torch.Tensor:
    """The used 128-slot chunks of compact rows (``sa_xt_compact_rows`` layout: row i at
    ``ell[i * pe:]``, ``row_chunks[i]`` = ceil(len_i / 128) chunks used), packed in row order:
    ``total`` (= row_chunks.sum(), host-known) chunks, int32 [total * 128].  Device ops only (a
    prefix sum and one chunk gather): no host read."""
    dev = ell.device
    n = row_chunks.numel()
    if total == 0 or n == 0:
        return torch.zeros(0, dtype=ell.dtype, device=dev)
    rc = row_chunks.to(torch.int64)
    row_of = torch.repeat_interleave(torch.arange(n, device=dev), rc, output_size=total)
    first = torch.cumsum(rc, 0) - rc
    k = torch.arange(total, device=dev) - first[row_of]
    return ell.view(-1, 128)[row_of * (pe // 128) + k].reshape(-1)


def unpack_compact_rows(packs: torch.Tensor, stride: int, rank_chunks: np.ndarray,
                        row_chunks: torch.Tensor, B: int, pe: int, out: torch.Tensor) -> torch.Tensor:
    """The inverse for every rank at once: ``packs`` = the ranks' packs, rank q's at chunk
    ``q * stride`` (an all-gather of equal-size buffers), ``rank_chunks[q]`` its chunk count
    (host), ``row_chunks`` [C] every row's chunk count (device), rank q holding rows
    [q B, (q + 1) B).  Writes the rows' used chunks into ``out`` (int32 [C * pe]; slots past a
    row's length are left as they are: the iterations mask them by the row length)."""
    dev = out.device
    C = row_chunks.numel()
    total = int(rank_chunks.sum())
    if total == 0:
        return out
    rc = row_chunks.to(torch.int64)
    row_of = torch.repeat_interleave(torch.arange(C, device=dev), rc, output_size=total)
    first = torch.cumsum(rc, 0) - rc
    j = torch.arange(total, device=dev)
    k = j - first[row_of]
    q = row_of // B
    start = torch.from_numpy(np.concatenate([[0], np.cumsum(rank_chunks)[:-1]]).astype(np.int64)).to(dev)
    src = q * stride + (j - start[q])
    out.view(-1, 128)[row_of * (pe // 128) + k] = packs.view(-1, 128)[src]
    return out


def _solve_compact_exchange(rows, shot, goal, move, C: int, B: int, eps: float, max_iter: int,
                            group, exact_order: bool = False, stats=None):
    """Step 5 of :func:`xt_fit_bands_sharded` with ``solve='compact'``: this rank holds the
    count rows [r B, r B + B) (``rows``); returns None (nothing exchanged) when a count of any
    rank reaches 65535, else ``(mats, heatmaps, n_iter)`` of the replicated iteration over the
    gathered compact form.  The compact rows are exchanged as their used 128-slot chunks only,
    packed per rank in row order (:func:`pack_compact_rows`); the ranks' row blocks are
    consecutive, so the gathered packs unpack into the full form (:func:`unpack_compact_rows`).
    ONE host read: the gathered row lengths and the escaped-count flag."""
    import torch.distributed as dist

    from . import _native
    from .batch import stream_handle
    W = dist.get_world_size(group)
    r = dist.get_rank(group)
    dev = rows.device
    lib = _native.lib()
    ptr = lambda t: t.data_ptr()  # noqa: E731
    r0 = r * B
    nrows = max(0, min(B, C - r0))
    pe = int(lib.sa_xt_compact_bytes(C, 1)) // 4  # slots per compact row
    ell = torch.empty(max(nrows, 1) * pe, dtype=torch.int32, device=dev)
    slen = torch.zeros(B + 1, dtype=torch.int32, device=dev)  # [B] row lengths | escaped flag
    with _phase(stats, 'compact_build'):
        if nrows:
            _native.check(lib.sa_xt_compact_rows(ptr(rows), C, nrows, ptr(ell), ptr(slen),
                                                 stream_handle()))
            slen[B] = (rows[:nrows * C].max() >= 65535).to(torch.int32)
    with _phase(stats, 'row_length_all_gather'):  # incl. the compact exchange's one host read
        lens = torch.empty(W * (B + 1), dtype=torch.int32, device=dev)
        _all_gather(lens, slen, group=group)
        lens = lens.view(W, B + 1)
        h = _to_host(lens, stats)
    if h[:, B].any():
        return None
    nch = (lens[:, :B].reshape(-1)[:C].to(torch.int64) + 127) // 128  # chunks of every row
    nch_h = ((h[:, :B].reshape(-1)[:C].astype(np.int64) + 127) // 128)
    rank_chunks = np.array([nch_h[q * B:min(C, (q + 1) * B)].sum() for q in range(W)], np.int64)
    mx = max(int(rank_chunks.max()), 1)
    with _phase(stats, 'compact_all_gather'):  # pack, all-gather, unpack
        send = torch.zeros(mx * 128, dtype=torch.int32, device=dev)
        if nrows:
            mine = pack_compact_rows(ell, nch[r0:r0 + nrows], pe, int(rank_chunks[r]))
            send[:mine.numel()] = mine
        recv = torch.empty(W * mx * 128, dtype=torch.int32, device=dev)
        _all_gather(recv, send, group=group)
        full = torch.empty(C * pe, dtype=torch.int32, device=dev)
        unpack_compact_rows(recv, mx, rank_chunks, nch, B, pe, full)
    lens_c = lens[:, :B].reshape(-1)[:C].contiguous()
    if stats is not None:
        stats['compact_gathered_bytes'] = W * mx * 128 * 4
        stats['compact_used_bytes'] = int(rank_chunks.sum()) * 128 * 4
    del recv, send, ell
    mats = torch.empty((4, C), dtype=torch.float64, device=dev)
    gp = torch.empty((2, C), dtype=torch.float64, device=dev)
    _native.check(lib.sa_xt_probabilities(ptr(shot), ptr(goal), ptr(move), C, ptr(mats), ptr(gp[0]),
                                          ptr(gp[1]), stream_handle()))
    # the whole iteration on every rank from the same compact form (sa_xt_solve_compact: the
    # single-GPU fit's own solve, so the same bits); cnt_rows is read for counts >= 65535 only,
    # which no rank has (checked above)
    from .ops import xt_solve_compact
    with _phase(stats, 'solve'):  # replicated: the same iteration on every rank
        heat, iters, path = xt_solve_compact(full, lens_c, rows, move, gp[0], gp[1], C, eps,
                                             max_iter, exact_order)
    if stats is not None:
        stats['solve_path'] = path
    if iters < 0:
        raise RuntimeError(f'xT value iteration did not converge within {max_iter} iterations')
    mats[3].copy_(heat[iters])
    return mats, heat[:iters + 1], iters


# per source rank and destination: its number of local batches, then the key count of each batch
_MAX_ROUNDS = 64


def exchange_band_keys(parts, n_bands: int, group=None, dev=None, stats=None):
    """Step 2 of :func:`xt_fit_bands_sharded`: ``parts`` = this rank's ``(keys, band_off)`` per
    local batch (keys sorted by band, ``band_off`` [NB + 1]); returns the key sets of THIS rank's
    bands, one per (local batch index, source rank): ``(keys list, band offsets list)`` where set
    k holds its band lb's keys at ``keys[k][off[k][lb] .. off[k][lb + 1])``.  Every rank runs
    the same number of exchanges (max local batches over the ranks; a rank with fewer sends
    nothing in the extra ones).

    ONE host read for the whole exchange: a first all-to-all of fixed-size headers (every
    rank's batch count and, per batch, the keys it sends each destination; at most
    ``_MAX_ROUNDS`` batches per rank) gives every rank all the split sizes at once; then per
    round one all-to-all of the keys (host-known splits, as RCCL's all_to_all_single needs) and
    one of the band offsets (equal splits, device only).  ``stats`` (dict): host reads and bytes."""
    import torch.distributed as dist
    W = dist.get_world_size(group)
    NB = n_bands
    ranges = band_ranges(NB, W)
    per = -(-NB // W)
    dev = dev if dev is not None else (parts[0][0].device if parts else torch.device('cpu'))
    R = len(parts)
    # a rank over the limit still takes part in the header exchange (its true R in the header,
    # no split sizes), and EVERY rank raises after it: raising before the collective would leave
    # the other ranks waiting in it
    Rh = min(R, _MAX_ROUNDS)
    cuts = torch.tensor([q0 for q0, _ in ranges] + [NB], dtype=torch.int64, device=dev)
    # the band offsets each destination needs: its bands q0 .. q0 + per (clamped), [W, per + 1]
    want = torch.tensor([[min(NB, q0 + k) for k in range(per + 1)] for q0, _ in ranges],
                        dtype=torch.int64, device=dev)
    hdr = torch.zeros((W, 1 + _MAX_ROUNDS), dtype=torch.int64, device=dev)
    hdr[:, 0] = R
    hc = (torch.stack([off[cuts] for _, off in parts[:Rh]]) if Rh else
          torch.zeros((0, W + 1), dtype=torch.int64, device=dev))  # [Rh, W + 1] key cuts
    if Rh:
        hdr[:, 1:1 + Rh] = (hc[:, 1:] - hc[:, :-1]).T
    rhdr = torch.empty_like(hdr)
    _all_to_all(rhdr.view(-1), hdr.view(-1), group=group)
    h = _to_host(torch.cat([rhdr.view(-1), hc.view(-1)]), stats)  # the exchange's one host read
    rh = h[:W * (1 + _MAX_ROUNDS)].reshape(W, 1 + _MAX_ROUNDS)
    hcuts = h[W * (1 + _MAX_ROUNDS):].reshape(Rh, W + 1)
    rounds = int(rh[:, 0].max())
    # the keys' dtype (int16 bins of sa_xt_count_bucket; any, for the host tests): the same on
    # every rank, so a rank without batches takes the default
    kdt = parts[0][0].dtype if parts else torch.int16
    if rounds > _MAX_ROUNDS:  # on every rank alike (every rank read the same batch counts)
        raise ValueError(f'at most {_MAX_ROUNDS} local batches per rank in one band exchange '
                         f'(a rank has {rounds})')
    sets_keys, sets_off = [], []
    sent = recvd = 0
    for k in range(rounds):
        if k < R:
            keys_k, off_k = parts[k]
            send = (hcuts[k, 1:] - hcuts[k, :-1]).astype(np.int64)
            keys = keys_k[int(hcuts[k, 0]):int(hcuts[k, W])]
            offs = off_k[want.reshape(-1)].reshape(W, per + 1)
            offs = offs - offs[:, :1]  # relative to each destination's first band
        else:  # nothing of this round here, but every rank takes part in every exchange
            send = np.zeros(W, np.int64)
            keys = torch.zeros(0, dtype=kdt, device=dev)
            offs = torch.zeros((W, per + 1), dtype=torch.int64, device=dev)
        recv_n = rh[:, 1 + k].astype(np.int64)
        total = int(recv_n.sum())
        recv = torch.empty(max(total, 1), dtype=kdt, device=dev)
        _all_to_all(recv[:total], keys.contiguous(), recv_n.tolist(), send.tolist(), group=group)
        roff = torch.empty((W, per + 1), dtype=torch.int64, device=dev)
        _all_to_all(roff.reshape(-1), offs.contiguous().reshape(-1), group=group)
        sent += int(send.sum())
        recvd += total
        starts = np.concatenate([[0], np.cumsum(recv_n)])
        for q in range(W):
            sets_keys.append(recv[int(starts[q]):])
            sets_off.append(roff[q])
    if stats is not None:
        ks = torch.tensor([], dtype=kdt).element_size()
        stats['keys_sent_bytes'] = stats.get('keys_sent_bytes', 0) + ks * sent
        stats['keys_recv_bytes'] = stats.get('keys_recv_bytes', 0) + ks * recvd
        stats['exchange_rounds'] = rounds
    return sets_keys, sets_off
