"""The pandas boundary of the batched path as a pipeline (SURVEY §8(f) "DataFrame boundary"):
actions DataFrame in -> features, labels and (given probabilities) VAEP values out, for many
games at once, with the host link kept busy.

One call of :func:`value_frames` splits the frame at game boundaries into chunks of about
``chunk_rows`` actions and, per chunk:

1. encodes it on the host (``ActionBatch.from_frame``: validation, team codes, the H2D copy);
2. runs the kernels into one of two device slots (the feature pass, labels, formula);
3. copies the slot's blocks into the frame-sized pinned host blocks on a copy stream -- one
   pitched DMA per block (``sa_copy2d_async``: the chunk's [cols x rows] block to its column
   range of the column-major [cols x n] host block) -- and moves on.

So the host encodes chunk k + 1 while the DMA engine moves chunk k, and the kernels of chunk
k + 1 wait only for the copy out of the slot they reuse (chunk k - 1).  The DataFrames are
built zero-copy over the pinned host blocks at the end (``catalog.assemble_frame``).  Every
value equals ``compute_features_batch`` / ``compute_labels_batch`` / the formula of the same
games (one segment per game; ``tests/test_gpu_dropin.py``).
"""
from __future__ import annotations

import time
from typing import Optional, Tuple

import numpy as np
import pandas as pd
import torch

from . import _native, catalog, ops
from .batch import ActionBatch, segment_offsets


def _pinned(shape, dtype) -> torch.Tensor:
    return torch.empty(shape, dtype=dtype, pin_memory=True)


def _chunks(seg_off: np.ndarray, chunk_rows: int, look: int = 16, ramp=(4, 2)):
    """Game-aligned cuts: segments [s0, s1) of about chunk_rows actions each, each cut at a game
    boundary whose row is a multiple of 4 when one lies within ``look`` games: the DMA engine
    moves a pitched copy at the link rate only from and to 4-byte aligned addresses (the bool
    and label blocks are 1 byte per row: 57 vs 14 GB/s, scripts/e2e_link.py probe, r06g).
    The first chunks are chunk_rows / ramp[i]: the link idles until the first chunk is encoded
    and valued, so a small first chunk starts the copies sooner."""
    cuts, s0 = [], 0
    nseg = len(seg_off) - 1
    while s0 < nseg:
        k = len(cuts)
        target = seg_off[s0] + (max(1, chunk_rows // ramp[k]) if k < len(ramp) else chunk_rows)
        s1 = int(np.searchsorted(seg_off, target, side='right')) - 1
        s1 = min(max(s1, s0 + 1), nseg)
        if s1 < nseg and seg_off[s1] % 4:
            near = [t for t in range(max(s0 + 1, s1 - look), min(nseg, s1 + look + 1)) if seg_off[t] % 4 == 0]
            if near:
                s1 = min(near, key=lambda t: abs(t - s1))
        cuts.append((s0, s1))
        s0 = s1
    return cuts


class _Slot:
    """Device outputs of one chunk: feature blocks (one tile of R rows), labels, values."""

    def __init__(self, plan, R: int, dev, values_dtype):
        self.fb = ops.alloc_feature_blocks(plan, R, dev)
        self.R = self.fb.Rb
        self.lab = torch.empty((3, self.R), dtype=torch.uint8, device=dev)
        self.val = torch.empty((3, self.R), dtype=values_dtype, device=dev) if values_dtype else None
        self.done = torch.cuda.Event()  # the copy out of this slot finished
        self.used = False


def value_frames(model, games: pd.DataFrame, actions: pd.DataFrame,
                 p_scores: Optional[np.ndarray] = None, p_concedes: Optional[np.ndarray] = None,
                 chunk_rows: int = 1 << 18, timeline: Optional[list] = None, ramp=(4, 2),
                 labels: bool = True
                 ) -> Tuple[pd.DataFrame, Optional[pd.DataFrame], Optional[pd.DataFrame]]:
    """(features, labels, values) of ``actions`` (each game's rows contiguous, ``games`` maps
    game_id -> home_team_id) for a VAEP / AtomicVAEP ``model`` whose transformers are all
    known ones.  ``values`` is None without probabilities (float32 or float64; values take
    their dtype, the reference's rule); ``labels=False``: features only (labels None; the
    pipelined ``compute_features_batch``)."""
    t_call = time.perf_counter()
    known, unknown = model._split_xfns()
    if unknown:
        raise ValueError('the pipelined batch path takes the built-in transformers only')
    atomic = model._atomic
    n = len(actions)
    plan = catalog.build_plan(known, model.nb_prev_actions, atomic)
    dev = torch.device('cuda', torch.cuda.current_device())
    gid = actions['game_id'].to_numpy()
    seg_off = segment_offsets(gid)
    home_map = games.set_index('game_id')['home_team_id']
    seg_gid = gid[seg_off[:-1]] if n else gid[:0]
    missing = ~pd.Index(seg_gid).isin(home_map.index)
    if missing.any():  # as the per-game lookup of compute_features_batch
        raise KeyError(seg_gid[np.flatnonzero(missing)[0]])
    homes = home_map.reindex(seg_gid).to_numpy()
    lab = model._lab
    names = {lab.scores: 'scores', lab.concedes: 'concedes', lab.goal_from_shot: 'goal_from_shot'}
    if labels and not all(f in names for f in model.yfns):
        raise ValueError('the pipelined batch path takes the built-in label functions only')
    lrow = {'scores': 0, 'concedes': 1, 'goal_from_shot': 2}
    vdt = None
    if p_scores is not None and not labels:
        raise ValueError('values come with the labels pass (labels=True)')
    if p_scores is not None:
        ps = np.asarray(p_scores)
        pc = np.asarray(p_concedes)
        if len(ps) != n or len(pc) != n:
            raise ValueError('one probability per action is required')
        vdt = torch.float32 if (ps.dtype == np.float32 and pc.dtype == np.float32) else torch.float64
        nd = np.float32 if vdt == torch.float32 else np.float64
        # the probabilities go up chunk by chunk with the chunk's columns (below), while the host
        # would otherwise wait for the copies out: not as one blocking copy before the first chunk
        ps = np.ascontiguousarray(ps, nd)
        pc = np.ascontiguousarray(pc, nd)
    # the whole frame's host blocks, column-major [cols, ld] (pinned: the DMA writes them), rows
    # on 16-byte boundaries (aligned DMA; the frames view [:, :n])
    ld = max(16, (n + 15) // 16 * 16)
    hb = _pinned((plan.n_bool, ld), torch.uint8)
    hf = _pinned((plan.n_f64, ld), torch.float64)
    hi = _pinned((plan.n_i64, ld), torch.int64)
    hl = _pinned((3, ld), torch.uint8) if labels else None
    hv = _pinned((3, ld), vdt) if vdt is not None else None
    cuts = _chunks(seg_off, chunk_rows, ramp=ramp) if n else []
    rmax = max((int(seg_off[s1] - seg_off[s0]) for s0, s1 in cuts), default=16)
    slots = [_Slot(plan, rmax, dev, vdt) for _ in range(min(2, max(1, len(cuts))))]
    main = torch.cuda.current_stream()
    copy = torch.cuda.Stream()
    lib = _native.lib()

    def d2h(dst: torch.Tensor, src: torch.Tensor, r0: int, m: int, rows: int):
        """rows x m elements of the [rows, R] device block src into dst[:, r0:r0 + m]."""
        if rows == 0 or m == 0:
            return
        es = src.element_size()
        _native.check(lib.sa_copy2d_async(dst.data_ptr() + r0 * es, dst.shape[1] * es,
                                           src.data_ptr(), src.shape[-1] * es, m * es, rows,
                                           copy.cuda_stream))
    t_start = time.perf_counter()
    if timeline is not None:
        timeline.append({'setup_ms': round((t_start - t_call) * 1e3, 2)})
    evs = []
    for k, (s0, s1) in enumerate(cuts):
        r0, r1 = int(seg_off[s0]), int(seg_off[s1])
        m = r1 - r0
        slot = slots[k % len(slots)]
        th0 = time.perf_counter()
        # 1. host encode + H2D of this chunk (overlaps the copy out of the previous chunk)
        ab = ActionBatch.from_frame(actions.iloc[r0:r1], atomic=atomic, home_team_id=list(homes[s0:s1]),
                                    segments='game', dev=dev, pinned=True)
        th1 = time.perf_counter()
        # 2. kernels, once the slot's previous copy is done
        if slot.used:
            main.wait_event(slot.done)
        fb = ops.FeatureBlocks(plan, m, slot.R, slot.R, slot.fb.bool_block, slot.fb.f64_block,
                               slot.fb.i64_block)
        ops.features_into(ab.struct(), fb)
        lb = ops.LabelBlocks(m, slot.lab[0], slot.lab[1], slot.lab[2])
        if labels and vdt is not None:
            tps = torch.from_numpy(ps[r0:r1]).to(dev, non_blocking=True)
            tpc = torch.from_numpy(pc[r0:r1]).to(dev, non_blocking=True)
            ops.labels_formula(ab, tps, tpc, labels_out=lb, values_out=slot.val)
        elif labels:
            ops.labels(ab, out=lb)
        # 3. pitched copies into the frame's host blocks, on the copy stream
        ev = torch.cuda.Event()
        ev.record(main)
        copy.wait_event(ev)
        if timeline is not None:  # diagnostics: the copy's device-side start / end
            ea, eb = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            ea.record(copy)
        d2h(hb, slot.fb.bool_block[0], r0, m, plan.n_bool)
        d2h(hf, slot.fb.f64_block[0], r0, m, plan.n_f64)
        d2h(hi, slot.fb.i64_block[0], r0, m, plan.n_i64)
        if labels:
            d2h(hl, slot.lab, r0, m, 3)
        if vdt is not None:
            d2h(hv, slot.val, r0, m, 3)
        slot.done.record(copy)
        if timeline is not None:
            eb.record(copy)
            evs.append((k, m, th0 - t_start, th1 - t_start, time.perf_counter() - t_start, ea, eb))
        slot.used = True
        slot.keep = (ab, tps, tpc) if vdt is not None else ab  # alive until the slot is reused
    copy.synchronize()
    main.synchronize()
    if timeline is not None and evs:
        e0 = evs[0][5]
        for k, m, a, b, c, ea, eb in evs:  # host ms: encode start / end, launches queued; device ms
            timeline.append({'chunk': k, 'rows': m, 'encode_ms': (round(a * 1e3, 2), round(b * 1e3, 2)),
                             'queued_ms': round(c * 1e3, 2),
                             'd2h_ms_from_first': (round(e0.elapsed_time(ea), 2), round(e0.elapsed_time(eb), 2))})
        timeline.append({'host_total_ms': round((time.perf_counter() - t_start) * 1e3, 2)})
    t_frames = time.perf_counter()
    X = catalog.assemble_frame(plan, hb.numpy(), hf.numpy(), hi.numpy(), n, pd.RangeIndex(n))
    Y = None
    if labels:
        hln = hl.numpy()  # numpy views keep their pinned tensors alive (so do the frames over them)
        ycols = {}
        for f in model.yfns:  # compute_labels' columns (atomic: goal_from_shot is named 'goal')
            key = names[f]
            ycols['goal' if (atomic and key == 'goal_from_shot') else key] = hln[lrow[key], :n].view(bool)
        Y = pd.DataFrame(ycols, index=pd.RangeIndex(n), copy=False)  # views, as X (a copy: 5 ms)
    V = None
    if vdt is not None:
        hvn = hv.numpy()
        V = pd.DataFrame({'offensive_value': hvn[0, :n], 'defensive_value': hvn[1, :n],
                          'vaep_value': hvn[2, :n]}, copy=False)
    if timeline is not None:
        timeline.append({'frames_ms': round((time.perf_counter() - t_frames) * 1e3, 2)})
    return X, Y, V
