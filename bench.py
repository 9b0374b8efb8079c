#!/usr/bin/env python
"""Benchmark: SPADL actions/s valued (VAEP features + labels + formula) on MI355X.

One *step* = one pass of the valuation hot path over one batch: the reference's
``VAEP.compute_features`` (k=3, default xfns: 568 columns) + ``compute_labels``
(scores, concedes) + ``formula.value`` (f64 probabilities) for every game of the
batch, all kernels on device-resident inputs (synthetic data, cfg2 of BASELINE.json:
10k games, ~16M actions per GPU).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--games G]

N > 1 runs one rank per GPU under torch.distributed.run; each rank values its own
10k games (weak scaling, no data-path collective) and rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import contextlib
import copy
import json
import os
import sys
import time
from typing import Tuple

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from socceraction_amd import batch as B  # noqa: E402
from socceraction_amd import _native, catalog, ops, synthetic  # noqa: E402
from socceraction_amd._native import XFN  # noqa: E402

SPADL_DEFAULT = ['actiontype_onehot', 'result_onehot', 'actiontype_result_onehot',
                 'bodypart_onehot', 'time', 'startlocation', 'endlocation', 'startpolar',
                 'endpolar', 'movement', 'team', 'time_delta', 'space_delta', 'goalscore']

# algorithmic bytes per action of each kernel (its inputs read once + outputs written once;
# DESIGN.md "Kernels and rooflines")
BYTES = {'bool_features': 7 + 515,             # type/result/bodypart u8 + team i32 -> 515 bools
         # 5 f64 + 4 u8 + team -> 47 f64 + 6 i64 (period ids, and goalscore fused in)
         'num_features': 48 + 47 * 8 + 6 * 8,
         'num_features_nogs': 48 + 47 * 8 + 3 * 8,  # A/B: goalscore as its own scan
         # the numeric pass with labels + f64 formula riding in it (sa_vaep_step_f64): + 2 probs
         # in, + 2 labels + 3 values out
         'num_step': 48 + 16 + 47 * 8 + 6 * 8 + 2 + 24,
         'goalscore': 6 + 24, 'labels': 6 + 2, 'formula': 30 + 24,
         'labels_formula': 30 + 2 + 24,  # type/result/team/time/2 probs -> 2 labels + 3 values
         # count pass 34 B + its 4-B rate codes, rate 4 + 8 B (solve: 192 cells)
         'xt_fit_rate': 34 + 4 + 4 + 8}
KERNELS = ('bool_features', 'num_features', 'num_step', 'num_features_nogs', 'goalscore', 'labels',
           'formula', 'labels_formula', 'xt_fit_rate')
STEP_CALLS = ('bool_features', 'num_features', 'goalscore', 'labels', 'formula')
# launch entries that cover several of STEP_CALLS in one kernel
FUSED_CALLS = {'labels_formula': ('labels', 'formula'), 'num_features': ('num_features', 'goalscore'),
               'num_features_nogs': ('num_features',),
               'num_step': ('num_features', 'goalscore', 'labels', 'formula')}
# the HIP kernel each step entry launches (socceraction_amd/csrc/sa_vaep.hip)
KERNEL_NAMES = {'bool_features': 'bool_colgroup_kernel', 'num_features': 'num_features_kernel',
                'num_features_nogs': 'num_features_kernel', 'num_step': 'num_features_kernel',
                'goalscore': 'goalscore_wave16_kernel', 'labels': 'labels_kernel',
                'formula': 'formula_kernel', 'labels_formula': 'labels_formula_kernel',
                'xt_fit_rate': 'xt_count_kernel + xt_solve_reg_kernel + xt_rate_cells_kernel'}


def step_bytes(xt_source: str) -> dict:
    """Algorithmic bytes per action of each step entry for an xT source (bench xt_step)."""
    b = dict(BYTES)
    if xt_source == 'cells':  # the f64 pass writes the cell code; count reads it, rate it + 8
        from socceraction_amd import _native
        cb = 2 if 16 * 12 <= _native.SA_XT_CELLS16_MAX_C else 4  # 16-bit codes on the 16 x 12 grid
        b['num_features'] += cb
        b['num_features_nogs'] += cb
        b['num_step'] += cb
        b['xt_fit_rate'] = cb + cb + 8
    elif xt_source == 'coords':  # count 34 B, rate 34 + 8
        b['xt_fit_rate'] = 34 + 34 + 8
    return b
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
STEP_BYTES = 1029  # VAEP feat + labels + formula, inputs read once + outputs written once


def launch_ranks(n: int, argv, run=None) -> int:
    """``bench.py --gpus N`` started outside torch.distributed.run: start one rank per GPU as a
    CHILD ``python -m torch.distributed.run`` (this process has not touched the GPU; it never
    execs) with the same arguments, let the child's rank 0 print the JSON line, and return the
    child's exit status."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', f'--nproc-per-node={n}',
           '--master-addr', '127.0.0.1', '--master-port', str(port), os.path.abspath(__file__)]
    cmd += list(argv)
    env = dict(os.environ, MASTER_ADDR='127.0.0.1')
    env.setdefault('HSA_ENABLE_IPC_MODE_LEGACY', '0')  # dmabuf IPC only on this driver
    return (run or subprocess.run)(cmd, env=env).returncode


def check_world(gpus: int) -> None:
    """Under torch.distributed.run the launched world must be the --gpus the line reports."""
    ws = int(os.environ.get('WORLD_SIZE', '1'))
    if ws != gpus:
        print(f'bench.py: --gpus {gpus} but WORLD_SIZE={ws}', file=sys.stderr)
        raise SystemExit(2)


def _dist():
    """One process per GPU (torch.distributed.run); backend nccl = RCCL over xGMI.
    SA_DIST_BACKEND=gloo is for rehearsing several ranks on one GPU."""
    ws = int(os.environ.get('WORLD_SIZE', '1'))
    # SA_BENCH_DIST=1: the process-group path even at one rank (RCCL with world size 1), so the
    # N-GPU code runs end to end in -m gpu on a one-GPU box (tests/test_gpu_bench.py)
    if ws > 1 or os.environ.get('SA_BENCH_DIST') == '1':
        import torch.distributed as dist
        lr = int(os.environ.get('LOCAL_RANK', '0'))
        backend = os.environ.get('SA_DIST_BACKEND', 'nccl')
        torch.cuda.set_device(lr % max(1, torch.cuda.device_count()))
        if backend == 'nccl':
            dist.init_process_group('nccl', device_id=torch.device('cuda', lr))
        else:
            dist.init_process_group(backend)
        return dist, dist.get_rank(), ws
    return None, 0, 1


def _reduce(dist, value, op, dev):
    """All-reduce one scalar (RCCL on device tensors; gloo on host tensors)."""
    on_dev = dist.get_backend() == 'nccl'
    t = torch.tensor([value], dtype=torch.float64, device=dev if on_dev else 'cpu')
    dist.all_reduce(t, op=op)
    return float(t.item())


def allreduce_counts(dist, acc) -> None:
    """The xT fit's one exchange: every rank's count buffers summed by ONE all-reduce (RCCL; a
    gloo rehearsal sums the same buffer through host memory)."""
    from socceraction_amd import shard
    if dist is None:
        return
    shard.allreduce_xt_counts(acc)  # ONE all-reduce of the whole count allocation


def xt_step(ab, dist, source: str = 'cells', cells=None, shared: bool = True, sync_solve: bool = False):
    """BASELINE cfg4 inside the step: xT 16x12 fit on the step's actions (count pass, RCCL
    all-reduce of the counts across ranks, value iteration to eps=1e-5; the solve synchronises
    its stream) and ExpectedThreat.rate of every action, as two phases so the caller can enqueue
    the VAEP kernels in between. Returns (start, finish, holder of the last solution).

    source 'cells': count and rate read the 4-B cell codes the f64 feature pass wrote into
    ``cells`` (sa_vaep_features_xt); 'codes': the count pass reads the coordinates and writes a
    4-B rate operand per action for the rate; 'coords': both passes read the coordinates."""
    from socceraction_amd import shard
    state = {}
    cur_cells = cells if callable(cells) else (lambda: cells)  # the step's cell-code buffer
    # the step's count buffers, allocated once and zeroed by ONE fill on the side stream while
    # the numeric pass runs (zero()), not by per-step allocations on the main stream
    acc0 = ops.xt_zero_counts(16, 12, ab.device)
    codes = ops.xt_rate_codes_buffer(ab.n, ab.device) if source == 'codes' else None
    rate_out = torch.empty(max((ab.n + 15) // 16 * 16, 16), dtype=torch.float64, device=ab.device)

    def count():
        if source == 'none':  # --ab diagnostic only: the VAEP kernels without the xT part
            return
        if source == 'cells':
            state['acc'] = ops.xt_count_cells(cur_cells(), ab.n, 16, 12, acc=acc0, shared=shared)
        else:
            state['acc'] = ops.xt_count(ab, 16, 12, acc=acc0, codes=codes, shared=shared)

    def zero():
        acc0.zero_()

    def reduce():
        if source == 'none':
            return
        allreduce_counts(dist, state['acc'])

    def start():
        count()
        reduce()

    def finish():
        if source == 'none':
            return
        # the solve without a host round trip (its iteration count stays on the device until
        # the report), so the rate is enqueued right behind it; sync_solve: the round-trip form
        sol = (ops.xt_solve(state.pop('acc')) if sync_solve else ops.xt_solve_async(state.pop('acc')))
        if source == 'cells':
            ops.xt_rate_cells(cur_cells(), ab.n, 16, 12, sol.mats[3], out=rate_out)
        elif source == 'codes':
            ops.xt_rate_codes(codes, ab.n, sol.mats[3], out=rate_out)
        else:
            ops.xt_rate(ab, sol.mats[3].reshape(12, 16), 16, 12)
        state['sol'] = sol
    start.count, start.reduce, start.zero = count, reduce, zero
    state['acc_buf'], state['rate'] = acc0, rate_out  # the parity check reads the last step's
    return start, finish, state


class Parity:
    """The line's own correctness check, OUTSIDE the timed region: the timed step's output
    buffers for sampled games against the numpy oracle (the checker; never the thing measured).
    Bit-exact for bools, ints, counts, iteration counts and the xT surface; floats within
    |a - b| <= 1e-6 |ref| + 1e-12 (north_star's bar), NaN / inf in the same places."""

    def __init__(self):
        self.ok, self.max_rel_err, self.failures, self.games, self.values = True, 0.0, [], 0, 0

    def _fail(self, what: str) -> None:
        self.ok = False
        if len(self.failures) < 20:
            self.failures.append(what)

    def exact(self, name: str, got, ref) -> None:
        got, ref = np.asarray(got), np.asarray(ref)
        self.values += ref.size
        if got.shape != ref.shape or not np.array_equal(got.astype(np.int64), ref.astype(np.int64)):
            self._fail(name)

    def close(self, name: str, got, ref) -> None:
        a, b = np.asarray(got, np.float64), np.asarray(ref, np.float64)
        self.values += b.size
        if a.shape != b.shape or (np.isnan(a) != np.isnan(b)).any():
            return self._fail(name + ' (shape / NaN pattern)')
        fin = np.isfinite(b)
        if (a[~fin & ~np.isnan(b)] != b[~fin & ~np.isnan(b)]).any():
            return self._fail(name + ' (inf)')
        err = np.abs(a[fin] - b[fin])
        if err.size:
            rel = err / np.maximum(np.abs(b[fin]), 1e-300)
            self.max_rel_err = max(self.max_rel_err, float(np.max(np.where(err == 0, 0.0, rel))))
            if (err > 1e-6 * np.abs(b[fin]) + 1e-12).any():
                self._fail(name)

    def merge(self, dist, dev) -> None:
        """Every rank checked its own games: the line reports the worst rank."""
        if dist is None:
            return
        bad = _reduce(dist, 0.0 if self.ok else 1.0, dist.ReduceOp.MAX, dev)
        self.max_rel_err = _reduce(dist, self.max_rel_err, dist.ReduceOp.MAX, dev)
        self.games = int(_reduce(dist, self.games, dist.ReduceOp.SUM, dev))
        self.values = int(_reduce(dist, self.values, dist.ReduceOp.SUM, dev))
        if bad and self.ok:
            self._fail('another rank')

    def record(self) -> dict:
        return {'games': self.games, 'values_checked': self.values, 'ok': self.ok,
                'max_rel_err': float(f'{self.max_rel_err:.3e}'), 'failures': self.failures,
                'oracle': 'oracle/vaep_oracle.py, oracle/xt_oracle.py (numpy restatement pinned '
                          'by reference goldens), outside the timed region'}


SPADL_COLS = ('period_id', 'time_seconds', 'team_id', 'start_x', 'start_y', 'end_x', 'end_y',
              'type_id', 'result_id', 'bodypart_id')
ATOMIC_COLS = ('period_id', 'time_seconds', 'team_id', 'x', 'y', 'dx', 'dy', 'type_id',
               'bodypart_id')


def sample_games(n_games: int, k: int = 12, seed: int = 2026) -> list:
    """The checked games: the first, the last and k - 2 seeded random ones."""
    if n_games <= k:
        return list(range(n_games))
    rest = np.random.default_rng(seed).choice(np.arange(1, n_games - 1), k - 2, replace=False)
    return [0, n_games - 1] + sorted(int(g) for g in rest)


def check_vaep(par: Parity, d, out, scores, concedes, val, probs, atomic: bool = False,
               games=None) -> None:
    """Features (every column), labels and (when ``val``) the f64 formula of sampled games of
    the batch ``d`` in the device buffers vs the oracle, per game as the reference's
    compute_features / compute_labels / formula.value (vaep/base.py:97-137, formula.py:116-151)."""
    from oracle import vaep_oracle as vo
    off = d['game_off']
    xfns = vo.ATOMIC_DEFAULT if atomic else vo.SPADL_DEFAULT
    for g in (sample_games(len(off) - 1) if games is None else games):
        s, e = int(off[g]), int(off[g + 1])
        cols = {c: d[c][s:e] for c in (ATOMIC_COLS if atomic else SPADL_COLS)}
        ref = vo.features(cols, 3, xfns, atomic=atomic, home=[d['home_team_id'][g]])
        if [r[0] for r in ref] != out.plan.names:
            par._fail(f'game {g}: column names')
            continue
        blocks = {k: out.rows(k, s, e).cpu().numpy() for k in 'bfi'}
        for (name, kind, col), (_, _, rv) in zip(out.plan.order, ref):
            (par.close if kind == 'f' else par.exact)(f'game {g} {name}', blocks[kind][col], rv)
        lab = vo.labels(cols, atomic=atomic)
        par.exact(f'game {g} scores', scores[s:e].cpu().numpy().astype(bool), lab['scores'])
        par.exact(f'game {g} concedes', concedes[s:e].cpu().numpy().astype(bool), lab['concedes'])
        if val is not None:
            fo = vo.formula(cols, probs['scores'][s:e], probs['concedes'][s:e], atomic=atomic)
            v = val[:, s:e].cpu().numpy()
            for r, c in enumerate(('offensive_value', 'defensive_value', 'vaep_value')):
                par.close(f'game {g} {c}', v[r], fo[c])
        par.games += 1


def oracle_counts(d, l: int, w: int, dist=None, dev=None, acc: dict = None) -> dict:
    """The oracle's xT counts of the batch ``d`` (added to ``acc`` when given), summed over the
    ranks when ``dist`` (the same exchange the device counts go through)."""
    from oracle import xt_oracle as xo
    cnt = xo.counts({c: d[c] for c in ('start_x', 'start_y', 'end_x', 'end_y', 'type_id',
                                        'result_id')}, l, w) if d is not None else None
    if acc is not None and cnt is not None:
        cnt = {k: acc[k] + cnt[k] for k in cnt}
    elif cnt is None:
        cnt = acc
    if dist is not None:
        on_dev = dist.get_backend() == 'nccl'
        for k in cnt:
            t = torch.from_numpy(np.ascontiguousarray(cnt[k])).to(dev if on_dev else 'cpu')
            dist.all_reduce(t)
            cnt[k] = t.cpu().numpy()
    return cnt


def check_surface(par: Parity, tag: str, got: np.ndarray, ref: np.ndarray, rtol: float) -> None:
    """The xT surface: bit for bit (rtol 0: the reference's summation order), or within rtol
    relative (the large grids' reordered sums, whose iteration count is still checked exactly);
    the largest relative difference goes into the parity record."""
    par.values += ref.size
    err = np.abs(got - ref)
    rel = float(np.max(np.where(err == 0, 0.0, err / np.maximum(np.abs(ref), 1e-300)))) if ref.size else 0.0
    par.surface_rel_err = max(getattr(par, 'surface_rel_err', 0.0), rel)
    if got.shape != ref.shape or (np.isnan(got) != np.isnan(ref)).any() or rel > rtol:
        par._fail(f'{tag} surface')


def check_xt(par: Parity, cnt: dict, acc, xT_dev, n_iter: int, l: int, w: int,
             rtol: float = 0.0) -> np.ndarray:
    """xT fit (xthreat.py:322-345): the counts the device solved from (all ranks' counts after
    the all-reduce) == the oracle's counts of the same actions, bit for bit; the iteration count
    == the oracle's value iteration over them (xthreat.py:278-320), the surface bit for bit
    (``rtol`` 0) or within ``rtol`` relative. Returns the oracle surface."""
    from oracle import xt_oracle as xo
    tag = f'xT {l}x{w}'
    for k, t in (('shot', acc.shot), ('goal', acc.goal), ('move', acc.move)):
        par.exact(f'{tag} {k} counts', t.cpu().numpy(), cnt[k].reshape(-1))
    # the counts the solve read: the compact rows when the count wrote them (cfg5 writes no
    # dense table on one rank), else the dense table
    idx, tc = ops.xt_transition_entries(acc)
    tr = np.zeros(l * w * l * w, np.int64)
    tr[idx.cpu().numpy()] = tc.cpu().numpy()
    par.exact(f'{tag} transition counts', tr, cnt['trans'].reshape(-1))
    fit = xo.solve(cnt, l, w)
    par.exact(f'{tag} iterations', n_iter + 1, len(fit['heatmaps']))
    check_surface(par, tag, xT_dev.cpu().numpy().reshape(w, l), fit['xT'], rtol)
    return fit['xT']


def check_xt_rate(par: Parity, d, rate_dev, xT: np.ndarray, interp: bool = False,
                  games=None) -> None:
    """ExpectedThreat.rate (xthreat.py:408-465) of sampled games: the device values == the
    oracle's rate on the same surface (NaN for every action but successful moves)."""
    from oracle import xt_oracle as xo
    off = d['game_off']
    for g in (sample_games(len(off) - 1) if games is None else games):
        s, e = int(off[g]), int(off[g + 1])
        cols = {c: d[c][s:e] for c in ('start_x', 'start_y', 'end_x', 'end_y', 'type_id', 'result_id')}
        par.close(f'xT rate game {g}', rate_dev[s:e].cpu().numpy(),
                  xo.rate(cols, xT, use_interpolation=interp))


ATOMIC_DEFAULT = ['actiontype', 'actiontype_onehot', 'bodypart', 'bodypart_onehot', 'time',
                  'team', 'time_delta', 'location', 'polar', 'movement_polar', 'direction',
                  'goalscore']


def _iterations(sol) -> int:
    """The value iteration's count (a device tensor for the asynchronous solve)."""
    n = sol.n_iter if isinstance(sol.n_iter, int) else int(sol.n_iter.item())
    if n < 0:
        raise RuntimeError('xT value iteration did not converge')
    return n


def _num_index(order) -> int:
    """Position of the numeric feature pass (num_features or num_features_nogs) in a step order."""
    return next(i for i, k in enumerate(order) if k.startswith('num_'))


# the event class of the step's stream forks / joins and per-kernel timings: 'native' =
# socceraction_amd.events.DeviceEvent (no system-scope fence on record), 'torch' =
# torch.cuda.Event (set by --events; --ab variants may override it with ev=...)
EVENTS = {'kind': 'native'}


def _event(enable_timing: bool = False, kind: str = None):
    if (kind or EVENTS['kind']) == 'native':
        from socceraction_amd.events import DeviceEvent
        return DeviceEvent(enable_timing)
    return torch.cuda.Event(enable_timing=enable_timing)


def _record(stream, kind: str = None):
    e = _event(kind=kind)
    e.record(stream)
    return e


_LAST_TIMES: list = []


def _events_median_ms(fn, reps: int) -> Tuple[float, float, float]:
    """(median, min, max) ms of ``reps`` back-to-back calls of ``fn``, one HIP event pair per
    call on the current stream, after one untimed call."""
    fn()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(reps)]
    for a, b in ev:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    t = [a.elapsed_time(b) for a, b in ev]
    _LAST_TIMES[:] = t  # the per-call series of the last call (scripts/cfg3_time.py)
    return float(np.median(t)), float(np.min(t)), float(np.max(t))


def _events_ms(fn, reps: int) -> float:
    """Mean ms of ``fn`` over ``reps`` back-to-back calls (HIP events, current stream)."""
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


def atomic_extra(dist, rank, world, dev, games: int, reps: int = 21, check: bool = True,
                 contiguous='require', batch_contiguous: bool = False) -> dict:
    """BASELINE cfg3 alongside the main line: Atomic-VAEP features (k=3, default xfns, 154
    columns) + labels of cfg3's ``games`` synthetic atomic games (10,000 ≈ 4.0e7 atomic
    actions), sharded by game over the ranks (this entry scales strongly)."""
    mine = games // world + (1 if rank < games % world else 0)
    first = rank * (games // world) + min(rank, games % world)
    d = synthetic.atomic_games(mine, game_id0=first)
    ab = B.ActionBatch.from_columns(d, atomic=True, dev=dev, contiguous=batch_contiguous)
    # the bool block in physically contiguous VRAM, as the main step's (the bool
    # pass is sensitive to its address translations; from the caching allocator its time
    # followed the allocations placed before it: 3.80 vs 3.41 - 3.43 ms per step on one box,
    # profiles/r04_cfg3_contig_ab.json)
    plan = catalog.build_plan(ATOMIC_DEFAULT, 3, True)
    torch.cuda.empty_cache()  # cached blocks of earlier entries out of the way of the range
    # 'require': no silent fall-back to the caching allocator (the line says which served it)
    out = ops.alloc_feature_blocks(plan, ab.n, dev, 1024, 128, contiguous=contiguous)
    ops.features(ab, ATOMIC_DEFAULT, 3, out=out, bool_tile=1024, num_tile=128)
    lab = ops.labels(ab)

    s = ab.struct()

    def step():  # features, then the labels as their own launch (sa_vaep_step_f64 routes every
        ops.step_into(s, out, None, None, 10, lab, None)  # atomic step to separate launches)
    ms, ms_lo, ms_hi = _events_median_ms(step, reps)
    par = Parity()
    if check:  # the timed launches' own buffers: sampled atomic games vs the oracle
        torch.cuda.synchronize()
        check_vaep(par, d, out, lab.scores, lab.concedes, None, None, atomic=True)
        par.merge(dist, dev)
    # placement: the same step into a second, freshly allocated set of blocks, timed the same way
    # (never the value): some allocations run every step ~10 % slower with the same bytes, TLB
    # misses and clock (profiles/r06p_*); the line says which kind the first one was
    placement = None
    try:
        out2 = ops.alloc_feature_blocks(plan, ab.n, dev, 1024, 128, contiguous=contiguous)
        ops.features(ab, ATOMIC_DEFAULT, 3, out=out2, bool_tile=1024, num_tile=128)

        def step2():
            ops.step_into(s, out2, None, None, 10, lab, None)
        ms2 = _events_median_ms(step2, reps)[0]
        placement = {'realloc_ms_per_step': round(ms2, 4), 'first_over_realloc': round(ms / ms2, 4),
                     'mode': ('slow placement: the first (timed) allocation >= 4 % slower than a fresh one'
                              if ms > 1.04 * ms2 else
                              'the fresh allocation got the slow placement (>= 4 % slower); the timed one did not'
                              if ms2 > 1.04 * ms else 'no slow placement seen')}
        del out2
    except (RuntimeError, ValueError, MemoryError) as e:  # no second contiguous range: skip
        placement = {'error': f'{type(e).__name__}: {e}'}
    n, total, wall = ab.n, ab.n, ms
    if dist is not None:
        wall = _reduce(dist, ms, dist.ReduceOp.MAX, dev)
        total = int(_reduce(dist, n, dist.ReduceOp.SUM, dev))
    p = out.plan
    bpa = 47 + p.n_bool + 8 * (p.n_f64 + p.n_i64) + 2
    return {'workload': f'cfg3: Atomic-VAEP features (k=3, default xfns, 154 cols) + labels of '
                        f'{games:,} synthetic atomic games over {world} rank(s)',
            'atomic_actions_per_gpu': n, 'atomic_actions_total': total, 'scaling': 'strong',
            'bool_block': out.bool_alloc,
            'ms_per_step': round(wall, 4),
            'placement': placement,
            'timing': f'median of {reps} steps (HIP events per step; min {ms_lo:.4f}, max '
                      f'{ms_hi:.4f} ms on rank {rank})',
            'atomic_actions_per_s': round(total / wall * 1e3, 1), 'bytes_per_action': bpa,
            'frac_of_8TBs_per_gpu': round(bpa * n / ms * 1e-6 / HBM_PEAK_GBS, 4),
            **({'parity': par.record()} if check else {})}


def xt105_extra(ab, dist, dev, sharded: bool = False, cfg5_games: int = 62500,
                rank: int = 0, world: int = 1, step_games: int = 10000, d=None,
                check: bool = True, reps: int = 21, solve: str = 'compact') -> dict:
    """BASELINE cfg5 alongside the main line: xT 105x68 fit of cfg5's 62,500 games (≈1.0e8
    actions; split over the ranks, so this entry scales strongly) -- count pass over this
    rank's games, RCCL all-reduce of the 7140-cell count vectors and 204 MB transition counts,
    value iteration over the 7140^2 system -- + rate(use_interpolation=True) of every action on
    the 1050x680 surface. The rank's games are the step's own batch (when it holds no more
    than the rank's share) plus freshly generated synthetic games, each a device-resident batch
    before the timed region; ``cfg5_games=0`` times the step's batch alone."""
    from socceraction_amd import shard
    l, w = 105, 68
    batches = [ab]
    first = d  # host columns of the first batch (its rate is checked game by game)
    # the oracle's counts of every batch, accumulated while the batches are generated (the
    # host columns are not kept): the checker of the fit below
    ocnt = oracle_counts(d, l, w) if check and d is not None else None
    if cfg5_games > 0:
        mine = cfg5_games // world + (1 if rank < cfg5_games % world else 0)
        batches = [ab] if mine >= step_games else []
        if not batches:
            first, ocnt = None, None
        left = mine - (step_games if batches else 0)
        gid = 10_000_000 + rank * (cfg5_games + 1)  # ids disjoint from the step's games
        while left > 0:
            c = min(left, step_games)
            dc = synthetic.spadl_games(c, game_id0=gid)
            batches.append(B.ActionBatch.from_columns(dc, dev=dev))
            if check:
                ocnt = oracle_counts(dc, l, w, acc=ocnt)
                first = dc if first is None else first
            gid += c
            left -= c

    def once(mode, marks=None, timer=None):
        """One fit + rate in ``mode`` = (sharded, solve); ``timer`` (shard.PhaseTimes): HIP
        events around every phase, incl. the exchange's collectives."""
        msharded, msolve = mode

        def mark():  # the instrumented call only: phase boundaries (synchronised)
            if marks is not None:
                torch.cuda.synchronize()
                marks.append(time.perf_counter())

        def phase(name):
            return timer.phase(name) if timer is not None else contextlib.nullcontext()
        mark()
        # the count of every batch: band-owned (sa_xt_count_bucket per batch, the C x C table
        # written once by sa_xt_count_from_buckets; no global atomics), into a fresh accumulator
        # and, per action, the operand of the interpolated rate below (start / end node of the
        # 1050 x 680 grid: 8 B read by the rate instead of 34 B of coordinates and ids)
        if msharded and dist is not None:  # band-sharded: all-to-all of the counted actions,
            mark()                          # each rank counts its bands; row-sharded iteration
            mark()  # (count and exchange happen inside the sharded fit)
            xstats.clear()
            if timer is not None:
                xstats['timer'] = timer
            mats, _, n_iter, err = shard.xt_fit_bands_sharded(batches, l, w, interp_codes=icodes,
                                                              solve=msolve, stats=xstats)
            xstats.pop('timer', None)
            acc = None  # each rank holds only its row block of the transition counts
            path[0] = xstats.get('solve_path', 'sequential')
        else:  # one all-reduce of the counts, replicated solve
            # one rank: the compact count rows alone (the solve reads nothing else; no 204 MB
            # dense flush); replicated over ranks: the dense table the all-reduce sums
            with phase('count'):
                acc = ops.xt_count_many(batches, l, w, interp_codes=icodes, dense=dist is not None)
            mark()
            with phase('count_all_reduce'):
                allreduce_counts(dist, acc)
            mark()
            if marks is None and timer is None:  # the timed calls: solve + rate in one call, the
                # rate queued behind the solve before its host round trip (sa_xt_fit_rate_interp_codes)
                sol, rates, _ = ops.xt_fit_rate_interp_codes(acc, icodes, [b.n for b in batches],
                                                             axes=axes, outs=rate_out)
                path[0] = sol.path
                return sol.n_iter, acc, sol.mats, rates
            with phase('solve'):
                sol = ops.xt_solve(acc, transition=False)  # synchronises; ExpectedThreat.fit's
            mats, n_iter = sol.mats, sol.n_iter           # call above 1024 cells
            path[0] = sol.path
        mark()
        # rate(use_interpolation=True): each action's two node values evaluated in place from
        # the 105 x 68 surface staged in LDS (sa_xt_rate_interp_codes_many: every batch in one
        # launch), bit-identical to the 1050 x 680 grid gather
        xT = mats[3].reshape(w, l)
        with phase('rate'):
            rates, _ = ops.xt_rate_interp_codes_many(icodes, [b.n for b in batches], xT, l, w,
                                                     1050, 680, axes=axes, outs=rate_out)
        mark()
        return n_iter, acc, mats, rates
    path = ['sequential']  # the value iteration's summation path of the last call
    xstats = {}  # band-sharded exchange: kind, bytes and host reads of the last call (this rank)
    axes = ops.xt_interp_axes(l, w, dev)  # node positions (constants of the reference's grid)
    icodes = [ops.xt_interp_codes_buffer(b.n, dev) for b in batches]
    rate_out = [torch.empty(max(b.n, 16), dtype=torch.float64, device=dev) for b in batches]
    if check:
        ocnt = oracle_counts(None, l, w, dist, dev, acc=ocnt)  # every rank's counts
    n = sum(b.n for b in batches)
    total = n
    if dist is not None:
        total = int(_reduce(dist, n, dist.ReduceOp.SUM, dev))

    def run(mode, nreps):
        """Time ``mode`` (median of ``nreps`` wall-clocked calls), one call with synchronised
        phase marks, one with per-phase HIP events, then check an untouched call's outputs."""
        once(mode)  # warm-up (allocator, first launches)
        torch.cuda.synchronize()
        times = []
        for _ in range(nreps):  # each call wall-timed alone (the solve synchronises with the host)
            if dist is not None:
                dist.barrier()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            once(mode)
            torch.cuda.synchronize()
            times.append(time.perf_counter() - t0)
        dt = float(np.median(times))
        marks = []
        once(mode, marks)  # one more call, synchronised between phases: where the time goes
        phases = dict(zip(('count', 'exchange', 'solve', 'rate'),
                          (round((b - a) * 1e3, 3) for a, b in zip(marks, marks[1:]))))
        timer = shard.PhaseTimes(dev)
        once(mode, timer=timer)  # and one with HIP events around each phase (no host syncs added)
        events = timer.ms()
        n_iter, acc, mats, rates = once(mode)  # the checked outputs come from an untouched call
        torch.cuda.synchronize()
        par = Parity()
        # reordered sums: the iteration count exact, the surface within 1e-12 relative (the
        # error bound allows 4e-11 after 26 iterations; north_star's bar is 1e-6); in order: bit
        # for bit
        rtol = 0.0 if path[0] == 'sequential' else 1e-12
        if check:  # the last call's counts, surface, iterations and the first batch's rates
            if acc is None:  # row-sharded solve: the surface is checked, the counts are not held
                from oracle import xt_oracle as xo
                fit = xo.solve(ocnt, l, w)
                xT = fit['xT']
                par.exact('xT 105x68 iterations', n_iter + 1, len(fit['heatmaps']))
                check_surface(par, 'xT 105x68', mats[3].cpu().numpy().reshape(w, l), xT, rtol)
            else:
                xT = check_xt(par, ocnt, acc, mats[3], n_iter, l, w, rtol)
            if first is not None:
                check_xt_rate(par, first, rates[0], xT, interp=True)
                par.games += len(sample_games(len(first['game_off']) - 1))
            par.merge(dist, dev)
        wall = dt
        if dist is not None:
            wall = _reduce(dist, dt, dist.ReduceOp.MAX, dev)
        msharded, msolve = mode
        return {
            'ms_fit_and_rate': round(wall * 1e3, 3), 'actions_per_s': round(total / wall, 1),
            'iterations': n_iter,
            'timing': f'median of {nreps} calls (wall clock around each, after a warm-up call; '
                      f'min {min(times) * 1e3:.3f}, max {max(times) * 1e3:.3f} ms on rank {rank})'
                      + ('; max over ranks' if dist is not None else ''),
            'solve': (('band-sharded (all-to-all of counted actions, '
                       + ('compact rows all-gathered once, replicated iteration)' if msolve == 'compact'
                          else 'row-sharded iteration)'))
                      if (msharded and dist is not None) else
                      ('replicated (one all-reduce of the dense counts)' if dist is not None else
                       'one GPU (compact count rows only, no dense table)')),
            'phases_ms': dict(phases, note='one extra call synchronised between phases (rank '
                              f'{rank}): count = band buckets + table; exchange = the counts\' '
                              'all-reduce (band-sharded: count and exchange inside solve); '
                              'solve = normalise + value '
                              'iteration incl. its host syncs; rate (the timed calls with one GPU '
                              'or the replicated solve run solve + rate as one call, the rate '
                              'queued behind the solve before its host round trip)'),
            'phase_events_ms': dict(events, note=f'HIP events around each phase of one more call '
                                    f'(rank {rank}; current stream, the collectives ordered on it)'),
            **({'exchange': {k: v for k, v in dict(xstats, rank=rank).items() if k != 'timer'}}
               if (msharded and dist is not None and xstats) else {}),
            'solve_path': path[0] + (' (one launch, rows summed in a fixed parallel order under '
                                     'an error bound that keeps every convergence decision)'
                                     if path[0] == 'reordered' else ''),
            **({'parity': dict(par.record(),
                               surface_tolerance=('bit-exact' if rtol == 0 else
                                                  f'{rtol:g} relative, iteration count exact'),
                               surface_max_rel_err=float(f"{getattr(par, 'surface_rel_err', 0.0):.3e}"))}
               if check else {})}

    main = run((sharded, solve), reps)
    games = (f'{cfg5_games:,} synthetic games over {world} rank(s)' if cfg5_games > 0 else
             'the step batch')
    out = {'workload': f'cfg5: xT 105x68 fit (count + all-reduce + value iteration) + '
                       f'rate(use_interpolation=True) of {games}',
           'actions_per_gpu': n, 'actions_total': total,
           'scaling': 'strong' if cfg5_games > 0 else 'weak',
           'pipeline': 'band-owned count (per batch: one key per counted action, bucketed by '
                       'start-cell band; the 7140^2 table written once, no global atomics) '
                       'writing each action\'s 8-B interpolated-rate operand; value iteration '
                       'over the compact count rows; rate from the operands (LDS surface)',
           **main}
    if dist is not None and sharded:
        # north_star's all-reduce-only scheme beside the band-sharded default, on the same
        # batches: the departure is judged by measurement
        out['compare_replicated'] = run((False, 'compact'), max(5, reps // 3))
    return out


def rotate_extra(args, dist, dev, d, ps, pc, inp, step, n, total_actions, world) -> dict:
    """The headline step over ``--rotate`` K device copies of the batch (inputs and
    probabilities at other addresses), used in turn: no step finds its inputs left in the 256 MB
    Infinity Cache by the step before it, as a stream of fresh batches would not (the main
    line's steps re-value one batch, whose id / team columns the bool pass then reads from the
    Infinity Cache).  Same outputs, same buffers; timed like the main loop."""
    K = int(args.rotate)
    sets = [(inp['s'], inp['ps'], inp['pc'])]
    keep = []
    for _ in range(K - 1):
        b = B.ActionBatch.from_columns(d, dev=dev)
        keep.append(b)
        sets.append((b.struct(), ps.clone(), pc.clone()))
    first = dict(inp)

    def use(k):
        inp['s'], inp['ps'], inp['pc'] = sets[k % K]
    for k in range(max(args.warmup, K)):
        use(k)
        step()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        use(k)
        step()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    wall = time.perf_counter() - t0
    if dist:
        wall = _reduce(dist, wall, dist.ReduceOp.MAX, dev)
    inp.update(first)
    ms = wall / args.steps * 1e3
    return {'batches': K, 'ms_per_step': round(ms, 4),
            'value': round(total_actions * args.steps / wall, 1),
            'step_frac': round(STEP_BYTES * total_actions / (ms * 1e-3) / (world * HBM_PEAK_GBS * 1e9), 4),
            'what': f'the step over {K} device copies of the batch in turn (inputs at other '
                    'addresses each step: none left in the Infinity Cache by the step before); '
                    'not the headline value'}


def convert_extra(d, dist, dev, reps: int = 3) -> dict:
    """SURVEY §8(f) row 1 alongside the main line: SPADL -> Atomic-SPADL conversion of this
    rank's cfg2 games on device (count + scan + emit), then Atomic-VAEP features + labels on
    the converted rows without leaving HBM (the producer of cfg3's input)."""
    from socceraction_amd.atomic.spadl import base as cb
    frame = cb.SpadlFrame.from_columns(d, dev=dev)
    out = cb.convert_device(frame)  # warm-up
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        out = cb.convert_device(frame)
    torch.cuda.synchronize()
    ms_conv = (time.perf_counter() - t0) / reps * 1e3
    ab = out.to_batch(frame, d['home_team_id'])
    fo = ops.features(ab, ATOMIC_DEFAULT, 3, bool_tile=1024, num_tile=128)
    lab = ops.labels(ab)

    def step():
        ops.features(ab, ATOMIC_DEFAULT, 3, out=fo)
        ops.labels(ab, 10, lab)
    ms_feat = _events_ms(step, reps)
    n_in, n_out = frame.n, out.n
    # count pass reads the 60-B input row (and its successor, cache-resident); emit reads it
    # again and writes 59 B per atomic row
    conv_bytes = 2 * 60 * n_in + 59 * n_out
    return {'workload': 'SPADL -> Atomic-SPADL conversion (count + scan + emit) of the cfg2 '
                        'games, then Atomic-VAEP features + labels on device',
            'spadl_actions_per_gpu': n_in, 'atomic_actions_per_gpu': n_out,
            'ms_convert_incl_host_sync': round(ms_conv, 4),
            'convert_GBs': round(conv_bytes / ms_conv * 1e-6, 1),
            'ms_atomic_features_labels': round(ms_feat, 4),
            'spadl_actions_per_s_end_to_atomic_features': round(n_in / (ms_conv + ms_feat) * 1e3, 1)}


def rate_extra(ab, out, n, dev, reps: int = 5) -> dict:
    """VAEP.rate fully on device alongside the main line: the features already computed by
    the main step feed two xgboost-shaped learners (100 trees, depth 3: the reference's default
    XGBClassifier, vaep/base.py:226-231; random splits, xgboost is not installed) evaluated on
    the feature blocks, then formula.value on their float32 probabilities."""
    from socceraction_amd import trees
    kinds = [k for _, k, _ in out.plan.order]
    models = [trees.TreeEnsemble.from_xgboost_json(
        trees.synthetic_xgboost_json(len(kinds), n_trees=100, depth=3, seed=s, feature_kinds=kinds))
        for s in (1, 2)]
    # VAEP.rate's features for xgboost learners: the bool features as bitmaps and the numeric
    # features in float32 (what the staged walk reads); the float64 numeric form beside it
    fbits = ops.features(ab, SPADL_DEFAULT, 3, num_tile=out.Rn, bool_bits=True, num32=True)
    ps = models[0].predict_blocks(fbits)
    pc = models[1].predict_blocks(fbits)
    val = torch.empty((3, (n + 15) // 16 * 16), dtype=torch.float32, device=dev)
    ms_feat = _events_ms(lambda: ops.features(ab, SPADL_DEFAULT, 3, out=fbits), reps)
    ms_tree = _events_ms(lambda: models[0].predict_blocks(fbits, out=ps), reps)
    # VAEP.rate's default for xgboost learners: the split conditions evaluated in the feature
    # passes (sa_vaep_features_conditions), both walks over bitmaps only
    from socceraction_amd import trees as T
    ms_cond = _events_ms(lambda: T.predict_pair_conditions(ab, out.plan, models), reps)
    prep, cbits, words = T.condition_bitmaps(ab, out.plan, models)
    ms_cond_feat = _events_ms(lambda: T.condition_bitmaps(ab, out.plan, models, bits=cbits), reps)
    ms_cond_walk = [_events_ms(lambda k=k: T.walk_conditions(prep, k, models[k], cbits, words, n, dev,
                                                             out=ps), reps) for k in range(2)]
    cond_counts = {'union': prep['n_cond_union'], 'per_model': [w[5] for w in prep['walks']]}
    del cbits
    f64bits = ops.features(ab, SPADL_DEFAULT, 3, num_tile=out.Rn, bool_bits=True)
    ms_feat64 = _events_ms(lambda: ops.features(ab, SPADL_DEFAULT, 3, out=f64bits), reps)
    ms_tree64 = _events_ms(lambda: models[0].predict_blocks(f64bits, out=ps), reps)
    del f64bits
    ms_block = _events_ms(lambda: models[0].predict_blocks(out, out=ps), reps)
    ms_gather = _events_ms(lambda: models[0].predict_blocks(out, out=ps, method='gather'), reps)
    ms_formula = _events_ms(lambda: ops.formula(ab, ps, pc, val), reps)
    del fbits
    return {'workload': 'VAEP.rate on device: the feature passes + 2 x xgboost-shaped tree '
                        'ensembles (100 trees, depth 3) + formula (float32 probabilities), cfg2 '
                        'actions',
            'method': 'VAEP.rate default (vaep/base.py): the split conditions evaluated inside the '
                      'feature passes as bitmaps (sa_vaep_features_conditions), then one staged '
                      'walk per learner over the condition bitmaps only',
            'ms_features_conditions': round(ms_cond_feat, 4),
            'ms_per_model': [round(x, 4) for x in ms_cond_walk],
            'conditions': cond_counts,
            'ms_features_and_both_models': round(ms_cond, 4),
            'ms_formula_f32': round(ms_formula, 4),
            'ms_rate_total': round(ms_cond + ms_formula, 4),
            'actions_per_s_rate': round(n / (ms_cond + ms_formula) * 1e3, 1),
            'staged_walk_over_feature_blocks': {
                'what': 'the other tree path (sa_tree_predict_staged over the bool bitmaps and '
                        'the numeric blocks: VAEP.rate for learners whose splits are not xgboost float32 `<` '
                        'conditions, or whose conditions do not fit the condition bitmaps)',
                'ms_features_bitmap_form': round(ms_feat, 4), 'ms_per_model': round(ms_tree, 4),
                'ms_features_bitmap_f64_form': round(ms_feat64, 4),
                'ms_per_model_f64_numeric': round(ms_tree64, 4),
                'ms_per_model_from_bool_block': round(ms_block, 4),
                'ms_per_model_gather_walk': round(ms_gather, 4),
                'ms_rate_total': round(ms_feat + 2 * ms_tree + ms_formula, 4)}}


def link_rates(nbytes: int = 1 << 30, reps: int = 3) -> dict:
    """The host link measured in-process: pinned D2H and H2D of ``nbytes`` (best of ``reps``)."""
    dev = torch.empty(nbytes, dtype=torch.uint8, device='cuda')
    host = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
    out = {}
    for name, dst, src in (('d2h', host, dev), ('h2d', dev, host)):
        t = []
        for _ in range(reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            dst.copy_(src, non_blocking=True)
            torch.cuda.synchronize()
            t.append(time.perf_counter() - t0)
        out[f'{name}_GBs'] = round(nbytes / min(t) / 1e9, 2)
    del dev, host
    return out


def e2e_extra(d, games: int, reps: int = 3) -> dict:
    """End to end through the pandas drop-in, the way a notebook would call the batched API
    (SURVEY §8(d) "report end-to-end separately"): actions DataFrame in -> H2D -> features +
    labels + formula kernels -> D2H -> reference-shaped DataFrames out, for the first ``games``
    games of the step's batch (a bounded sample: the 16M x 568 frame of the whole batch is
    15 GB of host memory).  The headline is ``VAEP.compute_batch`` (one encode, game-aligned
    chunks, pitched DMAs out of two device slots while the host encodes the next chunk:
    socceraction_amd.pipeline) against the measured pinned D2H rate; the three separate
    batched calls are timed beside it."""
    from socceraction_amd import vaep
    from socceraction_amd.batch import ActionBatch
    off = d['game_off']
    m = int(off[games])
    sub = {k: (v[:m] if isinstance(v, np.ndarray) and v.shape == d['type_id'].shape else v)
           for k, v in d.items()}
    sub['game_off'] = off[:games + 1]
    sub['home_team_id'] = d['home_team_id'][:games]
    actions = synthetic.to_frame(sub)
    gframe = synthetic.games_frame(sub)
    p = synthetic.probabilities(m)
    model = vaep.VAEP()
    home_of = gframe.set_index('game_id')['home_team_id']
    import pandas as pd

    def separate():
        t = [time.perf_counter()]
        X = model.compute_features_batch(gframe, actions)
        t.append(time.perf_counter())
        Y = model.compute_labels_batch(gframe, actions)
        t.append(time.perf_counter())
        ab = ActionBatch.from_frame(actions, home_team_id=home_of, segments='game')
        v = ops.formula(ab, torch.from_numpy(p['scores']).to(ab.device),
                        torch.from_numpy(p['concedes']).to(ab.device)).cpu().numpy()[:, :m]
        V = pd.DataFrame({'offensive_value': v[0], 'defensive_value': v[1], 'vaep_value': v[2]})
        t.append(time.perf_counter())
        assert X.shape == (m, 568) and Y.shape == (m, 2) and len(V) == m
        return np.diff(t)

    def pipelined():
        t0 = time.perf_counter()
        X, Y, V = model.compute_batch(gframe, actions, p['scores'], p['concedes'])
        dt = time.perf_counter() - t0
        assert X.shape == (m, 568) and Y.shape == (m, 2) and len(V) == m
        return dt
    separate()  # warm-up (pinned buffers, first launches)
    pipelined()
    best = min((separate() for _ in range(reps)), key=lambda x: x.sum())
    tp = min(pipelined() for _ in range(reps))
    link = link_rates()
    # bytes over the link per action: features (515 bool + 53 x 8) + 3 label bytes + 3 x 8
    # formula bytes out, the encoded columns in (5 x 8 f64 + 4 u8 + 4 B team)
    d2h_bpa, h2d_bpa = 515 + 53 * 8 + 3 + 24, 48
    moved = m * (d2h_bpa + h2d_bpa)
    return {'workload': f'pandas in -> pandas out: features + labels + formula values of {games} '
                        'games (H2D, kernels, D2H, DataFrame assembly; bounded sample of the step '
                        'batch) through VAEP.compute_batch, the pipelined batched call',
            'actions': m, 'seconds': round(tp, 4), 'actions_per_s': round(m / tp, 1),
            'link': dict(link, note='pinned 1 GiB copies, best of 3, in this process'),
            'bytes_per_action': {'d2h': d2h_bpa, 'h2d': h2d_bpa},
            'link_GBs_achieved': round(moved / tp / 1e9, 2),
            'frac_of_link': round(m * d2h_bpa / tp / 1e9 / link['d2h_GBs'], 3),
            'frac_note': 'D2H bytes of the call / its wall time / the measured pinned D2H rate '
                         '(the H2D bytes travel the other direction at the same time)',
            'separate_calls': {
                'what': 'compute_features_batch + compute_labels_batch + formula (each encodes the '
                        'frame again)',
                'seconds': round(float(best.sum()), 4),
                'actions_per_s': round(m / float(best.sum()), 1),
                'split_seconds': {'features_frame': round(float(best[0]), 4),
                                  'labels_frame': round(float(best[1]), 4),
                                  'formula_frame': round(float(best[2]), 4)}}}


def reference_cpu_record() -> dict:
    """The reference's own CPU path (pandas), timed by scripts/time_reference.py in the BUILD
    container (the reference never travels): profiles/reference_cpu.json, or None."""
    path = os.path.join(ROOT, 'profiles', 'reference_cpu.json')
    if not os.path.exists(path):
        return None
    with open(path) as f:
        rec = json.load(f)
    return {'value': rec['one_process']['actions_per_s'], 'unit': 'actions/s', 'cores': 1,
            'kind': 'reference',
            'pool': {'value': rec['pool']['actions_per_s'], 'processes': rec['pool']['processes']},
            'step_one_process_with_xt_16x12': rec.get('step_one_process_actions_per_s'),
            'where': f"build container ({rec['host']['cpu']}, {rec['host']['os_cpu_count']} "
                     'vCPU), not the GPU host: the reference never travels',
            'sample': rec['workload'], 'source': 'profiles/reference_cpu.json '
                                                 '(scripts/time_reference.py)'}


def cpu_baseline(d, seconds: float) -> dict:
    """The oracle port (numpy, 1 thread) on the GPU box's host, over whole games: VAEP features
    + labels + formula per game, then the xT 16x12 fit + rate over the games done."""
    from oracle import vaep_oracle as vo
    from oracle import xt_oracle as xo
    p = synthetic.probabilities(int(d['game_off'][-1]))
    off = d['game_off']
    names = ('period_id', 'time_seconds', 'team_id', 'start_x', 'start_y', 'end_x', 'end_y',
             'type_id', 'result_id', 'bodypart_id')
    done, games, t0 = 0, 0, time.perf_counter()
    while games < len(off) - 1 and time.perf_counter() - t0 < seconds:
        s, e = int(off[games]), int(off[games + 1])
        cols = {c: d[c][s:e] for c in names}
        vo.features(cols, 3, vo.SPADL_DEFAULT, home=[d['home_team_id'][games]])
        vo.labels(cols)
        vo.formula(cols, p['scores'][s:e], p['concedes'][s:e])
        done += e - s
        games += 1
    # xT 16x12 fit + rate over the same sample (the step's second half)
    e = int(off[games])
    cols = {c: d[c][:e] for c in names}
    fit = xo.fit(cols, 16, 12)
    xo.rate(cols, fit['xT'])
    dt = time.perf_counter() - t0
    return {'value': round(done / dt, 1), 'unit': 'actions/s', 'cores': 1, 'kind': 'port',
            'sample': f'{games} synthetic games ({done} actions) of the same workload (VAEP per '
                      f'game + xT 16x12 fit + rate), numpy oracle, 1 thread, {dt:.1f} s'}


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    # 50 timed steps by default: the last step's xT fit + rate (~0.5 ms on the side stream) is
    # the one part of the pipeline no later step hides; over 20 steps it added ~10 us per step
    # (profiles/r05w_steps_ab.log), over 50 about 4
    ap.add_argument('--steps', type=int, default=50)
    ap.add_argument('--warmup', type=int, default=3)
    ap.add_argument('--games', type=int, default=10000, help='games per GPU (cfg2: 10k)')
    ap.add_argument('--cpu-seconds', type=float, default=15.0)
    ap.add_argument('--rotate', type=int, default=2,
                    help='also time the step over K device copies of the batch in turn (K >= 2; '
                         '0: skip): the figure without cross-step Infinity Cache reuse')
    ap.add_argument('--e2e-games', type=int, default=1000,
                    help='games of the end-to-end (pandas in -> pandas out) side entry (0: skip)')
    ap.add_argument('--no-cpu', action='store_true')
    ap.add_argument('--no-check', action='store_true',
                    help='dev A/B only: skip the parity check of the timed buffers (the line '
                         'then carries no "parity" field)')
    ap.add_argument('--no-side', action='store_true',
                    help='skip the cfg3 (atomic) and cfg5 (xT 105x68) side measurements')
    ap.add_argument('--cfg5-games', type=int, default=62500,
                    help='games of the cfg5 side entry (BASELINE cfg5: 62,500 = 1.0e8 actions, '
                         'split over the ranks; 0 = the step batch)')
    ap.add_argument('--cfg5-solve', default='auto', choices=('auto', 'sharded', 'sharded-rows', 'replicated'),
                    help='cfg5 with N > 1: "sharded" = each rank counts its own start-cell bands '
                         'after ONE all-to-all of the counted actions, then one all-gather of the '
                         'compact count rows and the iteration on every rank '
                         '(shard.xt_fit_bands_sharded); "sharded-rows" = the same count, each rank '
                         'iterating its own rows with an all-gather of x per iteration; '
                         '"replicated" = one all-reduce of the 204 MB count table and the whole '
                         'solve on every rank; auto = sharded (the projection in DESIGN.md §6)')
    ap.add_argument('--xt-sharded', action='store_true', help='same as --cfg5-solve sharded')
    ap.add_argument('--atomic-games', type=int, default=10000,
                    help='atomic games of the cfg3 side entry, split over the ranks (BASELINE '
                         'cfg3: 10,000 = 4.0e7 atomic actions)')
    ap.add_argument('--serial', action='store_true',
                    help='run the xT fit + rate after the VAEP kernels on the same stream '
                         '(default: on a side stream, overlapped)')
    ap.add_argument('--xt-fork', type=int, default=-1,
                    help='overlapped mode: VAEP calls enqueued before the side stream forks for '
                         'the xT count pass (-1: right after num_features with --xt-source cells, '
                         'else 0)')
    ap.add_argument('--bool-tile', type=int, default=1024,
                    help='rows per bool-block tile (0 = one tile: plain column-major)')
    ap.add_argument('--order', default='bool_features,num_step',
                    help='launch order of the VAEP kernels in the step (default bool first: the xT '
                         'count, solve and rate of step k then run on the side stream beside step '
                         'k+1\'s bool pass, 2.955 - 2.970 vs 2.975 - 2.993 ms with num first and '
                         'the count on the main stream, profiles/r03_numeric_pass_ab.md); num_step = the numeric '
                         'pass with goalscore, labels and the f64 formula in it (sa_vaep_step_f64; '
                         '3.115 vs 3.195 ms, profiles/r02u_goalscore_fused_ab.md); num_features = '
                         'the numeric pass with goalscore; num_features_nogs + goalscore: the '
                         'separate scan; labels_formula = labels + '
                         'formula in one launch (num first: 1.3 %% faster than bool first, '
                         'profiles/r01h_order_ab.log; fused tail 3.236 vs 3.244 ms, '
                         'profiles/r02_step_ab.md)')
    ap.add_argument('--xt-source', default='cells', choices=('cells', 'codes', 'coords'),
                    help='what the xT count + rate passes read: the cell codes the f64 feature '
                         'pass writes (4 B/action, default), or the coordinates (34 B/action; '
                         '"codes": the count pass writes 4-B rate operands for the rate)')
    ap.add_argument('--ab', default='',
                    help='dev tool: ";"-separated step variants "name:key=value/..." (keys xt, '
                         'order with "+", fork, prio) timed round-robin in one process')
    ap.add_argument('--side-priority', default='normal', choices=('normal', 'high'),
                    help='priority of the xT side stream (profiles/r02_step_ab.md)')
    ap.add_argument('--xt-count', default='main', choices=('main', 'side'),
                    help='where the xT count pass runs: on the main stream right after '
                         'num_features in its one-workgroup-per-CU shape (default: 3.19 - 3.24 vs '
                         '3.24 - 3.31 ms per step, profiles/r02_step_ab.md), or on the side stream')
    ap.add_argument('--num-tile', type=int, default=128,
                    help='rows per f64/i64-block tile (0 = one tile: plain column-major)')
    ap.add_argument('--event-every', type=int, default=10,
                    help='per-launch HIP events on every Nth timed step (1 = every step); the '
                         'kernels\' mean durations come from those steps')
    ap.add_argument('--events', default='native', choices=('native', 'torch'),
                    help='event kind of the step\'s stream forks / joins and per-kernel timings: '
                         'native = sa_event_* without the system-scope fence (default), torch = '
                         'torch.cuda.Event')
    ap.add_argument('--alloc-order', default='contig',
                    choices=('contig', 'contig-all', 'bool-first', 'num-first', 'single', 'single-bool-first'),
                    help='output blocks: contig = the bool block in physically contiguous VRAM '
                         '(default; profiles/r02u_goalscore_fused_ab.md r02aq - r02au), else '
                         'placement A/B knobs (bool-first = three caching-allocator blocks)')
    args = ap.parse_args()
    EVENTS['kind'] = args.events
    if args.gpus < 1:
        raise SystemExit('--gpus must be >= 1')
    if 'WORLD_SIZE' not in os.environ and args.gpus > 1:
        raise SystemExit(launch_ranks(args.gpus, sys.argv[1:]))
    check_world(args.gpus)

    dist, rank, world = _dist()
    dev = B.device()
    d = synthetic.spadl_games(args.games, game_id0=rank * args.games)
    ab = B.ActionBatch.from_columns(d, dev=dev)
    n = ab.n
    plan = catalog.build_plan(SPADL_DEFAULT, 3)
    if args.alloc_order in ('contig', 'contig-all'):  # the bool block (or all three) in contiguous VRAM
        out = ops.alloc_feature_blocks(plan, n, dev, bool_tile=args.bool_tile or None,
                                       num_tile=args.num_tile or None,
                                       contiguous='all' if args.alloc_order == 'contig-all' else True)
    elif args.alloc_order in ('num-first', 'single', 'single-bool-first'):  # dev knob: block placement A/B
        Rb, Rn = args.bool_tile or (n + 15) // 16 * 16, args.num_tile or (n + 15) // 16 * 16
        shapes = [((-(-n // Rn), plan.n_f64, Rn), torch.float64), ((-(-n // Rn), plan.n_i64, Rn), torch.int64),
                  ((-(-n // Rb), plan.n_bool, Rb), torch.uint8)]
        if args.alloc_order.startswith('single'):  # one allocation, the three blocks carved from it
            if args.alloc_order == 'single-bool-first':
                shapes = shapes[2:] + shapes[:2]
            sizes = [int(np.prod(sh)) * torch.tensor([], dtype=dt).element_size() for sh, dt in shapes]
            offs = np.cumsum([0] + [-(-z // 4096) * 4096 for z in sizes])
            arena = torch.empty(int(offs[-1]), dtype=torch.uint8, device=dev)
            blks = [arena[int(o):int(o) + z].view(dt).view(sh) for o, z, (sh, dt) in zip(offs, sizes, shapes)]
            fblk, iblk, bblk = blks[1:] + blks[:1] if args.alloc_order == 'single-bool-first' else blks
        else:
            fblk, iblk, bblk = [torch.empty(sh, dtype=dt, device=dev) for sh, dt in shapes]
        out = ops.FeatureBlocks(plan, n, Rb, Rn, bblk, fblk, iblk)
    else:
        out = ops.alloc_feature_blocks(plan, n, dev, bool_tile=args.bool_tile or None,
                                       num_tile=args.num_tile or None)
    ld = (n + 15) // 16 * 16

    def sub(keep):  # the same block layout with only some column families launched ('g': goalscore)
        q = copy.copy(plan)
        q.struct = copy.deepcopy(plan.struct)
        for x in range(len(q.struct.bool_col)):
            if 'b' not in keep:
                q.struct.bool_col[x] = -1
            if 'f' not in keep:
                q.struct.f64_col[x] = -1
            if 'i' not in keep or (x == XFN['goalscore'] and 'g' not in keep):
                q.struct.i64_col[x] = -1
        return ops.FeatureBlocks(q, n, out.Rb, out.Rn, out.bool_block, out.f64_block,
                                 out.i64_block)

    bool_out, num_out, num_nogs = sub('b'), sub('fig'), sub('fi')
    p = synthetic.probabilities(n)
    ps = torch.from_numpy(p['scores']).to(dev)
    pc = torch.from_numpy(p['concedes']).to(dev)
    lab_buf = torch.empty((3, ld), dtype=torch.uint8, device=dev)
    lab = ops.LabelBlocks(n, lab_buf[0], lab_buf[1], None)
    val = torch.empty((3, ld), dtype=torch.float64, device=dev)
    # the step's inputs (--rotate swaps in other device copies of the same batch between steps)
    inp = {'s': ab.struct(), 'ps': ps, 'pc': pc}
    # two cell-code buffers used by alternate steps: with the xT side stream of step k still
    # rating from its codes while step k+1's numeric pass writes the other buffer (pipelined)
    ring = {'bufs': [ops.xt_cells_buffer(n, dev), ops.xt_cells_buffer(n, dev)], 'k': 0, 'done': [None, None]}

    def cells():
        return ring['bufs'][ring['k']]
    main_s = torch.cuda.current_stream()
    overlap = not args.serial
    # the xT side stream; --side-priority high: a high-priority HIP stream, so its few
    # workgroups are dispatched ahead of the VAEP kernels' as CUs free up
    sides = {p: (torch.cuda.Stream(priority=-1 if p == 'high' else 0) if overlap else main_s)
             for p in ('normal', 'high')}
    par_s = torch.cuda.Stream()

    def make_step(spec):
        """One step of the given variant: the VAEP kernels in `order` on the main stream; the xT
        fit + rate on a side stream forked before VAEP call `fork` (after num_features at the
        latest when the feature pass writes the xT cell codes), joined at the end."""
        xt, order, fork = spec['xt'], spec['order'], spec['fork']
        side = sides[spec['prio']]
        covered = sorted(c for k in order for c in FUSED_CALLS.get(k, (k,)))
        if covered != sorted(STEP_CALLS) and not int(spec.get('diag', 0)):  # diag=1: A/B probes only
            raise SystemExit(f'order must cover {",".join(STEP_CALLS)} once each '
                             f'(fused entries: {FUSED_CALLS})')
        if xt == 'cells' and overlap and fork <= _num_index(order):
            raise SystemExit('xt=cells: the side stream forks after num_features')
        by_name = {'bool_features': lambda: ops.features_into(inp['s'], bool_out),
                   'num_features': (lambda: ops.features_into(inp['s'], num_out,
                                                              xt_cells=(16, 12, cells())))
                   if xt in ('cells', 'none') else (lambda: ops.features_into(inp['s'], num_out)),
                   'num_features_nogs': (lambda: ops.features_into(inp['s'], num_nogs,
                                                                   xt_cells=(16, 12, cells())))
                   if xt in ('cells', 'none') else (lambda: ops.features_into(inp['s'], num_nogs)),
                   'goalscore': lambda: ops.goalscore_into(ab, out),
                   'labels': lambda: ops.labels(ab, 10, lab),
                   'formula': lambda: ops.formula(ab, ps, pc, val),
                   'labels_formula': lambda: ops.labels_formula(ab, ps, pc, 10, lab, val),
                   'num_step': lambda: ops.step_into(inp['s'], num_out, inp['ps'], inp['pc'], 10, lab, val,
                                                     xt_cells=(16, 12, cells()) if xt in ('cells', 'none')
                                                     else None, chunk_rows=chunk, prefetch=pf)}
        # chunk / pf (A/B probe, sa_vaep_step_f64_chunked): the numeric pass in launches of chunk
        # rows, each after a pure-read pass pulling its inputs into the Infinity Cache (pf = 1)
        chunk, pf = int(spec.get('chunk', 0)), bool(int(spec.get('pf', 0)))
        calls = tuple(by_name[k] for k in order)
        # cm=1: the count pass runs on the main stream right after num_features, in the fast
        # one-workgroup-per-CU shape; the side stream takes the all-reduce, solve and rate
        cm = int(spec.get('cm', 0)) and overlap
        xt_start, xt_finish, xt_last = xt_step(ab, dist, xt, cells, shared=overlap and not cm,
                                               sync_solve=bool(int(spec.get('xsync', 0))))
        nv = len(calls)
        # par=1 (A/B only): bool_features on its own stream, concurrent with the calls before it
        par = int(spec.get('par', 0)) and 'bool_features' in order
        ib = order.index('bool_features') if par else -1

        pipe = int(spec.get('pipe', 1)) and overlap
        ek = spec.get('ev', EVENTS['kind'])  # event kind of this variant

        def step(ev=None):
            # ev[i] = (start, end) of VAEP call i on the main stream, ev[nv] = the xT side
            # stream's span (count pass + all-reduce, then solve -- a host sync of the side
            # stream -- and rate); --serial: everything on the one stream
            pj = None
            if pipe and ring['done'][ring['k']] is not None:
                # this step's cell-code buffer was last read by the xT rate two steps ago
                ring['done'][ring['k']].wait(main_s)
            # zero the xT counts on the side stream (idle until the fork) while the first VAEP
            # call runs; the count pass waits for it
            zs = side if overlap else main_s
            if cm and overlap and fork < nv:  # the count runs on the main stream: after its last use
                _record(main_s, ek).wait(zs)
            with torch.cuda.stream(zs):  # (else the side stream's own order covers the counts)
                xt_start.zero()
            zev = _record(zs, ek)
            if par:
                _record(main_s, ek).wait(par_s)
                with torch.cuda.stream(par_s):
                    calls[ib]()
                pj = _record(par_s, ek)
            for i, call in enumerate(calls):
                if overlap and i == fork:
                    if cm:  # the count pass on the main stream; its all-reduce on the side
                        if ev is not None:
                            ev[nv][0].record(main_s)
                        zev.wait(main_s)
                        xt_start.count()
                    _record(main_s, ek).wait(side)
                    with torch.cuda.stream(side):
                        if ev is not None and not cm:
                            ev[nv][0].record(side)
                        if cm:
                            xt_start.reduce()
                        else:
                            xt_start()
                if par and i == ib:
                    pj.wait(main_s)
                    continue
                if ev is not None:
                    if i > 0 and not (overlap and i == fork) and not par:
                        ev[i][0] = ev[i - 1][1]  # back to back on the main stream: one event
                    else:
                        ev[i][0].record(main_s)
                call()
                if ev is not None:
                    ev[i][1].record(main_s)
            if not overlap or fork >= nv:  # serial, or forked after the last VAEP call
                _record(main_s, ek).wait(side if overlap else main_s)
                with torch.cuda.stream(side):
                    if ev is not None:
                        ev[nv][0].record(side)
                    xt_start()
            with torch.cuda.stream(side):
                xt_finish()
                if ev is not None:
                    ev[nv][1].record(side)
            if pipe:  # pipelined: the xT work of this step overlaps the next step's passes
                ring['done'][ring['k']] = _record(side, ek)
                ring['k'] ^= 1
            elif overlap:
                _record(side, ek).wait(main_s)
        step.ev_kind = ek
        return step, xt_last

    base = {'xt': args.xt_source, 'order': args.order.split(','), 'fork': args.xt_fork,
            'prio': args.side_priority, 'cm': int(args.xt_count == 'main')}
    if base['fork'] < 0:  # default: before the first VAEP call, or right after num_features
        base['fork'] = (_num_index(base['order']) + 1) if args.xt_source == 'cells' else 0
    if args.ab:  # in-process A/B of step variants on the same allocations (dev tool)
        # ";"-separated "name:key=value/key=value" with keys xt, order (names joined by "+"), fork
        variants = {}
        for spec in args.ab.split(';'):
            name, _, opts = spec.partition(':')
            v = dict(base)
            for kv in [o for o in opts.split('/') if o]:
                k_, _, v_ = kv.partition('=')
                v[k_] = v_.split('+') if k_ == 'order' else (int(v_) if k_ in ('fork', 'par', 'cm', 'diag', 'xsync', 'pipe', 'tev', 'chunk', 'pf') else v_)
            variants[name] = (make_step(v)[0], v['order'])
        ab_ms = {k: [] for k in variants}
        ab_kern = {}
        for fn, _ in variants.values():
            for _ in range(args.warmup):
                fn()
        for _ in range(4):
            for k, (fn, _) in variants.items():
                fn()
                torch.cuda.synchronize()
                t = time.perf_counter()
                for _ in range(args.steps):
                    fn()
                torch.cuda.synchronize()
                ab_ms[k].append(round((time.perf_counter() - t) / args.steps * 1e3, 4))
        for k, (fn, vorder) in variants.items():  # per-call HIP event means, one more round
            evs = [[[_event(True, fn.ev_kind), _event(True, fn.ev_kind)]
                    for _ in range(len(vorder) + 1)] for _ in range(args.steps)]
            for e in evs:
                fn(e)
            torch.cuda.synchronize()
            ab_kern[k] = {c: round(float(np.mean([e[i][0].elapsed_time(e[i][1]) for e in evs])), 4)
                          for i, c in enumerate(list(vorder) + ['xt_side'])}
        if rank == 0:
            print(json.dumps({'ab_ms_per_step': ab_ms, 'ab_kernel_ms': ab_kern, 'n': n}), flush=True)
        return
    step, xt_last = make_step(base)
    order = base['order']
    nv = len(order)
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    evs = [[[_event(True), _event(True)] for _ in range(nv + 1)] for _ in range(args.steps)]
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    # per-launch HIP events on every `--event-every`-th step of the timed region (each record is
    # a marker between the kernels; the step's own launches keep their back-to-back order on the
    # other steps): the kernels' mean durations are the mean over the sampled steps
    sampled = [k for k in range(args.steps) if k % max(1, args.event_every) == 0]
    for k in range(args.steps):
        step(evs[k] if k in sampled else None)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    wall = time.perf_counter() - t0
    evs = [evs[k] for k in sampled]
    kern = {name: float(np.mean([e[i][0].elapsed_time(e[i][1]) for e in evs]))
            for i, name in enumerate(order)}
    kern['xt_fit_rate'] = float(np.mean([e[nv][0].elapsed_time(e[nv][1]) for e in evs]))
    total_actions = n
    if dist:
        wall = _reduce(dist, wall, dist.ReduceOp.MAX, dev)
        total_actions = int(_reduce(dist, n, dist.ReduceOp.SUM, dev))
    check = not args.no_check
    par = Parity()
    if check:  # outside the timed region: the last timed step's own buffers vs the oracle
        tc = time.perf_counter()
        check_vaep(par, d, out, lab_buf[0], lab_buf[1], val, p)
        if base['xt'] in ('cells', 'codes', 'coords'):
            sol = xt_last['sol']
            cnt = oracle_counts(d, 16, 12, dist, dev)
            xT_ref = check_xt(par, cnt, xt_last['acc_buf'], sol.mats[3], _iterations(sol), 16, 12)
            check_xt_rate(par, d, xt_last['rate'], xT_ref)
        par.merge(dist, dev)
        check_s = time.perf_counter() - tc
    rotate = None
    if args.rotate >= 2:  # the same step over K device copies of the batch, one per step in turn
        rotate = rotate_extra(args, dist, dev, d, ps, pc, inp, step, n, total_actions, world)
    extra_side = {}

    def side(name, fn):
        """A side entry never takes the main line down with it: an exception is reported in its
        place (and on stderr); its parity failures still fail the run below."""
        try:
            extra_side[name] = fn()
        except Exception as e:  # noqa: BLE001  (reported, not hidden)
            import traceback
            traceback.print_exc()
            extra_side[name] = {'error': f'{type(e).__name__}: {e}'}
    if not args.no_side:
        # cfg3 first: its bool block wants a physically contiguous range, which cfg5's ~1e8
        # actions of device batches (allocated and freed by its entry) would fragment
        side('atomic_cfg3', lambda: atomic_extra(dist, rank, world, dev, args.atomic_games, check=check))
        torch.cuda.empty_cache()
        cfg5_sharded = args.xt_sharded or args.cfg5_solve in ('auto', 'sharded', 'sharded-rows')
        side('xt105_cfg5', lambda: xt105_extra(ab, dist, dev, cfg5_sharded, args.cfg5_games, rank, world,
                                                args.games, d=d, check=check,
                                                solve='rows' if args.cfg5_solve == 'sharded-rows'
                                                else 'compact'))
        side('convert_to_atomic', lambda: convert_extra(d, dist, dev))
        side('rate_on_device', lambda: rate_extra(ab, out, n, dev))
        if args.e2e_games > 0 and rank == 0:
            side('end_to_end', lambda: e2e_extra(d, min(args.e2e_games, args.games)))
    side_ok = all(v.get('parity', {}).get('ok', True) for v in extra_side.values())
    if rank != 0:
        if dist:
            dist.destroy_process_group()
        if not (par.ok and side_ok):
            print(f'bench.py rank {rank}: PARITY FAILED: ' + json.dumps(
                {'step': par.failures, **{k: v['parity']['failures'] for k, v in extra_side.items()
                                          if 'parity' in v}}), file=sys.stderr)
            raise SystemExit(3)
        return
    ms_per_step = wall / args.steps * 1e3
    value = total_actions * args.steps / wall
    bts = step_bytes(base['xt'])
    # the dominant kernel is the step's longest launch by measured HIP-event time; the xT side
    # stream's span overlaps other kernels and waits for CUs, so it gets no GB/s and no frac
    vaep = [k for k in KERNELS if k in kern and k != 'xt_fit_rate']
    dom = max(vaep, key=lambda k: kern[k])
    achieved = bts[dom] * n / (kern[dom] * 1e-3) / 1e9
    per_kernel = {k: {'ms': round(kern[k], 4), 'bytes_per_action': bts[k],
                      'achieved_GBs': round(bts[k] * n / (kern[k] * 1e-3) / 1e9, 1),
                      'frac': round(bts[k] * n / (kern[k] * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}
                  for k in vaep}
    traffic, traffic_src = None, 'no PMC record (profiles/pmc_dominant_kernel.json)'
    pmc = os.path.join(ROOT, 'profiles', 'pmc_dominant_kernel.json')
    lib_id = (_native.lib().sa_build_id() or b'').decode()
    if os.path.exists(pmc):
        with open(pmc) as f:
            rec = json.load(f)
        if rec.get('build_id') != lib_id:  # counted on another build: not this kernel's bytes
            traffic_src = (f"PMC record {rec.get('tag')} was counted on build "
                           f"{rec.get('build_id')}, not the loaded {lib_id}: traffic omitted")
        else:
            for k, v in rec.get('per_kernel', {}).items():
                if KERNEL_NAMES[dom] in k and v is not None:
                    traffic = round(v * n)
                    traffic_src = f"rocprofv3 PMC, record {rec.get('tag')}, build {lib_id}"
    line = {
        'metric': 'SPADL actions/sec valued (VAEP feat+labels+formula, xT fit+rate) at 1/2/4/8 GPUs',
        'value': round(value, 1), 'unit': 'actions/s', 'n_gpus': world, 'steps': args.steps,
        'warmup': args.warmup, 'ms_per_step': round(ms_per_step, 4), 'higher_is_better': True,
        'scaling': 'weak', 'vs_baseline': None, 'dtype': 'f64',
        'data': 'synthetic (seeded SPADL games, BASELINE cfg2 shape; inputs resident in HBM)',
        'config': {'workload': 'cfg2 + cfg4: 10k-game synthetic SPADL per GPU, VAEP '
                               'compute_features (k=3, default xfns, 568 cols) + compute_labels + '
                               'formula.value (f64), and xT 16x12 fit (counts all-reduced over '
                               'the ranks) + rate of the same actions',
                   'games_per_gpu': args.games, 'actions_per_gpu': n,
                   'feature_layout': f'tiled column-major: bool {out.Rb}, f64/i64 {out.Rn} rows '
                                     'per tile' + ('; bool block in physically contiguous VRAM'
                                                   if getattr(out, '_arena', None) is not None else ''),
                   'parallelism': f'games sharded over {world} GPU(s)'},
        'kernels': per_kernel,
        'kernel_events': f'HIP events around each launch on {len(evs)} of the {args.steps} timed steps '
                         f'(every {max(1, args.event_every)}th)',
        'roofline': {'bound': 'hbm', 'achieved': round(achieved, 1), 'peak': HBM_PEAK_GBS,
                     'unit': 'GB/s', 'frac': round(achieved / HBM_PEAK_GBS, 4),
                     'traffic': traffic, 'traffic_unit': 'HBM bytes per launch (rocprofv3 PMC)',
                     'traffic_source': traffic_src,
                     'algorithmic_bytes': bts[dom] * n, 'kernel': KERNEL_NAMES[dom],
                     'bytes_per_action': bts[dom],
                     # the whole step against the roofline: the VAEP path's 1,029 B/action
                     #  of every action of every rank / step time / N x 8 TB/s
                     'step_frac': round(STEP_BYTES * total_actions / (ms_per_step * 1e-3)
                                        / (world * HBM_PEAK_GBS * 1e9), 4),
                     'step_bytes_per_action': STEP_BYTES},
    }
    line['xt_cfg4'] = {'workload': 'cfg4 inside the step: xT 16x12 fit (count + all-reduce + '
                                   'value iteration to eps=1e-5) + rate of the step\'s actions',
                       # overlapped: the side stream's span from its first launch to the
                       # rate's end (it shares the GPU with the VAEP kernels meanwhile)
                       'ms' if args.serial else 'span_ms': round(kern['xt_fit_rate'], 4),
                       'iterations': _iterations(xt_last['sol']),
                       'source': {'cells': 'cell codes written by the f64 feature pass',
                                  'codes': 'coordinates (count) + rate operands',
                                  'coords': 'coordinates'}[base['xt']],
                       'stream': 'main (serial)' if args.serial else
                       (f"count, all-reduce, solve and rate on a {base['prio']}-priority side stream "
                        'forked after the last VAEP call, overlapping the next step\'s first pass'
                        if base['fork'] >= len(order) else
                        f"count pass on the main stream after {base['fork']} VAEP call(s); all-reduce, "
                        f"solve and rate on a {base['prio']}-priority side stream overlapped with the rest"
                        if base['cm'] else
                        f"{base['prio']}-priority side stream, forked after {base['fork']} VAEP "
                        'call(s), overlapped with the rest')}
    ref_cpu = reference_cpu_record()
    if ref_cpu is not None and ref_cpu.get('step_one_process_with_xt_16x12'):
        # BASELINE.md publishes no number for this metric: the ratio is against the reference's
        # own pandas path (VAEP features + labels + formula and the xT 16x12 fit + rate, one
        # process), timed in the build container -- a cross-host figure, labelled as such
        line['vs_baseline'] = round(value / ref_cpu['step_one_process_with_xt_16x12'], 1)
        line['vs_baseline_basis'] = (
            f"value / {ref_cpu['step_one_process_with_xt_16x12']:,} actions/s: the pandas reference "
            '(VAEP + xT 16x12, one process) timed in the build container, not on the GPU host '
            '(cross-host; BASELINE.md publishes no number; profiles/reference_cpu.json)')
    if rotate is not None:
        line['rotate'] = rotate
    line['vaep_order'] = order
    line['streams'] = ('one stream' if args.serial else
                       'VAEP kernels on the main stream, xT solve + rate on a side stream without a '
                       'host round trip, pipelined: step k\'s xT work may finish during step k+1 (two '
                       'cell-code buffers); the timed region ends after every stream is synchronised')
    if check:
        line['parity'] = dict(par.record(), seconds=round(check_s, 2),
                              what='the last timed step\'s buffers: every feature column, both '
                                   'labels and the f64 formula of 12 sampled games per rank; the '
                                   'xT 16x12 counts the step solved from, its surface and '
                                   'iteration count, and its rate of the sampled games')
    line.update(extra_side)
    if not args.no_cpu and world == 1:  # the CPU comparator runs on rank 0 at N = 1 only
        line['cpu_baseline'] = cpu_baseline(d, args.cpu_seconds)
        ref = reference_cpu_record()
        if ref is not None:
            line['cpu_baseline']['reference'] = ref
    print(json.dumps(line), flush=True)
    if dist:
        dist.destroy_process_group()
    if not (par.ok and side_ok):
        print('bench.py: PARITY FAILED: ' + json.dumps(
            {'step': par.failures, **{k: v['parity']['failures'] for k, v in extra_side.items()
                                      if 'parity' in v}}), file=sys.stderr)
        raise SystemExit(3)


if __name__ == '__main__':
    main()
