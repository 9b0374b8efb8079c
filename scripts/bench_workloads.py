#!/usr/bin/env python
"""Side measurements next to bench.py's headline line (BASELINE.json configs 3-5 and the
pandas boundary).  Each workload prints one JSON line; the committed copies live under
profiles/.

    python scripts/bench_workloads.py atomic [--games 10000]   # cfg3: ~4.0e7 atomic actions
    python scripts/bench_workloads.py xt105 [--games 7812]      # cfg5 per-GPU slice: ~1.25e7
    python scripts/bench_workloads.py e2e [--games 500]         # pandas in -> pandas out
    python scripts/bench_workloads.py convert [--games 10000]   # SPADL -> Atomic-SPADL
    python scripts/bench_workloads.py dribbles [--games 10000]  # spadl.base._add_dribbles
    python scripts/bench_workloads.py store [--games 1000]      # per-game Parquet stores

All device timings are HIP events on torch's current stream (the launch stream); wall
times bracket torch.cuda.synchronize().
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from socceraction_amd import batch as B  # noqa: E402
from socceraction_amd import ops, synthetic  # noqa: E402

ATOMIC_DEFAULT = ['actiontype', 'actiontype_onehot', 'bodypart', 'bodypart_onehot', 'time',
                  'team', 'time_delta', 'location', 'polar', 'movement_polar', 'direction',
                  'goalscore']
SPADL_DEFAULT = ['actiontype_onehot', 'result_onehot', 'actiontype_result_onehot',
                 'bodypart_onehot', 'time', 'startlocation', 'endlocation', 'startpolar',
                 'endpolar', 'movement', 'team', 'time_delta', 'space_delta', 'goalscore']
HBM_PEAK_GBS = 8000.0


def _timed(fn, steps: int, warmup: int) -> float:
    """Mean ms per call from HIP events over ``steps`` back-to-back calls."""
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(steps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / steps


def atomic(args) -> dict:
    """cfg3: Atomic-VAEP features (k=3, default 12 xfns = 154 columns) + labels."""
    dev = B.device()
    t = time.perf_counter()
    d = synthetic.atomic_games(args.games)
    gen_s = time.perf_counter() - t
    ab = B.ActionBatch.from_columns(d, atomic=True, dev=dev)
    n = ab.n
    out = ops.features(ab, ATOMIC_DEFAULT, 3, bool_tile=1024, num_tile=128)
    plan = out.plan
    lab = ops.labels(ab)
    ms_f = _timed(lambda: ops.features(ab, ATOMIC_DEFAULT, 3, out=out), args.steps, 2)
    ms_l = _timed(lambda: ops.labels(ab, 10, lab), args.steps, 2)
    # algorithmic bytes: 5 f64 + 3 u8 + i32 in (47 B), 110 bool + 32 f64 + 12 i64 + 2 labels out
    in_b, out_b = 47, plan.n_bool + 8 * (plan.n_f64 + plan.n_i64) + 2
    step_ms = ms_f + ms_l
    return {'workload': 'cfg3: Atomic-VAEP features (k=3, default xfns) + labels, one GPU',
            'games': args.games, 'actions': n,
            'columns': {'bool': plan.n_bool, 'f64': plan.n_f64, 'i64': plan.n_i64},
            'ms_features': round(ms_f, 4), 'ms_labels': round(ms_l, 4),
            'ms_per_step': round(step_ms, 4), 'actions_per_s': round(n / step_ms * 1e3, 1),
            'bytes_per_action': in_b + out_b,
            'achieved_GBs': round((in_b + out_b) * n / step_ms * 1e-6, 1),
            'frac_of_8TBs': round((in_b + out_b) * n / step_ms * 1e-6 / HBM_PEAK_GBS, 4),
            'note': f'8-GPU cfg3 = 5e6 per GPU; synthetic generation {gen_s:.1f} s (untimed)'}


def xt105(args) -> dict:
    """cfg5 per-GPU slice: 105x68 xT fit (count, normalise, value iteration over the dense
    7140^2 transition matrix) + rate(use_interpolation=True) over the 1050x680 surface."""
    l, w = 105, 68
    C = l * w
    dev = B.device()
    d = synthetic.spadl_games(args.games)
    ab = B.ActionBatch.from_columns(d, dev=dev)
    n = ab.n
    acc = ops.xt_zero_counts(l, w, dev)

    def count():
        for t in (acc.shot, acc.goal, acc.move, acc.trans, acc.err):
            t.zero_()
        ops.xt_count(ab, l, w, acc)
    ms_count = _timed(count, 3, 1)
    ms_norm = _timed(lambda: ops.xt_normalize(acc), 3, 1)
    torch.cuda.synchronize()
    t = time.perf_counter()
    sol = ops.xt_solve(acc)
    torch.cuda.synchronize()
    ms_solve = (time.perf_counter() - t) * 1e3
    xT = sol.mats[3].reshape(w, l)
    ms_grid = _timed(lambda: ops.xt_interp_grid(xT, l, w), 5, 1)
    grid = ops.xt_interp_grid(xT, l, w)
    ms_rate = _timed(lambda: ops.xt_rate(ab, grid, 1050, 680), 5, 1)
    it_bytes = 8 * C * C + 32 * C
    per_it = (ms_solve - ms_norm) / max(sol.n_iter, 1)
    total = ms_count + ms_solve + ms_grid + ms_rate
    return {'workload': 'cfg5 per-GPU slice: xT 105x68 fit + rate(use_interpolation=True)',
            'actions': n, 'cells': C, 'iterations': sol.n_iter,
            'ms_count': round(ms_count, 3),
            'count_GBs': round(34 * n / ms_count * 1e-6, 1),
            'ms_normalize': round(ms_norm, 3),
            'ms_solve_incl_normalize': round(ms_solve, 3),
            'ms_per_iteration': round(per_it, 4),
            'iteration_GBs': round(it_bytes / per_it * 1e-6, 1),
            'iteration_frac_of_8TBs': round(it_bytes / per_it * 1e-6 / HBM_PEAK_GBS, 4),
            'ms_interp_grid': round(ms_grid, 4), 'ms_rate': round(ms_rate, 4),
            'rate_GBs': round(42 * n / ms_rate * 1e-6, 1),
            'ms_fit_and_rate': round(total, 3),
            'actions_per_s': round(n / total * 1e3, 1),
            'note': 'single rank: the RCCL all-reduce of the 204 MB transition counts is not '
                    'exercised here (8-GPU cfg5 adds it once per fit)'}


def e2e(args) -> dict:
    """The pandas boundary: DataFrame in -> compute_features_batch / compute_labels_batch
    DataFrames out + formula on host probabilities (the reference's notebook loop shape)."""
    import socceraction_amd.vaep as vaep
    d = synthetic.spadl_games(args.games)
    actions = synthetic.to_frame(d)
    games = synthetic.games_frame(d)
    n = len(actions)
    p = synthetic.probabilities(n)
    model = vaep.VAEP()
    model.compute_features_batch(games.head(2), actions[actions.game_id.isin(games.game_id.head(2))])

    def run():
        X = model.compute_features_batch(games, actions)
        Y = model.compute_labels_batch(games, actions)
        ab = B.ActionBatch.from_frame(actions, segments='game')
        v = ops.formula(ab, torch.from_numpy(p['scores']).to(ab.device),
                        torch.from_numpy(p['concedes']).to(ab.device)).cpu().numpy()
        return X, Y, v
    run()
    t = time.perf_counter()
    X, Y, v = run()
    dt = time.perf_counter() - t
    return {'workload': 'pandas boundary: compute_features_batch + compute_labels_batch + formula '
                        '(DataFrames in and out, includes H2D, D2H and DataFrame assembly)',
            'games': args.games, 'actions': n, 'feature_columns': X.shape[1],
            'seconds': round(dt, 3), 'actions_per_s': round(n / dt, 1)}


def convert(args) -> dict:
    """SPADL -> Atomic-SPADL conversion on device (count + scan + emit), cfg2 games."""
    from socceraction_amd.atomic.spadl import base as cb
    dev = B.device()
    d = synthetic.spadl_games(args.games)
    frame = cb.SpadlFrame.from_columns(d, dev=dev)
    out = cb.convert_device(frame)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(args.steps):
        out = cb.convert_device(frame)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t) / args.steps * 1e3
    return {'workload': 'SPADL -> Atomic-SPADL conversion (device)', 'spadl_actions': frame.n,
            'atomic_actions': out.n, 'ms_per_conversion': round(ms, 4),
            'GBs': round((2 * 60 * frame.n + 59 * out.n) / ms * 1e-6, 1)}


def dribbles(args) -> dict:
    """_add_dribbles on device (count + scan + emit) over cfg2 games, plus the drop-in's
    DataFrame-in / DataFrame-out time on a 500-game slice."""
    from socceraction_amd.atomic.spadl import base as cb
    from socceraction_amd.spadl import base as sb
    dev = B.device()
    d = synthetic.spadl_games(args.games)
    df = synthetic.to_frame(d)
    df['original_event_id'] = None
    aid = np.arange(len(df), dtype=np.int64)
    df['action_id'] = aid
    frame = cb.SpadlFrame.from_frame(df, dev=dev, sort=False)
    aid = torch.from_numpy(aid).to(dev)
    out = sb.add_dribbles_device(frame, aid)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(args.steps):
        out = sb.add_dribbles_device(frame, aid)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t) / args.steps * 1e3
    small = df.iloc[:int(d['game_off'][min(500, len(d['game_off']) - 1)])].copy()
    small['action_id'] = small.groupby('game_id').cumcount().astype(np.int64)
    sb._add_dribbles(small)
    t = time.perf_counter()
    res = sb._add_dribbles(small)
    ms_df = (time.perf_counter() - t) * 1e3
    return {'workload': '_add_dribbles (device count + scan + emit)', 'spadl_actions': frame.n,
            'out_actions': out.n, 'ms_per_call': round(ms, 4),
            'GBs': round((120 * frame.n + 68 * out.n) / ms * 1e-6, 1),
            'dropin_dataframe_actions': len(small), 'dropin_out_actions': len(res),
            'dropin_ms': round(ms_df, 2),
            'dropin_actions_per_s': round(len(small) / ms_df * 1e3, 1)}


def store(args) -> dict:
    """Feature + label stores (the notebooks' per-game to_hdf, as Parquet): device features ->
    device bitmaps -> Arrow -> part files written in parallel, against the same games written
    from the DataFrame (pandas -> Arrow conversion packs the bools on the host)."""
    import shutil
    import tempfile
    import socceraction_amd.vaep as vaep
    from socceraction_amd import store as S
    d = synthetic.spadl_games(args.games)
    actions = synthetic.to_frame(d)
    games = synthetic.games_frame(d)
    model = vaep.VAEP()
    root = tempfile.mkdtemp(prefix='sa_store_', dir=os.environ.get('TMPDIR', '/tmp'))
    out = {'workload': 'feature + label stores (Parquet, lz4), cfg2-shaped games',
           'actions': len(actions), 'games': len(games)}
    try:
        with S.FeatureStore(os.path.join(root, 'warm'), mode='w') as st:
            S.store_features_batch(model, games.iloc[:2], actions[actions.game_id.isin(
                games.game_id.iloc[:2])], st)
        torch.cuda.synchronize()
        t = time.perf_counter()
        with S.FeatureStore(os.path.join(root, 'features'), mode='w') as st:
            S.store_features_batch(model, games, actions, st, parts=16)
        with S.FeatureStore(os.path.join(root, 'labels'), mode='w') as st:
            S.store_labels_batch(model, games, actions, st, parts=16)
        dt = time.perf_counter() - t
        size = sum(os.path.getsize(os.path.join(dp, f)) for dp, _, fs in os.walk(root)
                   for f in fs)
        out.update(store_s=round(dt, 3), store_actions_per_s=round(len(actions) / dt, 1),
                   bytes_on_disk=size)
        # the feature blocks -> Arrow step alone (device bitmaps + pinned D2H)
        from socceraction_amd import ops
        ab = B.ActionBatch.from_frame(actions, home_team_id=games.set_index('game_id')[
            'home_team_id'], segments='game')
        fb = ops.features(ab, model._split_xfns()[0], 3)
        torch.cuda.synchronize()
        t = time.perf_counter()
        tab = S.features_to_arrow(fb)
        out['to_arrow_ms'] = round((time.perf_counter() - t) * 1e3, 2)
        t = time.perf_counter()
        X = fb.to_frame()
        out['to_frame_ms'] = round((time.perf_counter() - t) * 1e3, 2)
        t = time.perf_counter()
        tab2 = __import__('pyarrow').Table.from_pandas(X, preserve_index=False)
        out['frame_to_arrow_host_ms'] = round((time.perf_counter() - t) * 1e3, 2)
        assert tab2.num_rows == tab.num_rows
        # per-game DataFrame writes (the notebooks' loop shape) on a 50-game slice
        sub = games.iloc[:50]
        t = time.perf_counter()
        with S.FeatureStore(os.path.join(root, 'loop'), mode='w') as st:
            for g in sub.itertuples():
                ga = actions[actions.game_id == g.game_id].reset_index(drop=True)
                st.put(f'game_{g.game_id}', model.compute_features(g, ga))
        dt = time.perf_counter() - t
        n_sub = int(actions.game_id.isin(sub.game_id).sum())
        out['per_game_loop_actions_per_s'] = round(n_sub / dt, 1)
    finally:
        shutil.rmtree(root, ignore_errors=True)
    return out


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument('workload', choices=('atomic', 'xt105', 'e2e', 'convert', 'dribbles', 'store'))
    ap.add_argument('--games', type=int, default=None)
    ap.add_argument('--steps', type=int, default=10)
    args = ap.parse_args()
    if args.games is None:
        args.games = {'atomic': 10000, 'xt105': 7812, 'e2e': 500, 'convert': 10000,
                      'dribbles': 10000, 'store': 1000}[args.workload]
    line = {'atomic': atomic, 'xt105': xt105, 'e2e': e2e, 'convert': convert,
            'dribbles': dribbles, 'store': store}[args.workload](args)
    line['device'] = torch.cuda.get_device_name(0)
    print(json.dumps(line), flush=True)


if __name__ == '__main__':
    main()
