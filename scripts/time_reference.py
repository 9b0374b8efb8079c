"""Time the reference's own CPU path (rtelmore/socceraction, pandas) in the BUILD container.

    PYTHONDONTWRITEBYTECODE=1 python scripts/time_reference.py [--games 64] [--procs 0]

The reference never travels to the GPU box, so this runs here only; bench.py copies the record
it writes (profiles/reference_cpu.json) into its ``cpu_baseline.reference`` entry, labelled as
measured in the build container.  It imports /root/reference with the golden generator's shims
(tests/golden/make_golden.py: pandera stand-in, ``np.NaN`` alias, ``interp2d`` replacement) and
times the notebooks' per-game loop (public-notebooks/2-compute-features-and-labels.ipynb:142-184,
4-compute-vaep-values-and-top-players.ipynb:144-155): ``VAEP.compute_features`` +
``compute_labels`` (vaep/base.py:97-137) + ``formula.value`` (vaep/formula.py:116-151) with
seeded probabilities (xgboost is not installed), over BASELINE cfg1's 64 synthetic games, in one
process and in an ``os.cpu_count()``-process pool over games; then cfg4's xT 16 x 12 fit + rate
of the same actions (xthreat.py:322-345, 408-465) in one process.
"""
from __future__ import annotations

import argparse
import io
import json
import multiprocessing as mp
import os
import platform
import sys
import time
from contextlib import redirect_stdout

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'tests', 'golden'))
sys.path.insert(0, ROOT)

_G = {}


def _setup():
    import make_golden as mg  # noqa: F401  (imports the reference with the shims)
    from socceraction_amd import synthetic
    _G['mg'] = mg
    _G['syn'] = synthetic


def _games(n_games: int):
    syn = _G['syn']
    d = syn.spadl_games(n_games, seed=20250223)
    df = syn.to_frame(d)
    off = d['game_off']
    games = [(int(d['home_team_id'][g]), df.iloc[off[g]:off[g + 1]].reset_index(drop=True))
             for g in range(n_games)]
    return d, df, games


class _Game:
    def __init__(self, home):
        self.home_team_id = home


def _value_games(chunk):
    """The notebook loop over some games: features + labels + formula.value per game."""
    if 'mg' not in _G:
        _setup()
    mg = _G['mg']
    model = mg.ref_vaep.VAEP()
    n = 0
    for home, actions in chunk:
        game = _Game(home)
        model.compute_features(game, actions)
        model.compute_labels(game, actions)
        p = _G['syn'].probabilities(len(actions))
        import pandas as pd
        mg.ref_formula.value(mg.ref_spadl.add_names(actions), pd.Series(p['scores']),
                             pd.Series(p['concedes']))
        n += len(actions)
    return n


def cpu_model() -> str:
    try:
        with open('/proc/cpuinfo') as f:
            for line in f:
                if line.startswith('model name'):
                    return line.split(':', 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or 'unknown'


def _load() -> dict:
    """Host load (1 / 5 / 15-minute averages and runnable processes) at a point in time."""
    try:
        l1, l5, l15 = os.getloadavg()
        return {'loadavg_1_5_15': [round(l1, 2), round(l5, 2), round(l15, 2)]}
    except OSError:
        return {}


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument('--games', type=int, default=64)
    ap.add_argument('--procs', type=int, default=0, help='pool size (0 = os.cpu_count())')
    ap.add_argument('--repeats', type=int, default=3, help='timed runs per measurement (median kept)')
    ap.add_argument('--out', default=os.path.join(ROOT, 'profiles', 'reference_cpu.json'))
    args = ap.parse_args()
    _setup()
    d, df, games = _games(args.games)
    n = len(df)
    load_before = _load()
    _value_games(games[:1])  # warm-up (imports, first merges)

    t1s = []
    for _ in range(args.repeats):
        t = time.perf_counter()
        done = _value_games(games)
        t1s.append(time.perf_counter() - t)
        assert done == n
    procs = args.procs or os.cpu_count() or 1
    chunks = [games[i::procs] for i in range(procs)]
    tps = []
    with mp.get_context('fork').Pool(procs) as pool:
        pool.map(_value_games, [games[:1]] * procs)  # warm the workers
        for _ in range(args.repeats):
            t = time.perf_counter()
            done_p = sum(pool.map(_value_games, chunks))
            tps.append(time.perf_counter() - t)
            assert done_p == n

    mg = _G['mg']
    txts = []
    for _ in range(args.repeats):
        t = time.perf_counter()
        m = mg.ref_xt.ExpectedThreat(l=16, w=12)
        with redirect_stdout(io.StringIO()):
            m.fit(df)
        m.rate(df)
        txts.append(time.perf_counter() - t)
    load_after = _load()
    t1, tp, txt = (float(np.median(v)) for v in (t1s, tps, txts))
    rec = {
        'what': 'reference CPU path (rtelmore/socceraction, pandas), timed in the build container '
                '(the reference never travels to the GPU host)',
        'workload': f'cfg1: {args.games} synthetic games ({n} actions), notebook per-game loop '
                    'VAEP.compute_features (k=3, default xfns, 568 cols) + compute_labels + '
                    'formula.value (seeded probabilities)',
        'actions': n,
        'statistic': f'median of {args.repeats} timed runs (every run listed in "runs_s")',
        'one_process': {'seconds': round(t1, 3), 'actions_per_s': round(n / t1, 1), 'cores': 1,
                        'runs_s': [round(x, 3) for x in t1s]},
        'pool': {'seconds': round(tp, 3), 'actions_per_s': round(n / tp, 1), 'processes': procs,
                 'runs_s': [round(x, 3) for x in tps]},
        'xt_16x12_fit_rate_one_process': {'seconds': round(txt, 3),
                                          'actions_per_s': round(n / txt, 1),
                                          'iterations': len(m.heatmaps) - 1,
                                          'runs_s': [round(x, 3) for x in txts]},
        'step_one_process_actions_per_s': round(n / (t1 + txt), 1),
        'host': {'cpu': cpu_model(), 'os_cpu_count': os.cpu_count(),
                 'python': platform.python_version(), 'load_before': load_before,
                 'load_after': load_after},
        'script': 'scripts/time_reference.py',
    }
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    with open(args.out, 'w') as f:
        json.dump(rec, f, indent=1)
    print(json.dumps(rec))


if __name__ == '__main__':
    main()
