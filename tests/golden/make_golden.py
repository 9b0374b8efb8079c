"""Generate the golden parity fixtures by running the *reference* socceraction.

Run only in the build container (the reference never travels to the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

It imports the read-only reference at ``/root/reference`` with the local shims in
``tests/golden/_shims`` (pandera / pytest_mock stand-ins), plus two
in-process patches: ``np.NaN = np.nan`` (NumPy 2 removed it; ``xthreat.py:454``) and
``xthreat.interp2d`` -> a ``RectBivariateSpline(kx=ky=1, s=0)`` wrapper (scipy >= 1.14
removed ``interp2d``; this is scipy's documented replacement on regular grids).

Inputs are the reference's own fixtures (``tests/datasets/spadl/*.json``) plus small
synthetic games from :mod:`socceraction_amd.synthetic` (edge sizes n = 1..40, forced
goals/owngoals at the segment tail, full-size games). Every output is stored as plain
arrays in ``tests/golden/*.npz`` (no pickles): inputs, feature blocks split by dtype,
labels, formula values (f64 and f32 probabilities), and xT matrices/surfaces/rates.
"""
from __future__ import annotations

import io
import json
import os
import sys
from contextlib import redirect_stdout

import numpy as np
import pandas as pd

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = '/root/reference'
sys.dont_write_bytecode = True
sys.path.insert(0, os.path.join(HERE, '_shims'))
sys.path.insert(0, REF)
sys.path.insert(0, REPO)

np.NaN = np.nan  # noqa: N816  (reference uses the removed alias)

from scipy.interpolate import RectBivariateSpline  # noqa: E402

import socceraction.atomic.spadl as ref_aspadl  # noqa: E402
import socceraction.atomic.vaep as ref_avaep  # noqa: E402
import socceraction.atomic.vaep.features as ref_afs  # noqa: E402
import socceraction.atomic.vaep.formula as ref_aformula  # noqa: E402
import socceraction.atomic.vaep.labels as ref_alab  # noqa: E402
import socceraction.spadl as ref_spadl  # noqa: E402
import socceraction.vaep as ref_vaep  # noqa: E402
import socceraction.vaep.features as ref_fs  # noqa: E402
import socceraction.vaep.formula as ref_formula  # noqa: E402
import socceraction.vaep.labels as ref_lab  # noqa: E402
import socceraction.xthreat as ref_xt  # noqa: E402

from socceraction_amd import synthetic  # noqa: E402


def _interp2d(x, y, z, kind='linear', bounds_error=False):
    assert kind == 'linear'
    spl = RectBivariateSpline(x, y, np.asarray(z).T, kx=1, ky=1, s=0)
    return lambda xs, ys: spl(np.sort(xs), np.sort(ys)).T


ref_xt.interp2d = _interp2d

SPADL_IN = ['game_id', 'period_id', 'time_seconds', 'team_id', 'start_x', 'start_y',
            'end_x', 'end_y', 'type_id', 'result_id', 'bodypart_id']
ATOMIC_IN = ['game_id', 'period_id', 'time_seconds', 'team_id', 'x', 'y', 'dx', 'dy',
             'type_id', 'bodypart_id']


def _check_spadl(df: pd.DataFrame, atomic: bool) -> None:
    """What pandera's SPADLSchema (strict, coerce) would enforce on these inputs."""
    for c in ('period_id', 'type_id', 'bodypart_id') + (() if atomic else ('result_id',)):
        assert df[c].dtype == np.int64, c
    assert df.period_id.between(1, 5).all()
    assert (df.time_seconds >= 0).all()
    if atomic:
        assert df.x.between(0, 105).all() and df.y.between(0, 68).all()
        assert df.dx.between(-105, 105).all() and df.dy.between(-68, 68).all()
        assert df.type_id.between(0, 32).all()
    else:
        for c, hi in (('start_x', 105), ('end_x', 105), ('start_y', 68), ('end_y', 68)):
            assert df[c].between(0, hi).all(), c
        assert df.type_id.between(0, 22).all() and df.result_id.between(0, 5).all()
    assert df.bodypart_id.between(0, 3).all()


def _split_features(X: pd.DataFrame) -> dict:
    kinds = []
    for c in X.columns:
        dt = X[c].dtype
        if dt == np.bool_:
            kinds.append('b')
        elif dt == np.float64:
            kinds.append('f')
        elif dt == np.int64:
            kinds.append('i')
        else:
            raise AssertionError(f'unexpected dtype {dt} for {c}')
    kinds = np.array(kinds)
    names = np.array(list(X.columns))
    out = dict(names_all=names, kinds_all=kinds)
    for k, dt in (('b', np.uint8), ('f', np.float64), ('i', np.int64)):
        cols = names[kinds == k]
        out['names_' + k] = cols
        out['feat_' + k] = (X[list(cols)].to_numpy().astype(dt) if len(cols)
                            else np.zeros((len(X), 0), dt))
    return out


class _Game:
    def __init__(self, home):
        self.home_team_id = home


def _inputs(df: pd.DataFrame, cols) -> dict:
    return {'in_' + c: df[c].to_numpy() for c in cols}


def spadl_case(name: str, df: pd.DataFrame, home: int, ks=(3,), probs_seed: int = 1) -> None:
    """Per-game VAEP features/labels/formula of one frame (= one segment)."""
    _check_spadl(df, atomic=False)
    out = _inputs(df, SPADL_IN)
    out['home_team_id'] = np.array([home], np.int64)
    game = _Game(home)
    for k in ks:
        X = ref_vaep.VAEP(nb_prev_actions=k).compute_features(game, df)
        for key, v in _split_features(X).items():
            out[f'k{k}_{key}'] = v
    model = ref_vaep.VAEP()
    Y = model.compute_labels(game, df)
    assert list(Y.columns) == ['scores', 'concedes']
    out['scores'] = Y['scores'].to_numpy().astype(np.uint8)
    out['concedes'] = Y['concedes'].to_numpy().astype(np.uint8)
    withnames = ref_spadl.add_names(df)
    out['goal_from_shot'] = ref_lab.goal_from_shot(withnames)['goal_from_shot'].to_numpy().astype(np.uint8)
    p = synthetic.probabilities(len(df), seed=probs_seed)
    out['ps'], out['pc'] = p['scores'], p['concedes']
    for tag, dt in (('64', np.float64), ('32', np.float32)):
        ps = pd.Series(p['scores'].astype(dt))
        pc = pd.Series(p['concedes'].astype(dt))
        V = ref_formula.value(withnames, ps, pc)
        for c in ('offensive_value', 'defensive_value', 'vaep_value'):
            assert V[c].dtype == dt, (c, V[c].dtype)
            out[f'{c}_{tag}'] = V[c].to_numpy()
    np.savez_compressed(os.path.join(HERE, f'spadl_{name}.npz'), **out)
    print('spadl', name, len(df), 'rows')


def atomic_case(name: str, df: pd.DataFrame, home: int, ks=(3,), probs_seed: int = 2) -> None:
    _check_spadl(df, atomic=True)
    out = _inputs(df, ATOMIC_IN)
    out['home_team_id'] = np.array([home], np.int64)
    game = _Game(home)
    for k in ks:
        X = ref_avaep.AtomicVAEP(nb_prev_actions=k).compute_features(game, df)
        for key, v in _split_features(X).items():
            out[f'k{k}_{key}'] = v
    Y = ref_avaep.AtomicVAEP().compute_labels(game, df)
    out['scores'] = Y['scores'].to_numpy().astype(np.uint8)
    out['concedes'] = Y['concedes'].to_numpy().astype(np.uint8)
    withnames = ref_aspadl.add_names(df)
    g = ref_alab.goal_from_shot(withnames)['goal']
    out['goal_from_shot'] = g.to_numpy().astype(np.uint8)
    p = synthetic.probabilities(len(df), seed=probs_seed)
    out['ps'], out['pc'] = p['scores'], p['concedes']
    for tag, dt in (('64', np.float64), ('32', np.float32)):
        V = ref_aformula.value(withnames, pd.Series(p['scores'].astype(dt)),
                               pd.Series(p['concedes'].astype(dt)))
        for c in ('offensive_value', 'defensive_value', 'vaep_value'):
            assert V[c].dtype == dt
            out[f'{c}_{tag}'] = V[c].to_numpy()
    np.savez_compressed(os.path.join(HERE, f'atomic_{name}.npz'), **out)
    print('atomic', name, len(df), 'rows')


def xt_case(name: str, df: pd.DataFrame, grids, interp_grids=()) -> None:
    out = _inputs(df, SPADL_IN)
    for (l, w) in grids:
        m = ref_xt.ExpectedThreat(l=l, w=w)
        buf = io.StringIO()
        with redirect_stdout(buf):
            m.fit(df)
        tag = f'{l}x{w}'
        out[f'{tag}_scoring_prob'] = m.scoring_prob_matrix
        out[f'{tag}_shot_prob'] = m.shot_prob_matrix
        out[f'{tag}_move_prob'] = m.move_prob_matrix
        out[f'{tag}_transition'] = m.transition_matrix
        out[f'{tag}_xT'] = m.xT
        out[f'{tag}_heatmaps'] = np.stack(m.heatmaps)
        out[f'{tag}_rate'] = m.rate(df)
        if (l, w) in interp_grids:
            out[f'{tag}_rate_interp'] = m.rate(df, use_interpolation=True)
        print('xt', name, tag, 'iterations', len(m.heatmaps) - 1)
    np.savez_compressed(os.path.join(HERE, f'xt_{name}.npz'), **out)


def _force_tail_goals(d: dict, rng: np.random.Generator) -> None:
    """Put goals / owngoals near the end of each game (label tail clamping)."""
    off = d['game_off']
    for g in range(len(off) - 1):
        a, b = off[g], off[g + 1]
        n = b - a
        if n >= 1:
            j = b - 1 - int(rng.integers(0, min(n, 4)))
            d['type_id'][j] = 11
            d['result_id'][j] = int(rng.choice([1, 3]))
        if n >= 3:
            j = a + int(rng.integers(0, n))
            d['type_id'][j] = 12
            d['result_id'][j] = 1


def main() -> None:
    rng = np.random.default_rng(12345)
    # --- reference fixtures (tests/conftest.py:18-27) ---
    sp = pd.read_json(os.path.join(REF, 'tests/datasets/spadl/spadl.json'), orient='records')
    asp = pd.read_json(os.path.join(REF, 'tests/datasets/spadl/atomic_spadl.json'), orient='records')
    spadl_case('fixture', sp, 782, ks=(1, 2, 3, 5))
    atomic_case('fixture', asp, 782, ks=(1, 3))

    # --- synthetic edge games: tiny segments, forced tail goals ---
    for n in (1, 2, 3, 5, 9, 10, 11, 40, 300):
        d = synthetic.spadl_games(1, seed=100 + n, mean_actions=float(max(2 * n, 100)))
        keep = n
        for key in ('game_id', 'team_id', 'period_id', 'time_seconds', 'type_id', 'result_id',
                    'bodypart_id', 'start_x', 'start_y', 'end_x', 'end_y', 'pos', 'seg'):
            d[key] = d[key][:keep]
        d['game_off'] = np.array([0, min(keep, len(d['type_id']))], np.int64)
        _force_tail_goals(d, rng)
        df = synthetic.to_frame(d)
        home = int(d['home_team_id'][0]) if n != 9 else int(d['home_team_id'][0]) + 1
        spadl_case(f'n{n}', df, home, ks=(3,) if n not in (2, 40) else (1, 3, 4))

        da = synthetic.atomic_games(1, seed=200 + n, mean_actions=float(max(2 * n, 100)))
        for key in ('game_id', 'team_id', 'period_id', 'time_seconds', 'type_id',
                    'bodypart_id', 'x', 'y', 'dx', 'dy', 'pos', 'seg'):
            da[key] = da[key][:keep]
        if len(da['type_id']) >= 2:
            da['type_id'][-2] = 11
            da['type_id'][-1] = 27
        dfa = synthetic.to_frame(da, atomic=True)
        atomic_case(f'n{n}', dfa, int(da['home_team_id'][0]), ks=(3,) if n != 40 else (1, 3))

    # --- full-size synthetic games ---
    d = synthetic.spadl_games(2, seed=31)
    _force_tail_goals(d, rng)
    off = d['game_off']
    full = synthetic.to_frame(d)
    for g in range(2):
        sub = full.iloc[off[g]:off[g + 1]].reset_index(drop=True)
        spadl_case(f'full{g}', sub, int(d['home_team_id'][g]))
    # module-level semantics: a 2-game frame is ONE segment (no game_id split)
    spadl_case('concat2', full, int(d['home_team_id'][1]))

    da = synthetic.atomic_games(1, seed=41)
    atomic_case('full0', synthetic.to_frame(da, atomic=True), int(da['home_team_id'][0]))

    # --- xT ---
    xt_case('fixture', sp, grids=[(16, 12), (8, 6), (1, 1), (2, 2)], interp_grids=[(16, 12)])
    d = synthetic.spadl_games(8, seed=51)
    xt_case('synth8', synthetic.to_frame(d), grids=[(16, 12), (8, 6), (30, 20)],
            interp_grids=[(16, 12), (8, 6)])

    meta = dict(generator='tests/golden/make_golden.py', reference='/root/reference',
                pandas=pd.__version__, numpy=np.__version__)
    with open(os.path.join(HERE, 'META.json'), 'w') as f:
        json.dump(meta, f, indent=1)


if __name__ == '__main__':
    main()
