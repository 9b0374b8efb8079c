"""Golden vectors for SPADL -> Atomic-SPADL conversion, produced by running the *reference*.

Build container only (the reference never travels to the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_convert.py

Imports ``/root/reference`` with the same shims as ``make_golden.py`` (pandera stand-in:
``DataFrame[Schema]`` is a no-op cast, so inputs are asserted schema-valid here) and calls
``socceraction.atomic.spadl.convert_to_atomic`` (atomic/spadl/base.py:15-35) on:

* the reference's own fixture ``tests/datasets/spadl/spadl.json`` (200 rows, one game);
* its 0-, 1-, 2- and 3-row prefixes;
* synthetic multi-game frames with forced edge cases: passes followed by interception-like
  actions, goalkicks (same and other team) and throw-ins, offside passes, shots followed by
  corners / goalkicks, goals, owngoal results on non-shot actions, yellow / red cards, and a
  pair of consecutive games whose boundary actions qualify for a cross-game dribble;
* unsorted frames (games in descending game_id order; rows swapped inside a game), where the
  first pass reads input-order neighbours before the reference's sort.

Inputs and outputs are stored as plain arrays (original_event_id as a unicode array plus a
missing-value mask: no pickles).
"""
from __future__ import annotations

import os
import sys

import numpy as np
import pandas as pd

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = '/root/reference'
sys.dont_write_bytecode = True
sys.path.insert(0, os.path.join(HERE, '_shims'))
sys.path.insert(0, REF)
sys.path.insert(0, REPO)
np.NaN = np.nan  # noqa: N816

from socceraction.atomic.spadl import convert_to_atomic  # noqa: E402

from socceraction_amd import synthetic  # noqa: E402

IN_COLS = ['game_id', 'original_event_id', 'action_id', 'period_id', 'time_seconds', 'team_id',
           'player_id', 'start_x', 'start_y', 'end_x', 'end_y', 'type_id', 'result_id',
           'bodypart_id']
OUT_COLS = ['game_id', 'original_event_id', 'action_id', 'period_id', 'time_seconds', 'team_id',
            'player_id', 'x', 'y', 'dx', 'dy', 'type_id', 'bodypart_id']


def _check(df: pd.DataFrame) -> None:
    """What SPADLSchema (strict, coerce) would enforce on the inputs."""
    for c in ('period_id', 'type_id', 'result_id', 'bodypart_id', 'action_id'):
        assert df[c].dtype == np.int64, c
    assert df.period_id.between(1, 5).all() and (df.time_seconds >= 0).all()
    for c, hi in (('start_x', 105), ('end_x', 105), ('start_y', 68), ('end_y', 68)):
        assert df[c].between(0, hi).all(), c
    assert df.type_id.between(0, 22).all() and df.result_id.between(0, 5).all()
    assert df.bodypart_id.between(0, 3).all()


def _store(out: dict, prefix: str, df: pd.DataFrame, cols) -> None:
    for c in cols:
        v = df[c]
        if c == 'original_event_id':
            out[prefix + c] = np.array(['' if pd.isna(x) else str(x) for x in v], dtype=str)
            out[prefix + c + '_isna'] = v.isna().to_numpy()
        else:
            out[prefix + c] = v.to_numpy()


def case(name: str, df: pd.DataFrame) -> None:
    df = df[IN_COLS].reset_index(drop=True)
    _check(df)
    res = convert_to_atomic(df.copy())
    assert list(res.columns) == OUT_COLS
    out = {}
    _store(out, 'in_', df, IN_COLS)
    _store(out, 'out_', res, OUT_COLS)
    np.savez_compressed(os.path.join(HERE, f'convert_{name}.npz'), **out)
    print('convert', name, len(df), '->', len(res), 'rows')


def synthetic_frame(n_games: int, seed: int, rng: np.random.Generator) -> pd.DataFrame:
    d = synthetic.spadl_games(n_games, seed=seed, mean_actions=300.0)
    df = synthetic.to_frame(d)
    n = len(df)
    df['original_event_id'] = [f'e{g}-{i}' for g, i in zip(df.game_id, range(n))]
    df['action_id'] = df.groupby('game_id').cumcount().astype(np.int64)
    # forced edge cases at random positions
    t = df['type_id'].to_numpy().copy()
    r = df['result_id'].to_numpy().copy()
    team = df['team_id'].to_numpy().copy()
    for _ in range(n // 20):
        j = int(rng.integers(0, n - 1))
        kind = int(rng.integers(0, 9))
        if kind == 0:   # pass -> interception-like
            t[j], t[j + 1] = 0, int(rng.choice([10, 9, 16, 14, 15, 17]))
        elif kind == 1:  # pass-like -> goalkick (other or same team)
            t[j], t[j + 1] = int(rng.choice([0, 1, 2, 3, 4, 5, 6, 18, 22])), 22
        elif kind == 2:  # pass -> throw-in
            t[j], t[j + 1] = 0, 2
        elif kind == 3:  # offside pass
            t[j], r[j] = 0, 2
        elif kind == 4:  # shot -> corner / goalkick
            t[j], t[j + 1] = int(rng.choice([11, 12, 13])), int(rng.choice([5, 6, 22]))
        elif kind == 5:  # goal
            t[j], r[j] = int(rng.choice([11, 12, 13])), 1
        elif kind == 6:  # owngoal result on any action
            r[j] = 3
        elif kind == 7:  # cards
            t[j], r[j] = 8, int(rng.choice([4, 5]))
        else:            # same-team pair (receival / dribble candidates)
            team[j + 1] = team[j]
    df['type_id'], df['result_id'], df['team_id'] = t, r, team
    return df


def cross_game_pair() -> pd.DataFrame:
    """Two games: the first ends and the second starts in period 2 with the same team 10 m
    apart 4 s later, so `_add_dribbles` (no same-game test, spadl/base.py:57-69) inserts a
    dribble across the game boundary."""
    rows = []
    for i in range(4):
        rows.append(dict(game_id=1, original_event_id=f'a{i}', action_id=i, period_id=2,
                         time_seconds=100.0 + i, team_id=7 if i % 2 else 8, player_id=70 + i,
                         start_x=30.0 + i, start_y=30.0, end_x=40.0 + i, end_y=32.0,
                         type_id=7, result_id=1, bodypart_id=0))
    rows[-1].update(team_id=7)
    for i in range(3):
        rows.append(dict(game_id=2, original_event_id=f'b{i}', action_id=i, period_id=2,
                         time_seconds=1.0 + i, team_id=7, player_id=90 + i,
                         start_x=48.0 + i, start_y=36.0, end_x=60.0, end_y=40.0,
                         type_id=7, result_id=1, bodypart_id=1))
    return pd.DataFrame(rows)


def main() -> None:
    rng = np.random.default_rng(2024)
    sp = pd.read_json(os.path.join(REF, 'tests/datasets/spadl/spadl.json'), orient='records')
    case('fixture', sp)
    for n in (0, 1, 2, 3):
        case(f'fixture_n{n}', sp.iloc[:n])
    case('synth3', synthetic_frame(3, 61, rng))
    case('synth8', synthetic_frame(8, 62, rng))
    case('crossgame', cross_game_pair())
    df = synthetic_frame(3, 63, rng)
    rev = pd.concat([g for _, g in df.groupby('game_id', sort=True)][::-1], ignore_index=True)
    case('unsorted_games', rev)
    sw = synthetic_frame(2, 64, rng)
    idx = np.arange(len(sw))
    for j in rng.choice(len(sw) - 1, 12, replace=False):
        idx[j], idx[j + 1] = idx[j + 1], idx[j]
    case('unsorted_rows', sw.iloc[idx])


if __name__ == '__main__':
    main()
