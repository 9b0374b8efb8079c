"""Golden vectors for ``_add_dribbles`` (spadl/base.py:54-93), produced by running the *reference*.

Build container only (the reference never travels to the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_dribbles.py

Imports ``/root/reference`` with the shims of ``make_golden.py`` and calls
``socceraction.spadl.base._add_dribbles`` on:

* the reference's fixture ``tests/datasets/spadl/spadl.json`` (already holds its dribbles: no
  insertion) and the same game with every third row removed (gaps that qualify);
* its 0-, 1- and 2-row prefixes;
* synthetic multi-game frames (per-game action ids restarting at 0, so a dribble across a game
  boundary sorts into the next game) with extra columns: ``timestamp`` (strings, copied from
  the successor), an int64 and a bool column (missing on dribble rows);
* the two-game cross-boundary pair of ``make_golden_convert.py``;
* unsorted frames (games in descending game_id order; swapped rows inside a game).

Inputs and outputs are stored as plain arrays (object columns as unicode + missing mask).
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
sys.path.insert(0, HERE)
np.NaN = np.nan  # noqa: N816

from socceraction.spadl.base import _add_dribbles  # noqa: E402

from make_golden_convert import IN_COLS, _check, cross_game_pair, synthetic_frame  # noqa: E402


def _store(out: dict, prefix: str, df: pd.DataFrame) -> None:
    out[prefix + '__columns'] = np.array(list(df.columns), dtype=str)
    for c in df.columns:
        v = df[c]
        out[prefix + c + '__dtype'] = np.array(str(v.dtype))
        if v.dtype == object:
            out[prefix + c] = np.array(['' if pd.isna(x) else str(x) for x in v], dtype=str)
            out[prefix + c + '__isna'] = v.isna().to_numpy()
        elif v.dtype.kind == 'M':
            out[prefix + c] = v.to_numpy().astype('datetime64[ns]').astype(np.int64)
            out[prefix + c + '__isna'] = v.isna().to_numpy()
        else:
            out[prefix + c] = v.to_numpy()


def case(name: str, df: pd.DataFrame, extra=()) -> None:
    df = df[IN_COLS + list(extra)].reset_index(drop=True)
    _check(df)
    res = _add_dribbles(df.copy())
    out = {}
    _store(out, 'in_', df)
    _store(out, 'out_', res)
    np.savez_compressed(os.path.join(HERE, f'dribbles_{name}.npz'), **out)
    print('dribbles', name, len(df), '->', len(res), 'rows')


def with_extras(df: pd.DataFrame, rng: np.random.Generator) -> pd.DataFrame:
    df = df.copy()
    # a string column: under pandas 2 a datetime64 column makes the reference's
    # shift(-1, fill_value=0) raise TypeError
    df['timestamp'] = [f'00:{t:09.3f}' for t in df['time_seconds'].to_numpy()]
    df['xtra_int'] = rng.integers(0, 1000, len(df)).astype(np.int64)
    df['xtra_bool'] = rng.random(len(df)) < 0.5
    return df


def main() -> None:
    rng = np.random.default_rng(2025)
    sp = pd.read_json(os.path.join(REF, 'tests/datasets/spadl/spadl.json'), orient='records')
    case('fixture', sp)
    gaps = sp[np.arange(len(sp)) % 3 != 2].copy()
    case('fixture_gaps', gaps)
    for n in (0, 1, 2):
        case(f'fixture_gaps_n{n}', gaps.iloc[:n])
    extra = ['timestamp', 'xtra_int', 'xtra_bool']
    case('synth3', with_extras(synthetic_frame(3, 71, rng), rng), extra)
    case('synth8', synthetic_frame(8, 72, rng))
    case('crossgame', cross_game_pair())
    df = synthetic_frame(3, 73, rng)
    rev = pd.concat([g for _, g in df.groupby('game_id', sort=True)][::-1], ignore_index=True)
    case('unsorted_games', rev)
    sw = synthetic_frame(2, 74, rng)
    idx = np.arange(len(sw))
    for j in rng.choice(len(sw) - 1, 12, replace=False):
        idx[j], idx[j + 1] = idx[j + 1], idx[j]
    case('unsorted_rows', with_extras(sw.iloc[idx], rng), extra)


if __name__ == '__main__':
    main()
