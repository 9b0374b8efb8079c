"""GPU parity of ``_add_dribbles`` (reference spadl/base.py:54-93).

Against the reference's own outputs (tests/golden/dribbles_*.npz, made by
tests/golden/make_golden_dribbles.py: whole DataFrames, dtypes included) and, at larger sizes,
against the numpy restatement (oracle/atomic_convert_oracle.py ``add_dribbles``). Bar: every
column bit-exact (the kernel performs the reference's own f64 midpoint), same dtypes.
"""
import numpy as np
import pandas as pd
import pytest

from golden_io import assert_frame_same, cases, dribbles_frame, load

pytestmark = pytest.mark.gpu

torch = pytest.importorskip('torch')


@pytest.fixture(scope='module')
def sb():
    from socceraction_amd import _native
    from socceraction_amd.spadl import base
    _native.load_library()
    return base


@pytest.mark.parametrize('name', cases('dribbles'))
def test_add_dribbles_goldens(sb, name):
    g = load('dribbles', name)
    df = dribbles_frame(g, 'in_')
    ref = dribbles_frame(g, 'out_')
    assert_frame_same(sb._add_dribbles(df.copy()), ref, name)


def _synthetic(n_games, seed):
    from socceraction_amd import synthetic
    d = synthetic.spadl_games(n_games, seed=seed)
    df = synthetic.to_frame(d)
    df['original_event_id'] = [f'ev{i}' for i in range(len(df))]
    df['action_id'] = df.groupby('game_id').cumcount().astype(np.int64)
    return df


def _vs_oracle(got: pd.DataFrame, df: pd.DataFrame, name: str):
    from oracle import atomic_convert_oracle as co
    ref = co.add_dribbles({c: df[c].to_numpy() for c in co.COLS})
    assert len(got) == len(ref['type_id']), name
    for c in co.COLS:
        if c == 'original_event_id':
            np.testing.assert_array_equal(got[c].isna().to_numpy(), pd.isna(ref[c]), err_msg=name)
            continue
        np.testing.assert_array_equal(got[c].to_numpy(), np.asarray(ref[c]), err_msg=f'{name} {c}')


def test_add_dribbles_vs_oracle_300_games(sb):
    """~480k actions (per-game action ids: the game boundaries are checked for cross-game
    dribbles, which would take the general placement path)."""
    df = _synthetic(300, 95)
    got = sb._add_dribbles(df)
    _vs_oracle(got, df, 'synthetic-300')
    assert len(got) > len(df)


def test_add_dribbles_general_placement(sb):
    """Shuffled rows (stable lexsort placement) and global action ids (fast layout) agree
    with the oracle."""
    df = _synthetic(4, 96)
    rng = np.random.default_rng(0)
    shuffled = df.iloc[rng.permutation(len(df))].reset_index(drop=True)
    _vs_oracle(sb._add_dribbles(shuffled), shuffled, 'shuffled')
    glob = df.copy()
    glob['action_id'] = np.arange(len(glob), dtype=np.int64)
    _vs_oracle(sb._add_dribbles(glob), glob, 'global-ids')


def test_add_dribbles_thresholds_are_module_globals(sb):
    """The reference reads min/max_dribble_length and max_dribble_duration at call time."""
    from oracle import atomic_convert_oracle as co
    df = _synthetic(2, 97)
    base_n = len(sb._add_dribbles(df))
    old = sb.min_dribble_length, sb.max_dribble_length, sb.max_dribble_duration
    try:
        sb.min_dribble_length, sb.max_dribble_length, sb.max_dribble_duration = 1.0, 200.0, 100.0
        wide = sb._add_dribbles(df)
    finally:
        sb.min_dribble_length, sb.max_dribble_length, sb.max_dribble_duration = old
    assert len(wide) > base_n
    f = {c: df[c].to_numpy() for c in co.COLS}
    nx_team = np.r_[f['team_id'][1:], 0]
    dx = f['end_x'] - np.r_[f['start_x'][1:], 0.0]
    dy = f['end_y'] - np.r_[f['start_y'][1:], 0.0]
    dt = np.r_[f['time_seconds'][1:], 0.0] - f['time_seconds']
    d2 = dx ** 2 + dy ** 2
    same = (f['team_id'] == nx_team) & (f['period_id'] == np.r_[f['period_id'][1:], 0])
    expect = int((same & (d2 >= 1.0) & (d2 <= 40000.0) & (dt < 100.0)).sum())
    assert len(wide) - len(df) == expect


def test_add_dribbles_full_size(sb):
    """cfg2 size (10k games, ~16M actions) on device: n_out = n + dribbles; inputs keep their
    order; each dribble sits between its parent and successor with the reference's values."""
    from socceraction_amd import synthetic
    from socceraction_amd.atomic.spadl import base as cb
    d = synthetic.spadl_games(10000)
    df = synthetic.to_frame(d)
    df['original_event_id'] = None
    df['action_id'] = np.arange(len(df), dtype=np.int64)
    frame = cb.SpadlFrame.from_frame(df, sort=False)
    out = sb.add_dribbles_device(frame, df['action_id'].to_numpy())
    torch.cuda.synchronize()
    src = out.cols['src'][:out.n].cpu().numpy()
    orig = src >= 0
    np.testing.assert_array_equal(src[orig], np.arange(len(df)))
    pos = np.flatnonzero(~orig)
    assert len(pos) == out.n_dribbles > 0
    np.testing.assert_array_equal(src[pos - 1], ~src[pos] - 1)   # parent right before
    t = out.cols['time_seconds'][:out.n].cpu().numpy()
    ts = df['time_seconds'].to_numpy()
    q = ~src[pos]
    np.testing.assert_array_equal(t[pos], (ts[q - 1] + ts[q]) / 2)
    ty = out.cols['type_id'][:out.n].cpu().numpy()
    assert (ty[pos] == 21).all()
