"""GPU parity of SPADL -> Atomic-SPADL conversion (reference atomic/spadl/base.py:15-235).

Against the reference's own outputs (tests/golden/convert_*.npz, tests/golden/
make_golden_convert.py) and, at larger sizes, against the numpy restatement of the four
passes (oracle/atomic_convert_oracle.py). Bar: ids, codes, types, periods, bodyparts,
action ids and row counts bit-exact; floats bit-exact too (the kernel performs the
reference's own f64 operations), checked with the shared float bar as well.
"""
import numpy as np
import pandas as pd
import pytest

from golden_io import assert_convert_equal, cases, convert_input, convert_output, load

pytestmark = pytest.mark.gpu

torch = pytest.importorskip('torch')


@pytest.fixture(scope='module')
def conv():
    from socceraction_amd import _native
    from socceraction_amd.atomic import spadl as aspadl
    _native.load_library()
    return aspadl


def _cols(df):
    return {c: df[c].to_numpy() for c in df.columns}


@pytest.mark.parametrize('name', cases('convert'))
def test_convert_goldens(conv, name):
    g = load('convert', name)
    df = convert_input(g)
    out = conv.convert_to_atomic(df)
    ref = convert_output(g)
    assert list(out.columns) == ['game_id', 'original_event_id', 'action_id', 'period_id',
                                 'time_seconds', 'team_id', 'player_id', 'x', 'y', 'dx', 'dy',
                                 'type_id', 'bodypart_id']
    got = _cols(out)
    assert_convert_equal(got, ref, name)
    for c in ('time_seconds', 'x', 'y', 'dx', 'dy'):
        np.testing.assert_array_equal(got[c], ref[c], err_msg=f'{name} {c}')
    for c in ('action_id', 'period_id', 'type_id', 'bodypart_id'):
        assert out[c].dtype == np.int64, c
    assert out.index.equals(pd.RangeIndex(len(out)))


def _synthetic_frame(n_games, seed):
    from socceraction_amd import synthetic
    d = synthetic.spadl_games(n_games, seed=seed)
    df = synthetic.to_frame(d)
    df['original_event_id'] = [f'ev{i}' for i in range(len(df))]
    df['action_id'] = df.groupby('game_id').cumcount().astype(np.int64)
    return df


def test_convert_vs_oracle_300_games(conv):
    """~480k SPADL actions: the device expansion == the four-pass numpy restatement."""
    from oracle import atomic_convert_oracle as co
    df = _synthetic_frame(300, 91)
    out = conv.convert_to_atomic(df)
    ref = co.convert_to_atomic(_cols(df))
    assert_convert_equal(_cols(out), ref, 'synthetic-300')
    assert len(out) > 2 * len(df)


def test_convert_unsorted_and_errors(conv):
    from oracle import atomic_convert_oracle as co
    df = _synthetic_frame(4, 92)
    rng = np.random.default_rng(0)
    shuffled = df.iloc[rng.permutation(len(df))].reset_index(drop=True)
    out = conv.convert_to_atomic(shuffled)
    assert_convert_equal(_cols(out), co.convert_to_atomic(_cols(shuffled)), 'shuffled')
    with pytest.raises(AttributeError):
        conv.convert_to_atomic(df.drop(columns=['player_id']))
    # a repeated key takes the general path (first pass placed by the stable lexsort)
    dup = df.copy()
    dup.loc[5, 'action_id'] = dup.loc[4, 'action_id']
    assert_convert_equal(_cols(conv.convert_to_atomic(dup)), co.convert_to_atomic(_cols(dup)), 'dup')
    bad = df.copy()
    bad.loc[3, 'type_id'] = 23
    with pytest.raises(ValueError):
        conv.convert_to_atomic(bad)


def test_convert_duplicate_keys_vs_oracle(conv):
    """Repeated (game_id, period_id, action_id) keys at scale (general path: the first pass
    on its own, then the single expansion without it) == the four-pass restatement, sorted
    and shuffled; the reference-generated dupkeys goldens pin the small cases."""
    from oracle import atomic_convert_oracle as co
    from socceraction_amd.atomic.spadl import base as cb
    df = _synthetic_frame(200, 93)
    df['action_id'] = (df.groupby('game_id').cumcount() // 3).astype(np.int64)
    frame = cb.SpadlFrame.from_frame(df)
    assert frame.keys is not None  # the general path
    out = conv.convert_to_atomic(df)
    assert_convert_equal(_cols(out), co.convert_to_atomic(_cols(df)), 'dup-200')
    rng = np.random.default_rng(5)
    sh = df.iloc[rng.permutation(len(df))].reset_index(drop=True)
    assert_convert_equal(_cols(conv.convert_to_atomic(sh)), co.convert_to_atomic(_cols(sh)),
                         'dup-200-shuffled')


def test_convert_then_atomic_vaep(conv):
    """Chained drop-ins: convert_to_atomic on the GPU, then AtomicVAEP features / labels, vs
    the oracle chain (convert restatement -> atomic VAEP restatement)."""
    from golden_io import assert_close
    from oracle import atomic_convert_oracle as co
    from oracle import vaep_oracle as vo
    from socceraction_amd.atomic import vaep as avaep
    df = _synthetic_frame(1, 93)
    home = int(df.team_id.iloc[0])
    atomic = conv.convert_to_atomic(df)
    X = avaep.AtomicVAEP().compute_features(pd.Series({'home_team_id': home}), atomic)
    ref_atomic = co.convert_to_atomic(_cols(df))
    cols = {c: ref_atomic[c] for c in ('period_id', 'time_seconds', 'team_id', 'x', 'y', 'dx',
                                       'dy', 'type_id', 'bodypart_id')}
    ref = vo.features(cols, 3, vo.ATOMIC_DEFAULT, atomic=True, home=[home])
    assert list(X.columns) == [c[0] for c in ref]
    for name, kind, v in ref:
        if kind == 'f':
            assert_close(X[name].to_numpy(), v, name)
        else:
            np.testing.assert_array_equal(X[name].to_numpy().astype(np.int64),
                                          np.asarray(v).astype(np.int64), err_msg=name)
    Y = avaep.AtomicVAEP().compute_labels(pd.Series({'home_team_id': home}), atomic)
    lab = vo.labels(cols, atomic=True)
    np.testing.assert_array_equal(Y['scores'].to_numpy(), lab['scores'])
    np.testing.assert_array_equal(Y['concedes'].to_numpy(), lab['concedes'])


def test_convert_device_full_size(conv):
    """cfg3 producer at full size: 10k games (~16M SPADL actions) converted on device; the
    per-game output row counts equal the oracle's on sampled games (the expansion is local,
    so each game converts independently), and the output stays grouped by game."""
    from oracle import atomic_convert_oracle as co
    from socceraction_amd import synthetic
    from socceraction_amd.atomic.spadl import base as cb
    d = synthetic.spadl_games(10000)
    df = synthetic.to_frame(d)
    df['original_event_id'] = None
    frame = cb.SpadlFrame.from_frame(df)
    out = cb.convert_device(frame)
    torch.cuda.synchronize()
    games = out.cols['game'][:out.n].cpu().numpy()
    assert (np.diff(games) >= 0).all()
    counts = np.bincount(games, minlength=len(d['game_off']) - 1)
    off = d['game_off']
    rng = np.random.default_rng(1)
    for g in rng.choice(len(off) - 1, 5, replace=False):
        sub = df.iloc[off[g]:off[g + 1]]
        ref = co.convert_to_atomic(_cols(sub))
        # a dribble across the boundary into game g belongs to game g's rows
        assert abs(int(counts[g]) - len(ref['type_id'])) <= 1, g


def test_device_pipeline_convert_to_atomic_features(conv):
    """SPADL columns -> device conversion -> atomic ActionBatch (no host round trip) ->
    Atomic-VAEP features + labels for 20 games, vs the oracle chain with per-game segments."""
    from golden_io import assert_close
    from oracle import atomic_convert_oracle as co
    from oracle import vaep_oracle as vo
    from socceraction_amd import ops, synthetic
    from socceraction_amd.atomic.spadl import base as cb
    from socceraction_amd.batch import segment_offsets
    d = synthetic.spadl_games(20, seed=94)
    frame = cb.SpadlFrame.from_columns(d)
    out = cb.convert_device(frame)
    ab = out.to_batch(frame, d['home_team_id'])
    fb = ops.features(ab, vo.ATOMIC_DEFAULT, 3)
    lb = ops.labels(ab)
    df = synthetic.to_frame(d)
    df['original_event_id'] = None
    ref = co.convert_to_atomic(_cols(df))
    assert ab.n == len(ref['type_id'])
    so = segment_offsets(ref['game_id'])
    np.testing.assert_array_equal(ab.cols['seg_off'].cpu().numpy(), so)
    cols = {c: ref[c] for c in ('period_id', 'time_seconds', 'team_id', 'x', 'y', 'dx', 'dy',
                                'type_id', 'bodypart_id')}
    rf = vo.features(cols, 3, vo.ATOMIC_DEFAULT, atomic=True, seg_off=so,
                     home=list(d['home_team_id']))
    blocks = dict(zip('bfi', fb.to_numpy()))
    assert fb.plan.names == [c[0] for c in rf]
    for (name, kind, col), (_, _, rv) in zip(fb.plan.order, rf):
        got = blocks[kind][col, :ab.n]
        if kind == 'f':
            assert_close(got, rv, name)
        else:
            np.testing.assert_array_equal(got.astype(np.int64), np.asarray(rv).astype(np.int64),
                                          err_msg=name)
    lab = vo.labels(cols, atomic=True, seg_off=so)
    np.testing.assert_array_equal(lb.scores[:ab.n].cpu().numpy().astype(bool), lab['scores'])
    np.testing.assert_array_equal(lb.concedes[:ab.n].cpu().numpy().astype(bool), lab['concedes'])
