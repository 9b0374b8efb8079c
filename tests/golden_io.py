"""Load the golden fixtures of tests/golden (written by tests/golden/make_golden.py)."""
import glob
import os

import numpy as np
import pandas as pd

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden')

SPADL_IN = ['game_id', 'period_id', 'time_seconds', 'team_id', 'start_x', 'start_y', 'end_x',
            'end_y', 'type_id', 'result_id', 'bodypart_id']
ATOMIC_IN = ['game_id', 'period_id', 'time_seconds', 'team_id', 'x', 'y', 'dx', 'dy', 'type_id',
             'bodypart_id']


def cases(prefix):
    """Names of the golden cases with a given prefix ('spadl', 'atomic', 'xt')."""
    return sorted(os.path.basename(p)[len(prefix) + 1:-4]
                  for p in glob.glob(os.path.join(GOLDEN, f'{prefix}_*.npz')))


def load(prefix, name):
    with np.load(os.path.join(GOLDEN, f'{prefix}_{name}.npz'), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def inputs(g, atomic=False):
    """Input columns of a case as a dict of numpy arrays (raw reference dtypes)."""
    return {c: g['in_' + c] for c in (ATOMIC_IN if atomic else SPADL_IN)}


def frame(g, atomic=False):
    """The case's input as a reference-shaped DataFrame."""
    cols = inputs(g, atomic)
    df = pd.DataFrame(cols)
    df.insert(1, 'original_event_id', None)
    df.insert(2, 'action_id', np.arange(len(df)))
    df.insert(6, 'player_id', 0)
    return df


def ks(g):
    return sorted(int(k[1:k.index('_')]) for k in g if k.startswith('k') and k.endswith('_names_all'))


def assert_close(a, b, name=''):
    """float parity bar: |a-b| <= 1e-6*|b| + 1e-12, NaNs in the same places."""
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    assert a.shape == b.shape, (name, a.shape, b.shape)
    na, nb = np.isnan(a), np.isnan(b)
    assert (na == nb).all(), f'{name}: NaN pattern differs'
    ok = ~nb
    err = np.abs(a[ok] - b[ok])
    tol = 1e-6 * np.abs(b[ok]) + 1e-12
    bad = err > tol
    assert not bad.any(), f'{name}: {bad.sum()} mismatches, max err {err.max()}'


CONVERT_IN = ['game_id', 'original_event_id', 'action_id', 'period_id', 'time_seconds', 'team_id',
              'player_id', 'start_x', 'start_y', 'end_x', 'end_y', 'type_id', 'result_id',
              'bodypart_id']
CONVERT_OUT = ['game_id', 'original_event_id', 'action_id', 'period_id', 'time_seconds',
               'team_id', 'player_id', 'x', 'y', 'dx', 'dy', 'type_id', 'bodypart_id']


def _convert_cols(g, prefix, names):
    out = {}
    for c in names:
        v = g[prefix + c]
        if c == 'original_event_id':
            v = np.array([None if m else s for s, m in zip(v, g[prefix + c + '_isna'])],
                         dtype=object)
        out[c] = v
    return out


def convert_input(g):
    """Input SPADL frame of a convert_* golden (tests/golden/make_golden_convert.py)."""
    return pd.DataFrame(_convert_cols(g, 'in_', CONVERT_IN))


def convert_output(g):
    """The reference's Atomic-SPADL output of a convert_* golden as columns."""
    return _convert_cols(g, 'out_', CONVERT_OUT)


def assert_convert_equal(got: dict, ref: dict, name=''):
    """Bit-exact ids / codes / counts; floats within the assert_close bar; same NaN pattern
    of original_event_id."""
    assert set(got) >= set(CONVERT_OUT), name
    n = len(ref['type_id'])
    for c in CONVERT_OUT:
        a, b = got[c], ref[c]
        assert len(a) == n, (name, c, len(a), n)
        if c == 'original_event_id':
            ma = np.array([x is None or (isinstance(x, float) and np.isnan(x)) for x in a], bool)
            mb = np.array([x is None for x in b], bool)
            np.testing.assert_array_equal(ma, mb, err_msg=f'{name} {c} missing pattern')
            np.testing.assert_array_equal(np.asarray(a, object)[~ma].astype(str),
                                          np.asarray(b, object)[~mb].astype(str), err_msg=name)
        elif np.asarray(b).dtype.kind == 'f':
            assert_close(a, b, f'{name} {c}')
        else:
            np.testing.assert_array_equal(np.asarray(a).astype(np.int64),
                                          np.asarray(b).astype(np.int64), err_msg=f'{name} {c}')


def dribbles_frame(g, prefix='in_'):
    """A dribbles_* golden's input (``in_``) or the reference's output (``out_``) as a DataFrame
    with the stored dtypes (tests/golden/make_golden_dribbles.py)."""
    cols = {}
    for c in g[prefix + '__columns']:
        c = str(c)
        dt = str(g[prefix + c + '__dtype'])
        v = g[prefix + c]
        if dt == 'object':
            v = np.array([np.nan if m else s for s, m in zip(v, g[prefix + c + '__isna'])],
                         dtype=object)
        cols[c] = pd.Series(v, dtype=dt)
    return pd.DataFrame(cols)


def assert_frame_same(got: pd.DataFrame, ref: pd.DataFrame, name=''):
    """Same columns, order and dtypes; values bit-exact (floats too; NaN where the reference
    has NaN); object columns equal as strings with the same missing pattern."""
    assert list(got.columns) == list(ref.columns), (name, list(got.columns), list(ref.columns))
    assert len(got) == len(ref), (name, len(got), len(ref))
    assert got.index.equals(pd.RangeIndex(len(ref))), name
    for c in ref.columns:
        a, b = got[c], ref[c]
        assert a.dtype == b.dtype, (name, c, a.dtype, b.dtype)
        if b.dtype == object:
            ma, mb = a.isna().to_numpy(), b.isna().to_numpy()
            np.testing.assert_array_equal(ma, mb, err_msg=f'{name} {c} missing pattern')
            np.testing.assert_array_equal(a[~ma].astype(str).to_numpy(),
                                          b[~mb].astype(str).to_numpy(), err_msg=f'{name} {c}')
        else:
            np.testing.assert_array_equal(a.to_numpy(), b.to_numpy(), err_msg=f'{name} {c}')
