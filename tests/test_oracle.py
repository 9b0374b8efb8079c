"""The CPU oracle reproduces the reference's goldens (CPU only, no GPU)."""
import os

import numpy as np
import pandas as pd
import pytest

from golden_io import GOLDEN, assert_close, cases, inputs, ks, load
from oracle import vaep_oracle as vo
from oracle import xt_oracle as xo


def _check_features(got, g, k):
    names = list(g[f'k{k}_names_all'])
    assert [c[0] for c in got] == names
    kinds = list(g[f'k{k}_kinds_all'])
    assert [c[1] for c in got] == kinds
    for kind in 'bfi':
        ref = g[f'k{k}_feat_{kind}']
        mine = [c[2] for c in got if c[1] == kind]
        if not mine:
            assert ref.shape[1] == 0
            continue
        M = np.stack(mine, axis=1)
        if kind == 'f':
            assert_close(M, ref, f'k{k} float features')
        else:
            np.testing.assert_array_equal(M.astype(ref.dtype), ref)


@pytest.mark.parametrize('name', cases('spadl'))
def test_spadl_oracle(name):
    g = load('spadl', name)
    cols = inputs(g)
    home = [g['home_team_id'][0]]
    for k in ks(g):
        _check_features(vo.features(cols, k, vo.SPADL_DEFAULT, home=home), g, k)
    lab = vo.labels(cols)
    np.testing.assert_array_equal(lab['scores'], g['scores'].astype(bool))
    np.testing.assert_array_equal(lab['concedes'], g['concedes'].astype(bool))
    np.testing.assert_array_equal(lab['goal_from_shot'], g['goal_from_shot'].astype(bool))
    for tag, dt in (('64', np.float64), ('32', np.float32)):
        v = vo.formula(cols, g['ps'].astype(dt), g['pc'].astype(dt))
        for c in ('offensive_value', 'defensive_value', 'vaep_value'):
            assert v[c].dtype == dt
            if dt == np.float64:
                assert_close(v[c], g[f'{c}_{tag}'], c)
            else:
                np.testing.assert_array_equal(v[c], g[f'{c}_{tag}'])


@pytest.mark.parametrize('name', cases('atomic'))
def test_atomic_oracle(name):
    g = load('atomic', name)
    cols = inputs(g, atomic=True)
    home = [g['home_team_id'][0]]
    for k in ks(g):
        _check_features(vo.features(cols, k, vo.ATOMIC_DEFAULT, atomic=True, home=home), g, k)
    lab = vo.labels(cols, atomic=True)
    np.testing.assert_array_equal(lab['scores'], g['scores'].astype(bool))
    np.testing.assert_array_equal(lab['concedes'], g['concedes'].astype(bool))
    np.testing.assert_array_equal(lab['goal_from_shot'], g['goal_from_shot'].astype(bool))
    for tag, dt in (('64', np.float64), ('32', np.float32)):
        v = vo.formula(cols, g['ps'].astype(dt), g['pc'].astype(dt), atomic=True)
        for c in ('offensive_value', 'defensive_value', 'vaep_value'):
            np.testing.assert_allclose(v[c], g[f'{c}_{tag}'], rtol=1e-6, atol=1e-12)


@pytest.mark.parametrize('name', cases('xt'))
def test_xt_oracle(name):
    g = load('xt', name)
    cols = inputs(g)
    grids = sorted({k.split('_')[0] for k in g if k[0].isdigit()})
    for tag in grids:
        l, w = map(int, tag.split('x'))
        f = xo.fit(cols, l, w)
        np.testing.assert_array_equal(f['scoring_prob'], g[f'{tag}_scoring_prob'])
        np.testing.assert_array_equal(f['shot_prob'], g[f'{tag}_shot_prob'])
        np.testing.assert_array_equal(f['move_prob'], g[f'{tag}_move_prob'])
        np.testing.assert_array_equal(f['transition'], g[f'{tag}_transition'])
        assert f['heatmaps'].shape == g[f'{tag}_heatmaps'].shape  # same iteration count
        np.testing.assert_array_equal(f['xT'], g[f'{tag}_xT'])  # bit-exact summation order
        assert_close(xo.rate(cols, g[f'{tag}_xT']), g[f'{tag}_rate'], 'rate')
        if f'{tag}_rate_interp' in g:
            assert_close(xo.rate(cols, g[f'{tag}_xT'], True), g[f'{tag}_rate_interp'], 'interp')


def _xt105():
    with np.load(os.path.join(GOLDEN, 'xt105_interp.npz'), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def test_xt105_interpolated_rate_oracle():
    """cfg5's rate(use_interpolation=True) at 105 x 68 (reference-generated golden,
    tests/golden/make_golden_xt105.py): surface sample and per-action ratings."""
    g = _xt105()
    cols = inputs(g)
    rows, cs = g['grid_rows'], g['grid_cols']
    for tag in ('fit', 'random'):
        xT = g[f'{tag}_xT']
        assert xT.shape == (68, 105)
        assert_close(xo.interp_grid(xT)[np.ix_(rows, cs)], g[f'{tag}_grid_sample'], f'{tag} grid')
        assert_close(xo.rate(cols, xT), g[f'{tag}_rate'], f'{tag} rate')
        assert_close(xo.rate(cols, xT, True), g[f'{tag}_rate_interp'], f'{tag} interp rate')


@pytest.mark.parametrize('name', cases('dribbles'))
def test_add_dribbles_oracle(name):
    """oracle add_dribbles == the reference's spadl.base._add_dribbles (goldens)."""
    from golden_io import dribbles_frame
    from oracle import atomic_convert_oracle as co
    g = load('dribbles', name)
    df = dribbles_frame(g, 'in_')
    ref = dribbles_frame(g, 'out_')
    got = co.add_dribbles({c: df[c].to_numpy() for c in co.COLS})
    assert len(got['type_id']) == len(ref)
    for c in co.COLS:
        if c == 'original_event_id':
            np.testing.assert_array_equal(pd.isna(got[c]), ref[c].isna().to_numpy())
            continue
        np.testing.assert_array_equal(np.asarray(got[c]), ref[c].to_numpy(), err_msg=c)


@pytest.mark.parametrize('name', cases('convert'))
def test_convert_oracle(name):
    """oracle/atomic_convert_oracle.py == the reference's convert_to_atomic (goldens)."""
    from golden_io import assert_convert_equal, convert_input, convert_output
    from oracle import atomic_convert_oracle as co
    g = load('convert', name)
    df = convert_input(g)
    got = co.convert_to_atomic({c: df[c].to_numpy() for c in co.COLS})
    ref = convert_output(g)
    assert_convert_equal(got, ref, name)
    # floats are produced by the same operations as the reference: bit-exact here
    for c in ('time_seconds', 'x', 'y', 'dx', 'dy'):
        np.testing.assert_array_equal(got[c], ref[c], err_msg=f'{name} {c}')


def test_tree_oracle_matches_sklearn_predict_proba():
    """The tree walk of oracle/tree_oracle.py (float64, x <= threshold) equals scikit-learn's
    own HistGradientBoostingClassifier.predict_proba on VAEP features of a golden game, incl.
    missing values."""
    from sklearn.ensemble import HistGradientBoostingClassifier

    from oracle import tree_oracle as to
    g = load('spadl', 'full0')
    X = np.concatenate([g['k3_feat_b'].astype(np.float64), g['k3_feat_f'],
                        g['k3_feat_i'].astype(np.float64)], axis=1)
    y = g['scores'].astype(int)
    y[::7] = 1  # enough positives to grow real trees
    X = X.copy()
    X[::13, 520] = np.nan
    clf = HistGradientBoostingClassifier(max_iter=30, max_depth=3, random_state=0).fit(X, y)
    np.testing.assert_allclose(to.predict_sklearn_nodes(clf, X), clf.predict_proba(X)[:, 1],
                               rtol=1e-12, atol=0)


def test_tree_oracle_xgboost_rules():
    """Hand-checked xgboost rules: x < threshold goes left (equality goes right), NaN follows
    default_left, leaves sum in tree order in float32 onto logit(base_score)."""
    from oracle import tree_oracle as to
    tree = {'left_children': [1, -1, -1], 'right_children': [2, -1, -1],
            'split_indices': [0, 0, 0], 'split_conditions': [1.0, -0.5, 0.25],
            'default_left': [1, 0, 0]}
    model = {'learner': {'objective': {'name': 'binary:logistic'},
                         'learner_model_param': {'base_score': '5E-1'},
                         'gradient_booster': {'model': {'trees': [tree, tree]}}}}
    X = np.array([[0.5], [1.0], [2.0], [np.nan]])
    p = to.predict_xgboost_json(model, X)
    m = np.array([-1.0, 0.5, 0.5, -1.0], np.float32)
    np.testing.assert_array_equal(p, (1 / (1 + np.exp(-m))).astype(np.float32))
