"""GPU tree inference on the feature blocks (the predict_proba step of VAEP.rate,
reference vaep/base.py:284-333) and the device rate path.

scikit-learn HistGradientBoostingClassifier: pinned against its own predict_proba (float64,
rtol 1e-12). xgboost-format models (xgboost is not installed): against the numpy restatement in
oracle/tree_oracle.py (float32; within 1e-6 relative: expf vs numpy exp can differ in the last
bit). Features come from the golden games' device blocks, in the reference's column order.
"""
import numpy as np
import pandas as pd
import pytest

from golden_io import assert_close, frame, load

pytestmark = pytest.mark.gpu

torch = pytest.importorskip('torch')


@pytest.fixture(scope='module')
def sa():
    from socceraction_amd import _native, batch, ops, trees
    _native.load_library()
    return dict(batch=batch, ops=ops, trees=trees)


def _game(sa, name='full0'):
    from oracle import vaep_oracle as vo
    g = load('spadl', name)
    df = frame(g)
    ab = sa['batch'].ActionBatch.from_frame(df, home_team_id=g['home_team_id'][0])
    fb = sa['ops'].features(ab, vo.SPADL_DEFAULT, 3)
    b, f, i = fb.to_numpy()
    blocks = {'b': b, 'f': f, 'i': i}
    X = np.stack([blocks[k][c, :fb.n].astype(np.float64) for _, k, c in fb.plan.order], axis=1)
    return g, df, ab, fb, X


def test_sklearn_hgb_on_device_equals_predict_proba(sa):
    from sklearn.ensemble import HistGradientBoostingClassifier
    g, df, ab, fb, X = _game(sa)
    y = g['scores'].astype(int).copy()
    y[::5] = 1
    Xdf = pd.DataFrame(X, columns=fb.plan.names)
    clf = HistGradientBoostingClassifier(max_iter=40, max_depth=4, random_state=0).fit(Xdf, y)
    te = sa['trees'].TreeEnsemble.from_model(clf)
    assert te is not None and te.feature_names == fb.plan.names
    p = te.predict_blocks(fb).cpu().numpy()
    assert p.dtype == np.float64
    np.testing.assert_allclose(p, clf.predict_proba(Xdf)[:, 1], rtol=1e-12, atol=0)


def test_xgboost_json_on_device_equals_oracle(sa):
    from oracle import tree_oracle as to
    g, df, ab, fb, X = _game(sa)
    kinds = [k for _, k, _ in fb.plan.order]
    model = sa['trees'].synthetic_xgboost_json(len(kinds), n_trees=100, depth=3, seed=3,
                                               feature_kinds=kinds, base_score=0.3)
    te = sa['trees'].TreeEnsemble.from_model(model)
    p = te.predict_blocks(fb).cpu().numpy()
    assert p.dtype == np.float32
    ref = to.predict_xgboost_json(model, X)
    np.testing.assert_allclose(p, ref, rtol=1e-6, atol=0)


@pytest.mark.parametrize('kind', ['xgboost', 'sklearn'])
def test_fixed_depth_walk_equals_leaf_checked_walk(sa, kind):
    """The fixed-depth walk (per-tree depths given) and the leaf-checked walk (no depths) give
    bit-identical probabilities, on unbalanced scikit-learn trees too."""
    g, df, ab, fb, X = _game(sa)
    kinds = [k for _, k, _ in fb.plan.order]
    if kind == 'xgboost':
        model = sa['trees'].synthetic_xgboost_json(len(kinds), n_trees=37, depth=4, seed=5,
                                                   feature_kinds=kinds)
    else:
        from sklearn.ensemble import HistGradientBoostingClassifier
        y = g['scores'].astype(int).copy()
        y[::3] = 1
        model = HistGradientBoostingClassifier(max_iter=30, max_leaf_nodes=9,
                                               random_state=0).fit(X, y)
    te = sa['trees'].TreeEnsemble.from_model(model)
    assert te is not None and te.depths().max() >= 3
    fixed = te.predict_blocks(fb, method='gather').cpu().numpy()
    te._dev['depth'] = None
    walked = te.predict_blocks(fb, method='gather').cpu().numpy()
    np.testing.assert_array_equal(fixed, walked)


def test_missing_values_follow_default_direction(sa):
    """NaN written into a device feature column takes default_left, like the oracle."""
    from oracle import tree_oracle as to
    g, df, ab, fb, X = _game(sa)
    kinds = [k for _, k, _ in fb.plan.order]
    fcols = [j for j, k in enumerate(kinds) if k == 'f']
    model = sa['trees'].synthetic_xgboost_json(len(kinds), n_trees=50, depth=3, seed=4,
                                               feature_kinds=kinds)
    used = sorted({j for t in model['learner']['gradient_booster']['model']['trees']
                   for j, lc in zip(t['split_indices'], t['left_children']) if lc >= 0} & set(fcols))
    j = used[0]
    col = fb.plan.order[j][2]
    rows = np.arange(0, fb.n, 3)
    blk = fb.f64_block  # [tiles, C, R]; one tile here
    blk[0, col, torch.from_numpy(rows).to(blk.device)] = float('nan')
    X = X.copy()
    X[rows, j] = np.nan
    te = sa['trees'].TreeEnsemble.from_model(model)
    np.testing.assert_allclose(te.predict_blocks(fb).cpu().numpy(),
                               to.predict_xgboost_json(model, X), rtol=1e-6, atol=0)


def test_vaep_rate_on_device(sa):
    """VAEP.rate / rate_batch with tree learners: features, predict_proba and formula on the
    device == the reference's host path (host predict_proba on compute_features output ->
    formula.value)."""
    from oracle import vaep_oracle as vo
    from socceraction_amd import synthetic
    import socceraction_amd.vaep as vaep
    from sklearn.ensemble import HistGradientBoostingClassifier
    d = synthetic.spadl_games(6, seed=21)
    actions = synthetic.to_frame(d)
    games = synthetic.games_frame(d)
    model = vaep.VAEP()
    X = model.compute_features_batch(games, actions)
    Y = model.compute_labels_batch(games, actions)
    sk = {c: HistGradientBoostingClassifier(max_iter=20, max_depth=3, random_state=0)
          .fit(X, Y[c]) for c in ('scores', 'concedes')}
    model._VAEP__models = sk
    got = model.rate_batch(games, actions)
    assert list(got.columns) == ['offensive_value', 'defensive_value', 'vaep_value']
    off = d['game_off']
    for gi in range(len(off) - 1):
        s, e = int(off[gi]), int(off[gi + 1])
        cols = {c: d[c][s:e] for c in ('period_id', 'time_seconds', 'team_id', 'type_id',
                                       'result_id')}
        ps = sk['scores'].predict_proba(X.iloc[s:e])[:, 1]
        pc = sk['concedes'].predict_proba(X.iloc[s:e])[:, 1]
        fo = vo.formula(cols, ps, pc)
        for c in ('offensive_value', 'defensive_value', 'vaep_value'):
            assert_close(got[c].to_numpy()[s:e], fo[c], c)
    # per-game rate through the drop-in (device path) == the batched values
    g0 = games.iloc[0]
    one = model.rate(g0, actions[actions.game_id == g0.game_id].reset_index(drop=True))
    assert_close(one['vaep_value'].to_numpy(), got['vaep_value'].to_numpy()[:len(one)], 'rate')
    # xgboost-format learners: float32 probabilities -> float32 values (the reference's dtype)
    kinds = ['f'] * X.shape[1]
    xg = {c: sa['trees'].synthetic_xgboost_json(X.shape[1], n_trees=20, seed=s, feature_kinds=kinds)
          for s, c in enumerate(('scores', 'concedes'))}
    model._VAEP__models = xg
    got32 = model.rate_batch(games, actions)
    assert got32['vaep_value'].dtype == np.float32


@pytest.mark.parametrize('kind', ['xgboost', 'sklearn', 'xgboost_bool_only', 'xgboost_num_only',
                                  'depth1', 'depth5', 'plain_layout'])
def test_staged_walk_equals_gather_walk(sa, kind):
    """The staged condition walk (every split a condition bit in LDS) gives the gather walk's
    probabilities bit for bit: float32 xgboost / float64 scikit-learn models (unbalanced trees),
    bool-only and numeric-only models, depths 1 - 5, several tiles and a ragged last workgroup
    (300 games), NaN in a numeric feature, tiled and plain column-major blocks."""
    from socceraction_amd import synthetic
    from oracle import vaep_oracle as vo
    B, ops, trees = sa['batch'], sa['ops'], sa['trees']
    d = synthetic.spadl_games(300, seed=8)
    ab = B.ActionBatch.from_columns(d)
    tiles = (None, None) if kind == 'plain_layout' else (1024, 128)
    fb = ops.features(ab, vo.SPADL_DEFAULT, 3, bool_tile=tiles[0], num_tile=tiles[1])
    assert fb.n % 512 != 0
    kinds = [k for _, k, _ in fb.plan.order]
    depth = {'depth1': 1, 'depth5': 5}.get(kind, 3)
    if kind != 'sklearn':
        model = trees.synthetic_xgboost_json(len(kinds), n_trees=100, depth=depth, seed=11,
                                             feature_kinds=kinds)
        keep = {'xgboost_bool_only': 'b', 'xgboost_num_only': 'fi'}.get(kind)
        if keep:  # re-point every split at a feature of the wanted kinds
            cand = [j for j, k in enumerate(kinds) if k in keep]
            rng = np.random.default_rng(2)
            for t in model['learner']['gradient_booster']['model']['trees']:
                t['split_indices'] = [int(rng.choice(cand)) for _ in t['split_indices']]
        te = trees.TreeEnsemble.from_model(model)
    else:
        from sklearn.ensemble import HistGradientBoostingClassifier
        n = 20000
        b, f, i = fb.to_numpy()
        blocks = {'b': b, 'f': f, 'i': i}
        X = np.stack([blocks[k][c, :n].astype(np.float64) for _, k, c in fb.plan.order], axis=1)
        y = (X[:, 0] + np.random.default_rng(0).random(n) > 0.7).astype(int)
        te = trees.TreeEnsemble.from_model(
            HistGradientBoostingClassifier(max_iter=40, max_leaf_nodes=11, random_state=0).fit(X, y))
        assert te.depths().min() < te.depths().max()
    fcol = [c for _, k, c in fb.plan.order if k == 'f'][5]
    fb.f64_block[:, fcol, ::7] = float('nan')
    got = te.predict_blocks(fb, method='staged').cpu().numpy()
    ref = te.predict_blocks(fb, method='gather').cpu().numpy()
    np.testing.assert_array_equal(got, ref)
    np.testing.assert_array_equal(te.predict_blocks(fb).cpu().numpy(), ref)  # the default path


@pytest.mark.parametrize('atomic,k', [(False, 3), (True, 3), (False, 1), (False, 2), (True, 2)])
def test_bool_bitmap_features_and_trees(sa, atomic, k):
    """sa_vaep_features_bits: the bool features as bitmaps equal the bool block bit for bit
    (rows >= n clear), the f64 / i64 blocks are unchanged, host export of the bitmap form equals
    the block form, and the staged walk reading the bitmaps equals the walk reading the block
    (float32 xgboost, float64 scikit-learn) -- the on-device VAEP.rate path."""
    from socceraction_amd import synthetic, catalog
    from oracle import vaep_oracle as vo
    from sklearn.ensemble import HistGradientBoostingClassifier
    B, ops, trees = sa['batch'], sa['ops'], sa['trees']
    if atomic:
        d = synthetic.atomic_games(150, seed=6)
        xfns = ['actiontype', 'actiontype_onehot', 'bodypart', 'bodypart_onehot', 'time', 'team',
                'time_delta', 'location', 'polar', 'movement_polar', 'direction', 'goalscore']
    else:
        d = synthetic.spadl_games(150, seed=6)
        xfns = vo.SPADL_DEFAULT
    ab = B.ActionBatch.from_columns(d, atomic=atomic)
    ref = ops.features(ab, xfns, k, bool_tile=1024, num_tile=128)
    got = ops.features(ab, xfns, k, num_tile=128, bool_bits=True)
    assert got.bool_block is None and ref.n % 64 != 0
    rb = ref.block('b').cpu().numpy()
    bits = got.bool_bits.cpu().numpy().view(np.uint8)
    unpacked = np.unpackbits(bits, axis=1, bitorder='little')
    np.testing.assert_array_equal(unpacked[:, :ref.n], rb)
    assert not unpacked[:, ref.n:].any()
    for kb in 'fi':
        np.testing.assert_array_equal(got.block(kb).cpu().numpy(), ref.block(kb).cpu().numpy())
    if atomic or k != 3:
        return
    kinds = [k for _, k, _ in ref.plan.order]
    xg = trees.TreeEnsemble.from_model(trees.synthetic_xgboost_json(
        len(kinds), n_trees=80, depth=3, seed=31, feature_kinds=kinds))
    n = 12000
    b, f, i = ref.to_numpy()
    X = np.stack([{'b': b, 'f': f, 'i': i}[k][c, :n].astype(np.float64) for _, k, c in ref.plan.order], axis=1)
    sk = trees.TreeEnsemble.from_model(HistGradientBoostingClassifier(
        max_iter=25, max_depth=4, random_state=0).fit(X, (X[:, 7] + np.random.default_rng(0).random(n) > 0.6)))
    for te in (xg, sk):
        a = te.predict_blocks(got, method='staged').cpu().numpy()
        np.testing.assert_array_equal(a, te.predict_blocks(ref, method='gather').cpu().numpy())
        np.testing.assert_array_equal(te.predict_blocks(got, method='gather').cpu().numpy(), a)
    pd.testing.assert_frame_equal(got.to_frame(), ref.to_frame())


@pytest.mark.parametrize('atomic', [False, True])
def test_float32_numeric_blocks_and_trees(sa, atomic):
    """sa_vaep_features_bits_f32: the numeric blocks in float32 equal the float64 / int64 blocks
    rounded to nearest (torch's cast), the bitmaps are unchanged, and the staged walk of an
    xgboost learner over them gives the probabilities of the float64 form bit for bit (xgboost
    compares float32 values); scikit-learn learners and the gather walk refuse them."""
    from socceraction_amd import synthetic
    from oracle import vaep_oracle as vo
    B, ops, trees = sa['batch'], sa['ops'], sa['trees']
    if atomic:
        d = synthetic.atomic_games(150, seed=7)
        xfns = ['actiontype', 'actiontype_onehot', 'bodypart', 'bodypart_onehot', 'time', 'team',
                'time_delta', 'location', 'polar', 'movement_polar', 'direction', 'goalscore']
    else:
        d = synthetic.spadl_games(150, seed=7)
        xfns = vo.SPADL_DEFAULT
    ab = B.ActionBatch.from_columns(d, atomic=atomic)
    ref = ops.features(ab, xfns, 3, num_tile=128, bool_bits=True)
    got = ops.features(ab, xfns, 3, num_tile=128, bool_bits=True, num32=True)
    assert got.num32 and not ref.num32
    assert torch.equal(got.bool_bits, ref.bool_bits)
    for k in 'fi':
        assert torch.equal(got.block(k), ref.block(k).to(torch.float32)), k
    kinds = [k for _, k, _ in ref.plan.order]
    for seed in (31, 32):
        xg = trees.TreeEnsemble.from_model(trees.synthetic_xgboost_json(
            len(kinds), n_trees=80, depth=3, seed=seed, feature_kinds=kinds))
        assert torch.equal(xg.predict_blocks(got), xg.predict_blocks(ref))
        with pytest.raises(ValueError):
            xg.predict_blocks(got, method='gather')
    with pytest.raises(ValueError):
        ops.features(ab, xfns, 3, num32=True)
    with pytest.raises(ValueError):
        ops.features(ab, xfns, 4, bool_bits=True, num32=True)


@pytest.mark.parametrize('case', ['spadl', 'atomic', 'numeric_only'])
def test_condition_bitmaps_match_staged_walk(sa, case):
    """sa_vaep_features_conditions + the staged walk over bitmaps only (trees.predict_pair_conditions:
    the learners' numeric split conditions evaluated inside the numeric feature pass) == each
    learner's staged walk over the feature blocks, bit for bit: two xgboost-shaped learners over
    bool and numeric (f64 and i64) features with NaN-free and NaN-routed splits, several tiles and
    a batch whose length is not a multiple of 128; and a plan with no bool column at all
    (numeric-only xfns: the condition rows start at bitmap row 0)."""
    from socceraction_amd import synthetic, catalog
    from oracle import vaep_oracle as vo
    B, ops, trees = sa['batch'], sa['ops'], sa['trees']
    atomic = case == 'atomic'
    if atomic:
        d = synthetic.atomic_games(120, seed=8)
        xfns = ['actiontype', 'actiontype_onehot', 'bodypart', 'bodypart_onehot', 'time', 'team',
                'time_delta', 'location', 'polar', 'movement_polar', 'direction', 'goalscore']
    else:
        d = synthetic.spadl_games(120, seed=8)
        xfns = ['time', 'startlocation', 'goalscore'] if case == 'numeric_only' else vo.SPADL_DEFAULT
    ab = B.ActionBatch.from_columns(d, atomic=atomic)
    assert ab.n % 128
    if case == 'numeric_only':
        ref = ops.features(ab, xfns, 3, num_tile=128)
        assert ref.plan.n_bool == 0
    else:
        ref = ops.features(ab, xfns, 3, num_tile=128, bool_bits=True)
    kinds = [k for _, k, _ in ref.plan.order]
    models = [trees.TreeEnsemble.from_model(trees.synthetic_xgboost_json(
        len(kinds), n_trees=60, depth=3, seed=sd, feature_kinds=kinds)) for sd in (41, 42)]
    got = trees.predict_pair_conditions(ab, ref.plan, models)
    for m, g in zip(models, got):
        assert torch.equal(g, m.predict_blocks(ref, method='staged'))
