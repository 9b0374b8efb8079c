"""GPU tests of the pandas drop-in API, written like the reference's own tests
(tests/vaep/test_vaep.py, tests/atomic/test_atomic_vaep.py, tests/test_xthreat.py) but
checked value-for-value against the golden outputs of the reference."""
import numpy as np
import pandas as pd
import pytest

from golden_io import assert_close, cases, frame, ks, load

pytestmark = pytest.mark.gpu


class _Game:
    def __init__(self, home):
        self.home_team_id = home


class _FixedModel:
    """predict_proba returning fixed probabilities (stands in for the fitted learner)."""

    def __init__(self, p):
        self.p = np.asarray(p)

    def predict_proba(self, X):
        assert len(X) == len(self.p)
        return np.stack([1 - self.p, self.p], axis=1)


def _frame_equal(df, g, k):
    assert list(df.columns) == list(g[f'k{k}_names_all'])
    kinds = list(g[f'k{k}_kinds_all'])
    for kind, dt in (('b', np.bool_), ('f', np.float64), ('i', np.int64)):
        cols = [c for c, kk in zip(df.columns, kinds) if kk == kind]
        ref = g[f'k{k}_feat_{kind}']
        if not cols:
            continue
        assert all(df[c].dtype == dt for c in cols), kind
        got = df[cols].to_numpy()
        if kind == 'f':
            assert_close(got, ref, 'features')
        else:
            np.testing.assert_array_equal(got.astype(ref.dtype), ref)
    assert isinstance(df.index, pd.RangeIndex)


@pytest.mark.parametrize('atomic', [False, True])
def test_compute_features_labels_rate(atomic):
    if atomic:
        from socceraction_amd.atomic.vaep import AtomicVAEP as Model
        prefix, gfs = 'atomic', 'goal'
    else:
        from socceraction_amd.vaep import VAEP as Model
        prefix, gfs = 'spadl', 'goal_from_shot'
    for name in cases(prefix):
        g = load(prefix, name)
        df = frame(g, atomic)
        game = _Game(g['home_team_id'][0])
        for k in ks(g):
            model = Model(nb_prev_actions=k)
            _frame_equal(model.compute_features(game, df), g, k)
        model = Model()
        y = model.compute_labels(game, df)
        assert list(y.columns) == ['scores', 'concedes'] and y.dtypes.eq(bool).all()
        np.testing.assert_array_equal(y['scores'].to_numpy(), g['scores'].astype(bool))
        np.testing.assert_array_equal(y['concedes'].to_numpy(), g['concedes'].astype(bool))
        model.yfns = model.yfns + [model._lab.goal_from_shot]
        y = model.compute_labels(game, df)
        np.testing.assert_array_equal(y[gfs].to_numpy(), g['goal_from_shot'].astype(bool))
        # rate() with injected models (learners absent from the image), f64 and f32
        for tag, dt in (('64', np.float64), ('32', np.float32)):
            m = Model()
            m._VAEP__models = {'scores': _FixedModel(g['ps'].astype(dt)),
                               'concedes': _FixedModel(g['pc'].astype(dt))}
            v = m.rate(game, df)
            assert list(v.columns) == ['offensive_value', 'defensive_value', 'vaep_value']
            for c in v.columns:
                ref = g[f'{c}_{tag}']
                assert v[c].dtype == ref.dtype, (c, v[c].dtype)
                if tag == '64':
                    assert_close(v[c].to_numpy(), ref, c)
                else:  # float32: bit-exact (the reference's f32 operations in its order)
                    np.testing.assert_array_equal(v[c].to_numpy(), ref, err_msg=c)


def test_rate_errors():
    from sklearn.exceptions import NotFittedError

    from socceraction_amd.vaep import VAEP
    g = load('spadl', 'fixture')
    df = frame(g)
    game = _Game(g['home_team_id'][0])
    model = VAEP()
    with pytest.raises(NotFittedError):
        model.rate(game, df)
    model._VAEP__models = {'scores': _FixedModel(g['ps']), 'concedes': _FixedModel(g['pc'])}
    X = model.compute_features(game, df)
    del X['period_id_a0']
    with pytest.raises(ValueError):  # reference tests/vaep/test_vaep.py:423-431
        model.rate(game, df, X)
    with pytest.raises(ValueError):
        model.fit(X, model.compute_labels(game, df))


@pytest.mark.parametrize('atomic', [False, True])
@pytest.mark.parametrize('case,k', [('n300', 3), ('widek_n300', 12), ('widek_fixture', 17)])
def test_module_level_transformers(atomic, case, k):
    """Each transformer called on a user-built game-state list equals the reference, including
    game states of more frames than one launch takes (k = 12, 17: the frames go in groups)."""
    if atomic:
        from socceraction_amd.atomic.vaep import base, features as fs
        from socceraction_amd.atomic import spadl as sp
        prefix = 'atomic'
    else:
        from socceraction_amd.vaep import base, features as fs
        from socceraction_amd import spadl as sp
        prefix = 'spadl'
    g = load(prefix, case)
    df = sp.add_names(frame(g, atomic))
    gs = fs.play_left_to_right(fs.gamestates(df, k), g['home_team_id'][0])
    X = pd.concat([f(gs) for f in base.xfns_default], axis=1)
    _frame_equal(X.reset_index(drop=True), g, k)
    one = fs.actiontype_onehot.__wrapped__(df)
    assert one.columns[0] == 'type_pass'


def test_labels_and_formula_modules_single_segment():
    """Module-level functions treat the whole frame as one segment (no game_id split)."""
    from socceraction_amd import spadl as sp
    from socceraction_amd.vaep import formula, labels
    g = load('spadl', 'concat2')
    df = sp.add_names(frame(g))
    np.testing.assert_array_equal(labels.scores(df)['scores'].to_numpy(), g['scores'].astype(bool))
    np.testing.assert_array_equal(labels.concedes(df)['concedes'].to_numpy(),
                                  g['concedes'].astype(bool))
    np.testing.assert_array_equal(labels.goal_from_shot(df)['goal_from_shot'].to_numpy(),
                                  g['goal_from_shot'].astype(bool))
    v = formula.value(df, pd.Series(g['ps']), pd.Series(g['pc']))
    for c in v.columns:
        assert_close(v[c].to_numpy(), g[f'{c}_64'], c)
    v32 = formula.value(df, pd.Series(g['ps'].astype(np.float32)),
                        pd.Series(g['pc'].astype(np.float32)))
    assert v32.dtypes.eq(np.float32).all()
    off = formula.offensive_value(df, pd.Series(g['ps']), pd.Series(g['pc']))
    assert_close(off.to_numpy(), g['offensive_value_64'], 'offensive')


def test_atomic_goal_from_shot_label():
    """reference tests/atomic/test_atomic_vaep.py:6-22."""
    from socceraction_amd.atomic.spadl import config as spadlconfig
    from socceraction_amd.atomic.vaep import labels as lab
    df = pd.DataFrame([spadlconfig.actiontypes.index('shot'), spadlconfig.actiontypes.index('goal')],
                      columns=['type_id'])
    df['team_id'] = 1
    out = lab.goal_from_shot(df)
    assert (out == pd.DataFrame([[True], [False]], columns=['goal']))['goal'].all()


@pytest.mark.parametrize('atomic', [False, True])
def test_batched_api_equals_per_game(atomic):
    if atomic:
        from socceraction_amd.atomic.vaep import AtomicVAEP as Model
        prefix = 'atomic'
    else:
        from socceraction_amd.vaep import VAEP as Model
        prefix = 'spadl'
    names = [c for c in cases(prefix) if c != 'concat2']
    gs = [load(prefix, c) for c in names]
    dfs = []
    for i, g in enumerate(gs):
        d = frame(g, atomic)
        d['game_id'] = i
        dfs.append(d)
    actions = pd.concat(dfs, ignore_index=True)
    games = pd.DataFrame({'game_id': range(len(gs)), 'home_team_id': [g['home_team_id'][0] for g in gs]})
    model = Model()
    X = model.compute_features_batch(games, actions)
    Y = model.compute_labels_batch(games, actions)
    per = [model.compute_features(_Game(g['home_team_id'][0]), d) for g, d in zip(gs, dfs)]
    pd.testing.assert_frame_equal(X, pd.concat(per, ignore_index=True))
    np.testing.assert_array_equal(Y['scores'].to_numpy(),
                                  np.concatenate([g['scores'] for g in gs]).astype(bool))
    model._VAEP__models = {'scores': _FixedModel(np.concatenate([g['ps'] for g in gs])),
                           'concedes': _FixedModel(np.concatenate([g['pc'] for g in gs]))}
    v = model.rate_batch(games, actions, X)
    assert_close(v['vaep_value'].to_numpy(), np.concatenate([g['vaep_value_64'] for g in gs]), 'vaep')


@pytest.mark.parametrize('atomic', [False, True])
def test_pipelined_compute_batch_equals_separate_calls(atomic):
    """VAEP.compute_batch (socceraction_amd.pipeline: one encode, game-aligned chunks, the
    chunks' blocks copied out by pitched DMAs while the host encodes the next) == the separate
    batched calls, frame for frame: features (names, dtypes, values), labels incl.
    goal_from_shot, and the formula values in float64 and float32 -- with chunks small enough
    that both device slots are reused several times, and with one chunk."""
    import torch

    from socceraction_amd import ops, synthetic
    from socceraction_amd.batch import ActionBatch
    if atomic:
        from socceraction_amd.atomic.vaep import AtomicVAEP as Model
        d = synthetic.atomic_games(40, game_id0=3)
    else:
        from socceraction_amd.vaep import VAEP as Model
        d = synthetic.spadl_games(40, game_id0=3)
    actions = synthetic.to_frame(d, atomic=atomic)
    games = synthetic.games_frame(d)
    model = Model()
    model.yfns = model.yfns + [model._lab.goal_from_shot]
    # the reference frame from the per-game calls (compute_features_batch itself now takes the
    # pipelined path, features only: it must equal them too)
    X = pd.concat([model.compute_features(g, actions[actions['game_id'] == g.game_id].reset_index(drop=True))
                   for g in games.itertuples()], ignore_index=True)
    pd.testing.assert_frame_equal(model.compute_features_batch(games, actions), X)
    Y = model.compute_labels_batch(games, actions)
    n = len(actions)
    p = synthetic.probabilities(n)
    for chunk in (5000, 1 << 20):
        for dt in (np.float64, np.float32):
            ps, pc = p['scores'].astype(dt), p['concedes'].astype(dt)
            X2, Y2, V2 = model.compute_batch(games, actions, ps, pc, chunk_rows=chunk)
            pd.testing.assert_frame_equal(X2, X)
            pd.testing.assert_frame_equal(Y2, Y)
            ab = ActionBatch.from_frame(actions, atomic=atomic, segments='game')
            ref = ops.formula(ab, torch.from_numpy(ps).cuda(), torch.from_numpy(pc).cuda()).cpu().numpy()
            for r, c in enumerate(('offensive_value', 'defensive_value', 'vaep_value')):
                assert V2[c].dtype == dt
                np.testing.assert_array_equal(V2[c].to_numpy(), ref[r, :n], err_msg=c)
    X3, Y3, V3 = model.compute_batch(games, actions, chunk_rows=7000)
    pd.testing.assert_frame_equal(X3, X)
    pd.testing.assert_frame_equal(Y3, Y)
    assert V3 is None


def test_user_transformer_runs_on_host_gamestates():
    from socceraction_amd.vaep import VAEP
    from socceraction_amd.vaep import features as fs

    @fs.simple
    def double_x(actions):
        return pd.DataFrame({'double_x': actions['start_x'] * 2})

    g = load('spadl', 'n40')
    df = frame(g)
    game = _Game(g['home_team_id'][0])
    X = VAEP(xfns=[fs.startlocation, double_x, fs.goalscore], nb_prev_actions=2).compute_features(game, df)
    assert list(X.columns)[:6] == ['start_x_a0', 'start_y_a0', 'start_x_a1', 'start_y_a1',
                                   'double_x_a0', 'double_x_a1']
    np.testing.assert_array_equal(X['double_x_a0'].to_numpy(), 2 * X['start_x_a0'].to_numpy())
    np.testing.assert_array_equal(X['double_x_a1'].to_numpy(), 2 * X['start_x_a1'].to_numpy())


# ----------------------------------------------------------------------------- xT
def test_xt_fit_rate_match_reference():
    from socceraction_amd import xthreat as xt
    for name in cases('xt'):
        g = load('xt', name)
        df = frame(g)
        for tag in sorted({k.split('_')[0] for k in g if k[0].isdigit()}):
            l, w = map(int, tag.split('x'))
            m = xt.ExpectedThreat(l=l, w=w).fit(df)
            np.testing.assert_array_equal(m.scoring_prob_matrix, g[f'{tag}_scoring_prob'])
            np.testing.assert_array_equal(m.shot_prob_matrix, g[f'{tag}_shot_prob'])
            np.testing.assert_array_equal(m.move_prob_matrix, g[f'{tag}_move_prob'])
            np.testing.assert_array_equal(m.transition_matrix, g[f'{tag}_transition'])
            np.testing.assert_array_equal(m.xT, g[f'{tag}_xT'])
            assert len(m.heatmaps) == len(g[f'{tag}_heatmaps'])
            r = m.rate(df)
            assert r.dtype == np.float64 and r.shape == (len(df),)
            assert_close(r, g[f'{tag}_rate'], 'rate')
            if f'{tag}_rate_interp' in g:
                assert_close(m.rate(df, use_interpolation=True), g[f'{tag}_rate_interp'], 'interp')
            sp = xt.scoring_prob(df, l, w)
            np.testing.assert_array_equal(sp, g[f'{tag}_scoring_prob'])
            shot_p, move_p = xt.action_prob(df, l, w)
            np.testing.assert_array_equal(move_p, g[f'{tag}_move_prob'])
            np.testing.assert_array_equal(xt.move_transition_matrix(df, l, w),
                                          g[f'{tag}_transition'])


def test_xt_reference_known_answers():
    """reference tests/test_xthreat.py:80-85, 157-193, 223-238."""
    from socceraction_amd import xthreat as xt
    x = pd.Series([0, 105 / 2 - 1, 105.0, 115.0])
    y = pd.Series([0, 68 / 2 + 1, 68.0, 78.0])
    np.testing.assert_array_equal(xt._count(x, y, 2, 2), [[1, 2], [1, 0]])
    two = pd.DataFrame([{'game_id': 1, 'period_id': 1, 'time_seconds': t, 'team_id': 1,
                         'start_x': 10.0, 'end_x': 10.0, 'start_y': 10.0, 'end_y': 10.0,
                         'bodypart_id': 1, 'type_id': 0, 'result_id': 1} for t in (1.0, 1.2)])
    mm = xt.move_transition_matrix(two, 2, 2)
    assert np.sum(mm) == 1 and mm.shape == (4, 4) and mm[2, 2] == 1
    g = load('xt', 'fixture')
    df = frame(g)
    shot_p, move_p = xt.action_prob(df, 10, 5)
    assert shot_p.shape == (5, 10) and np.any(shot_p > 0) and np.any(move_p > 0)
    assert np.all(((move_p + shot_p) == 1) | ((move_p + shot_p) == 0))
    shots = df.type_id == 11
    goals = shots & (df.result_id == 1)
    assert sum(goals) / sum(shots) == xt.scoring_prob(df, 1, 1)[0]
    m = xt.ExpectedThreat().fit(df)
    idx = xt.get_successful_move_actions(df).index
    r = m.rate(df)
    assert np.all(~np.isnan(r[idx])) and np.all(np.isnan(np.delete(r, idx)))
    nan = df.copy()
    nan.loc[idx[0], 'end_x'] = np.nan
    with pytest.raises(ValueError):
        m.rate(nan)
    f = m.interpolator()
    grid = f(np.linspace(0, 105, 7), np.linspace(0, 68, 5))
    assert grid.shape == (5, 7)


def test_xt_large_grid_multi_launch_solver():
    """C = 40*30 = 1200 > 1024 cells: the large-grid solve.  exact_order=True sums in the
    reference's order (bit-exact with the oracle); the default reordered sums keep the oracle's
    iteration count and every heatmap within 1e-12 relative (the error-bound guard)."""
    from oracle import xt_oracle as xo
    from socceraction_amd import synthetic
    from socceraction_amd import xthreat as xt
    d = synthetic.spadl_games(4, seed=77)
    df = synthetic.to_frame(d)
    cols = {c: d[c] for c in ('start_x', 'start_y', 'end_x', 'end_y', 'type_id', 'result_id')}
    for l, w in ((40, 30),):
        f = xo.fit(cols, l, w)
        m = xt.ExpectedThreat(l=l, w=w).fit(df, exact_order=True)
        assert len(m.heatmaps) == len(f['heatmaps'])
        np.testing.assert_array_equal(m.xT, f['xT'])
        r = xt.ExpectedThreat(l=l, w=w).fit(df)
        assert r.solve_path in ('reordered', 'sequential')
        assert len(r.heatmaps) == len(f['heatmaps'])
        for a, b in zip(r.heatmaps, f['heatmaps']):
            np.testing.assert_allclose(a, b, rtol=1e-12, atol=1e-300)


@pytest.mark.parametrize('grid,mode', [('105x68', 'bands'), ('105x68', 'bands-rows'), ('105x68', 'rows'),
                                       ('40x30', 'bands'), ('16x12', 'rows')])
def test_xt_row_sharded_solve_two_ranks(grid, mode):
    """The row-sharded fits with two ranks over gloo on this GPU, each counting its own games,
    reproduce bit for bit the single-GPU fit of all the games (matrices, heatmaps, iteration
    count): shard.xt_solve_sharded (rows: all-reduce of the count vectors, reduce-scatter of the
    transition rows) and shard.xt_fit_bands_sharded (all-to-all of the counted actions, each
    rank counting its own bands; bands: the compact rows all-gathered once and every rank
    iterating all rows; bands-rows: a per-iteration all-gather of x).  The ranks run
    as child processes of torch.distributed.run (scripts/rehearse_xt_sharded.py checks and
    prints the verdict)."""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, SA_DIST_BACKEND='gloo', MASTER_ADDR='127.0.0.1')
    port = 29600 + (os.getpid() % 200) + 211 * ['105x68bands', '105x68rows', '40x30bands',
                                                '16x12rows', '105x68bands-rows'].index(grid + mode)
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', '--nproc-per-node', '2',
           '--master-addr', '127.0.0.1', '--master-port', str(port),
           os.path.join(root, 'scripts', 'rehearse_xt_sharded.py'), '--games', '40', '--grid', grid,
           '--mode', mode]
    r = subprocess.run(cmd, cwd=root, env=env, capture_output=True, text=True, timeout=110)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith('{')]
    assert r.returncode == 0 and lines, r.stdout[-2000:] + r.stderr[-2000:]
    out = json.loads(lines[-1])
    assert out['world'] == 2 and out['grid'] == grid and out['mode'] == mode
    assert out['ok'] and out['bit_identical_matrices'] and out['bit_identical_heatmaps']
    assert out['iterations'] == out['single_iterations']


def test_xt_module_functions_on_nan_move_ends():
    """The reference's scoring_prob never reads moves and action_prob reads only their (NaN
    dropped) starts, so NaN / inf end coordinates on passes leave both computable; only
    move_transition_matrix (and fit) cast every move coordinate and raise
    (xthreat.py:40-67, 74-98, 144-174, 177-218)."""
    from oracle import xt_oracle as xo
    from socceraction_amd import synthetic
    from socceraction_amd import xthreat as xt
    d = synthetic.spadl_games(6, seed=17)
    n = len(d['type_id'])
    rng = np.random.default_rng(3)
    moves = np.nonzero(np.isin(d['type_id'], (0, 1, 21)))[0]
    d['end_x'][rng.choice(moves, 25, replace=False)] = np.nan
    d['end_y'][rng.choice(moves, 5, replace=False)] = np.inf
    nan_start = rng.choice(moves, 9, replace=False)
    d['start_y'][nan_start] = np.nan  # dropped by _count, cast (raise) by the transition matrix
    df = synthetic.to_frame(d)
    cols = {c: d[c] for c in ('type_id', 'result_id', 'start_x', 'start_y', 'end_x', 'end_y')}
    ref = xo.fit(cols, 16, 12)  # its count() drops NaN starts like _count
    np.testing.assert_array_equal(xt.scoring_prob(df), ref['scoring_prob'])
    ps, pm = xt.action_prob(df)
    np.testing.assert_array_equal(ps, ref['shot_prob'])
    np.testing.assert_array_equal(pm, ref['move_prob'])
    with pytest.raises(ValueError):
        xt.move_transition_matrix(df)
    with pytest.raises(ValueError):
        xt.ExpectedThreat().fit(df)
    # an infinite move START raises in action_prob too, but not in scoring_prob
    d['start_y'][nan_start] = d['start_x'][nan_start]
    d['start_x'][moves[0]] = np.inf
    df = synthetic.to_frame(d)
    with pytest.raises(ValueError):
        xt.action_prob(df)
    assert xt.scoring_prob(df).shape == (12, 16)
    assert n == len(df)


def test_interp2d_uses_the_given_nodes():
    """xthreat.interp2d(x, y, z) interpolates between the nodes it is given (not always the
    cell centres): the oracle's bilinear rule on shifted, unevenly spaced nodes."""
    from socceraction_amd import xthreat as xt
    rng = np.random.default_rng(8)
    z = rng.random((5, 7))
    x = np.cumsum(rng.random(7) + 0.5)
    y = np.cumsum(rng.random(5) + 0.5)
    xs, ys = np.linspace(-1, x[-1] + 1, 41), np.linspace(-1, y[-1] + 1, 37)
    got = xt.interp2d(x=x, y=y, z=z, kind='linear', bounds_error=False)(xs, ys)

    def br(c, q):
        q = np.clip(q, c[0], c[-1])
        i = np.clip(np.searchsorted(c, q, side='right') - 1, 0, len(c) - 2)
        return i, (q - c[i]) / (c[i + 1] - c[i])
    i, tx = br(x, xs)
    j, ty = br(y, ys)
    ref = ((1 - tx) * z[j][:, i] + tx * z[j][:, i + 1]) * (1 - ty)[:, None] + \
        ((1 - tx) * z[j + 1][:, i] + tx * z[j + 1][:, i + 1]) * ty[:, None]
    assert_close(got, ref, 'interp2d nodes')
    with pytest.raises(ValueError):
        xt.interp2d(x=x[::-1], y=y, z=z)
