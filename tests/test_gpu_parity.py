"""GPU parity: the HIP kernels (through the C ABI) against the reference goldens and the oracle.

Bar: bit-exact for ids, one-hots, labels, goal scores and counts; floats within
|a-b| <= 1e-6*|ref| + 1e-12 (see golden_io.assert_close).
"""
import numpy as np
import pytest

from golden_io import assert_close, cases, frame, inputs, ks, load
from oracle import vaep_oracle as vo
from oracle import xt_oracle as xo

pytestmark = pytest.mark.gpu

torch = pytest.importorskip('torch')


@pytest.fixture(scope='module')
def sa():
    from socceraction_amd import _native, batch, catalog, ops, synthetic
    _native.load_library()
    return dict(batch=batch, catalog=catalog, ops=ops, synthetic=synthetic)


def _blocks_match(fb, g, k, n):
    names = list(g[f'k{k}_names_all'])
    assert fb.plan.names == names
    b, f, i = fb.to_numpy()
    blocks = {'b': b, 'f': f, 'i': i}
    got = {'b': [], 'f': [], 'i': []}
    for name, kind, col in fb.plan.order:
        got[kind].append(blocks[kind][col, :n])
    for kind in 'bfi':
        ref = g[f'k{k}_feat_{kind}']
        if not got[kind]:
            assert ref.shape[1] == 0
            continue
        M = np.stack(got[kind], axis=1)
        if kind == 'f':
            assert_close(M, ref, f'k{k} f64 block')
        else:
            np.testing.assert_array_equal(M.astype(ref.dtype), ref, err_msg=f'k{k} {kind} block')


@pytest.mark.parametrize('atomic', [False, True])
def test_features_labels_formula_goldens(sa, atomic):
    B, ops = sa['batch'], sa['ops']
    default = vo.ATOMIC_DEFAULT if atomic else vo.SPADL_DEFAULT
    prefix = 'atomic' if atomic else 'spadl'
    for name in cases(prefix):
        g = load(prefix, name)
        df = frame(g, atomic)
        n = len(df)
        ab = B.ActionBatch.from_frame(df, atomic=atomic, home_team_id=g['home_team_id'][0])
        for k in ks(g):
            fb = ops.features(ab, default, k)
            _blocks_match(fb, g, k, n)
        lb = ops.labels(ab)
        np.testing.assert_array_equal(lb.scores[:n].cpu().numpy(), g['scores'], err_msg=name)
        np.testing.assert_array_equal(lb.concedes[:n].cpu().numpy(), g['concedes'], err_msg=name)
        np.testing.assert_array_equal(lb.goal_from_shot[:n].cpu().numpy(), g['goal_from_shot'],
                                      err_msg=name)
        for tag, dt in (('64', torch.float64), ('32', torch.float32)):
            ps = torch.tensor(g['ps'], dtype=dt, device=ab.device)
            pc = torch.tensor(g['pc'], dtype=dt, device=ab.device)
            v = ops.formula(ab, ps, pc).cpu().numpy()[:, :n]
            for r, c in enumerate(('offensive_value', 'defensive_value', 'vaep_value')):
                if dt == torch.float32:  # a few IEEE f32 ops in the reference's order: bit-exact
                    np.testing.assert_array_equal(v[r], g[f'{c}_{tag}'], err_msg=f'{name} {c}')
                else:
                    assert_close(v[r], g[f'{c}_{tag}'], f'{name} {c}')


@pytest.mark.parametrize('atomic', [False, True])
def test_batched_segments_match_per_game(sa, atomic):
    """Many games in one batch (one segment each) == per-game reference outputs."""
    B, ops = sa['batch'], sa['ops']
    prefix = 'atomic' if atomic else 'spadl'
    default = vo.ATOMIC_DEFAULT if atomic else vo.SPADL_DEFAULT
    names = [c for c in cases(prefix) if c != 'concat2']
    gs = [load(prefix, c) for c in names]
    import pandas as pd
    dfs = []
    for idx, g in enumerate(gs):
        d = frame(g, atomic).copy()
        d['game_id'] = idx  # one contiguous run per case
        dfs.append(d)
    df = pd.concat(dfs, ignore_index=True)
    homes = [g['home_team_id'][0] for g in gs]
    ab = B.ActionBatch.from_frame(df, atomic=atomic, home_team_id=homes, segments='game')
    assert ab.n_segments == len(gs)
    fb = ops.features(ab, default, 3, bool_tile=1024, num_tile=128)  # tiled, several tiles
    assert fb.bool_block.shape[0] == -(-ab.n // 1024)
    lb = ops.labels(ab)
    ps = torch.tensor(np.concatenate([g['ps'] for g in gs]), device=ab.device)
    pc = torch.tensor(np.concatenate([g['pc'] for g in gs]), device=ab.device)
    v = ops.formula(ab, ps, pc).cpu().numpy()
    b, f, i = fb.to_numpy()
    o = 0
    for g in gs:
        n = len(g['type_id'] if 'type_id' in g else g['in_type_id'])
        sl = slice(o, o + n)
        blocks = {'b': b[:, sl], 'f': f[:, sl], 'i': i[:, sl]}
        for kind in 'bfi':
            cols = [blocks[kind][col] for _, kk, col in fb.plan.order if kk == kind]
            M = np.stack(cols, axis=1)
            ref = g[f'k3_feat_{kind}']
            if kind == 'f':
                assert_close(M, ref, 'batched f64')
            else:
                np.testing.assert_array_equal(M.astype(ref.dtype), ref)
        np.testing.assert_array_equal(lb.scores[sl].cpu().numpy(), g['scores'])
        np.testing.assert_array_equal(lb.concedes[sl].cpu().numpy(), g['concedes'])
        np.testing.assert_array_equal(lb.goal_from_shot[sl].cpu().numpy(), g['goal_from_shot'])
        for r, c in enumerate(('offensive_value', 'defensive_value', 'vaep_value')):
            assert_close(v[r, sl], g[f'{c}_64'], c)
        o += n


def test_tiled_and_plain_layouts_agree(sa):
    """The tiled layout (R = 1024, 2048) holds exactly the plain column-major values."""
    B, ops, syn = sa['batch'], sa['ops'], sa['synthetic']
    d = syn.spadl_games(7, seed=3)
    ab = B.ActionBatch.from_columns(d)
    plain = ops.features(ab, vo.SPADL_DEFAULT, 3)
    assert plain.bool_block.shape[0] == 1
    ref = plain.to_numpy()
    for Rb, Rn in ((1024, 128), (2048, 1024), (1024, None), (None, 256)):
        tiled = ops.features(ab, vo.SPADL_DEFAULT, 3, bool_tile=Rb, num_tile=Rn)
        for a, b in zip(tiled.to_numpy(), ref):
            np.testing.assert_array_equal(a, b)
    with pytest.raises(ValueError):
        ops.features(ab, vo.SPADL_DEFAULT, 3, bool_tile=1000)
    with pytest.raises(ValueError):
        ops.features(ab, vo.SPADL_DEFAULT, 3, num_tile=100)


def _small_games(syn, atomic, seed, n_small=300):
    """Full games plus ``n_small`` games of 1..40 actions (many segment starts per tile / wave)."""
    gen = syn.atomic_games if atomic else syn.spadl_games
    d = gen(6, seed=seed)
    n0 = int(d['game_off'][-1])
    sizes = np.random.default_rng(seed + 1).integers(1, 41, n_small)
    m = int(sizes.sum())
    rows = {c: v for c, v in d.items() if isinstance(v, np.ndarray) and v.shape == (n0,)}
    d2 = {c: np.concatenate([v, v[:m]]) for c, v in rows.items()}
    offs = n0 + np.concatenate([[0], np.cumsum(sizes)])
    d2['game_off'] = np.concatenate([d['game_off'], offs[1:]])
    d2['home_team_id'] = np.concatenate([d['home_team_id'], d2['team_id'][offs[:-1]]])
    return d2


@pytest.mark.parametrize('atomic', [False, True])
def test_segment_block_table(sa, atomic):
    """sa_segment_blocks: the segment of every 128-row block start equals numpy's search of the
    offsets (one-row games, games of exactly 128 rows, a block start on a game start); and the
    kernels started from the table (features at k = 1, 3, 12, labels, the fused step) write the
    same bytes as the binary-search start (seg_of_block = NULL)."""
    B, ops, syn = sa['batch'], sa['ops'], sa['synthetic']
    from socceraction_amd import _native
    default = vo.ATOMIC_DEFAULT if atomic else vo.SPADL_DEFAULT
    d = _small_games(syn, atomic, 23)
    n0 = int(d['game_off'][-1])
    extra = np.array([128, 1, 1, 128, 256, 3, 127, 129])  # exact-block and one-row games
    rows = {c: v for c, v in d.items() if isinstance(v, np.ndarray) and v.shape == (n0,)}
    d = dict(d, **{c: np.concatenate([v, v[:extra.sum()]]) for c, v in rows.items()})
    offs = n0 + np.cumsum(extra)
    d['game_off'] = np.concatenate([d['game_off'], offs])
    d['home_team_id'] = np.concatenate([d['home_team_id'], d['team_id'][offs - extra]])
    ab = B.ActionBatch.from_columns(d, atomic=atomic)
    s = ab.struct()
    assert s.seg_of_block
    table = ab.cols['seg_of_block'].cpu().numpy()
    starts = np.arange(len(table)) * _native.SA_SEG_BLOCK
    np.testing.assert_array_equal(table, np.searchsorted(d['game_off'], starts, 'right') - 1)
    s0 = ab.struct()
    s0.seg_of_block = None
    for k in (1, 3, 12):
        plan = sa['catalog'].build_plan(default, k, atomic)
        got = [ops.alloc_feature_blocks(plan, ab.n, ab.device, 1024, 128) for _ in range(2)]
        labs = [ops.labels(ab) for _ in range(2)]
        for st, out, lab in zip((s, s0), got, labs):
            for t in (out.bool_block, out.f64_block, out.i64_block, lab.scores, lab.concedes):
                t.zero_()
            ops.step_into(st, out, None, None, 10, lab, None)
        for a, b in zip(got[0].__dict__.values(), got[1].__dict__.values()):
            if isinstance(a, torch.Tensor):
                assert torch.equal(a, b), k
        assert torch.equal(labs[0].scores, labs[1].scores) and torch.equal(labs[0].concedes, labs[1].concedes)


@pytest.mark.parametrize('atomic', [False, True])
def test_many_small_segments_vs_oracle(sa, atomic):
    """Full games + 300 games of 1..40 actions in one batch: features at k = 1, 3, 5 (both
    layouts), labels at nr_actions 10 and 20 (the > 17 path reloads rows) and the formula with
    f64 and f32 probabilities == the oracle with the same segment offsets."""
    B, ops, syn = sa['batch'], sa['ops'], sa['synthetic']
    default = vo.ATOMIC_DEFAULT if atomic else vo.SPADL_DEFAULT
    d = _small_games(syn, atomic, 11)
    ab = B.ActionBatch.from_columns(d, atomic=atomic)
    assert ab.n_segments > 300
    n, so = ab.n, d['game_off']
    names = (('period_id', 'time_seconds', 'team_id', 'x', 'y', 'dx', 'dy', 'type_id',
              'bodypart_id') if atomic else
             ('period_id', 'time_seconds', 'team_id', 'start_x', 'start_y', 'end_x', 'end_y',
              'type_id', 'result_id', 'bodypart_id'))
    cols = {c: d[c] for c in names}
    for k in (1, 3, 5):
        ref = vo.features(cols, k, default, atomic=atomic, seg_off=so, home=d['home_team_id'])
        for Rb, Rn in ((1024, 128), (None, None)):
            fb = ops.features(ab, default, k, bool_tile=Rb, num_tile=Rn)
            assert fb.plan.names == [c[0] for c in ref]
            blocks = {kk: fb.block(kk)[:, :n].cpu().numpy() for kk in 'bfi'}
            for (name, kind, col), (_, _, rv) in zip(fb.plan.order, ref):
                got = blocks[kind][col]
                if kind == 'f':
                    assert_close(got, rv, f'{name} k={k}')
                else:
                    np.testing.assert_array_equal(got.astype(np.int64), rv.astype(np.int64),
                                                  err_msg=f'{name} k={k} {Rb}')
    for nr in (10, 20):
        lb = ops.labels(ab, nr_actions=nr)
        lab = vo.labels(cols, atomic=atomic, nr_actions=nr, seg_off=so)
        for c in ('scores', 'concedes', 'goal_from_shot'):
            np.testing.assert_array_equal(getattr(lb, c)[:n].cpu().numpy().astype(bool), lab[c],
                                          err_msg=f'{c} nr={nr}')
    rng = np.random.default_rng(4)
    for dt in (np.float64, np.float32):
        ps, pc = rng.random(n).astype(dt), rng.random(n).astype(dt)
        tps, tpc = torch.from_numpy(ps).to(ab.device), torch.from_numpy(pc).to(ab.device)
        v = ops.formula(ab, tps, tpc).cpu().numpy()[:, :n]
        for nr in (10, 20):  # the fused labels + formula launch == the two separate ones
            lf, vf = ops.labels_formula(ab, tps, tpc, nr_actions=nr)
            lb = ops.labels(ab, nr_actions=nr)
            for c in ('scores', 'concedes', 'goal_from_shot'):
                assert torch.equal(getattr(lf, c)[:n], getattr(lb, c)[:n]), (c, nr, dt)
            np.testing.assert_array_equal(vf.cpu().numpy()[:, :n], v)
        fo = vo.formula(cols, ps, pc, atomic=atomic, seg_off=so)
        for r, c in enumerate(('offensive_value', 'defensive_value', 'vaep_value')):
            if dt == np.float32:  # bit-exact (the reference's f32 operations in its order)
                np.testing.assert_array_equal(v[r], fo[c], err_msg=c)
            else:
                assert_close(v[r], fo[c], c)


def test_explicit_frames_match_windowed(sa):
    """Explicit-frame mode (module-level transformers) == windowed mode on the same states."""
    B, ops = sa['batch'], sa['ops']
    g = load('spadl', 'full0')
    df = frame(g)
    n = len(df)
    k = 3
    home = g['home_team_id'][0]
    cols = inputs(g)
    # build the k game-state frames like gamestates + play_left_to_right on the host
    frames = []
    away = cols['team_id'] != home
    for i in range(k):
        rows = np.maximum(np.arange(n) - i, 0)
        d = df.iloc[rows].reset_index(drop=True).copy()
        for c, ext in (('start_x', 105.0), ('end_x', 105.0), ('start_y', 68.0), ('end_y', 68.0)):
            d.loc[away, c] = ext - d.loc[away, c].to_numpy()
        frames.append(d)
    fbs = B.frames_batches(frames, atomic=False)
    fb = ops.features_explicit(fbs, vo.SPADL_DEFAULT)
    _blocks_match(fb, g, k, n)


def _same_rate(got, ref):
    """Two rate vectors bit for bit: the same NaN rows, equal values elsewhere."""
    a, b = got.cpu().numpy(), ref.cpu().numpy()
    np.testing.assert_array_equal(np.isnan(a), np.isnan(b))
    np.testing.assert_array_equal(a[~np.isnan(b)], b[~np.isnan(b)])


def test_xt_rate_interp_equals_grid_gather(sa):
    """sa_xt_rate_interp (node values evaluated per action from the surface) == the 1050 x 680
    grid + gather, bit for bit, on random surfaces at 105 x 68, 16 x 12 and 2 x 2 (a row of
    nodes clamped at each edge), with exact-edge and NaN / inf coordinates (error bit 4)."""
    B, ops, syn = sa['batch'], sa['ops'], sa['synthetic']
    d = syn.spadl_games(40, game_id0=3)
    n = len(d['type_id'])
    rng = np.random.default_rng(8)
    for col, v in (('start_x', 0.0), ('end_x', 105.0), ('start_y', 68.0), ('end_y', 0.0),
                   ('start_x', 104.99999999999999), ('end_y', 34.0)):
        d[col][rng.choice(n, 50, replace=False)] = v
    ab = B.ActionBatch.from_columns(d)
    for l, w in ((105, 68), (16, 12), (2, 2)):
        xT = torch.rand((w, l), dtype=torch.float64, device=ab.device)
        r, e = ops.xt_rate(ab, ops.xt_interp_grid(xT, l, w), 1050, 680)
        ri, ei = ops.xt_rate_interp(ab, xT, l, w)
        _same_rate(ri, r)
        assert int(ei.item()) == int(e.item()) == 0
    for col, v in (('start_x', np.nan), ('end_y', np.inf)):
        d[col][rng.choice(n, 9, replace=False)] = v
    ab = B.ActionBatch.from_columns(d)
    xT = torch.rand((68, 105), dtype=torch.float64, device=ab.device)
    r, e = ops.xt_rate(ab, ops.xt_interp_grid(xT, 105, 68), 1050, 680)
    ri, ei = ops.xt_rate_interp(ab, xT, 105, 68)
    _same_rate(ri, r)
    assert int(ei.item()) == int(e.item()) == 4


def test_xt_goldens(sa):
    B, ops = sa['batch'], sa['ops']
    for name in cases('xt'):
        g = load('xt', name)
        df = frame(g)
        ab = B.ActionBatch.from_frame(df)
        grids = sorted({k.split('_')[0] for k in g if k[0].isdigit()})
        for tag in grids:
            l, w = map(int, tag.split('x'))
            acc = ops.xt_count(ab, l, w)
            ops.xt_check_errors(acc)
            sol = ops.xt_solve(acc)
            C = l * w
            m = sol.mats.cpu().numpy()
            np.testing.assert_array_equal(m[0].reshape(w, l), g[f'{tag}_scoring_prob'])
            np.testing.assert_array_equal(m[1].reshape(w, l), g[f'{tag}_shot_prob'])
            np.testing.assert_array_equal(m[2].reshape(w, l), g[f'{tag}_move_prob'])
            np.testing.assert_array_equal(sol.trans_t.cpu().numpy().T, g[f'{tag}_transition'])
            assert sol.n_iter + 1 == len(g[f'{tag}_heatmaps']), (name, tag)
            np.testing.assert_array_equal(m[3].reshape(w, l), g[f'{tag}_xT'])
            np.testing.assert_array_equal(sol.heatmaps.cpu().numpy().reshape(-1, w, l),
                                          g[f'{tag}_heatmaps'])
            xT = sol.mats[3].reshape(w, l)
            r, err = ops.xt_rate(ab, xT, l, w)
            assert int(err.item()) == 0
            assert_close(r.cpu().numpy(), g[f'{tag}_rate'], f'{name} {tag} rate')
            if f'{tag}_rate_interp' in g:
                grid = ops.xt_interp_grid(xT, l, w)
                assert_close(grid.cpu().numpy(), xo.interp_grid(g[f'{tag}_xT']), 'interp grid')
                r, _ = ops.xt_rate(ab, grid, 1050, 680)
                assert_close(r.cpu().numpy(), g[f'{tag}_rate_interp'], f'{name} {tag} interp rate')
                ri, ei = ops.xt_rate_interp(ab, xT, l, w)  # per-action nodes, no grid: same bits
                _same_rate(ri, r)
                assert int(ei.item()) == 0


def test_xt105_interpolated_rate_golden(sa):
    """cfg5's ExpectedThreat(105, 68).rate(use_interpolation=True) == the reference's own output
    (tests/golden/make_golden_xt105.py): the 1050 x 680 surface (strided sample) and the rating
    of every action, through ops and through the drop-in ExpectedThreat."""
    import os

    from golden_io import GOLDEN
    from socceraction_amd import xthreat
    B, ops = sa['batch'], sa['ops']
    with np.load(os.path.join(GOLDEN, 'xt105_interp.npz'), allow_pickle=False) as z:
        g = {k: z[k] for k in z.files}
    df = frame(g)
    ab = B.ActionBatch.from_frame(df)
    rows, cols = g['grid_rows'], g['grid_cols']
    for tag in ('fit', 'random'):
        xT = torch.tensor(g[f'{tag}_xT'], device=ab.device)
        grid = ops.xt_interp_grid(xT, 105, 68)
        assert tuple(grid.shape) == (680, 1050)
        assert_close(grid.cpu().numpy()[np.ix_(rows, cols)], g[f'{tag}_grid_sample'], f'{tag} grid')
        r, err = ops.xt_rate(ab, grid, 1050, 680)
        assert int(err.item()) == 0
        assert_close(r.cpu().numpy(), g[f'{tag}_rate_interp'], f'{tag} interp rate')
        ri, ei = ops.xt_rate_interp(ab, xT, 105, 68)  # per-action nodes, no grid: same bits
        _same_rate(ri, r)
        assert int(ei.item()) == 0
        m = xthreat.ExpectedThreat(l=105, w=68)
        m.xT = g[f'{tag}_xT'].copy()
        assert_close(m.rate(df, use_interpolation=True), g[f'{tag}_rate_interp'], f'{tag} drop-in')
        assert_close(m.rate(df), g[f'{tag}_rate'], f'{tag} drop-in cells')


@pytest.mark.parametrize('l,w,games', [(16, 12, 2000), (40, 30, 300), (105, 68, 300)])
def test_xt_large_grid_vs_oracle(sa, l, w, games):
    """16 x 12 over ~3.2M actions: the one-workgroup-per-CU count pass (XC_WIDE, every CU's
    chunk flushed into the same bins). Grids above the single-workgroup solver (C > 1024) take
    the streaming count-row iteration. Iterates, iteration count and matrices must be
    bit-identical to the oracle."""
    B, ops, syn = sa['batch'], sa['ops'], sa['synthetic']
    d = syn.spadl_games(games, game_id0=77)
    ab = B.ActionBatch.from_columns(d)
    acc = ops.xt_count(ab, l, w)
    ops.xt_check_errors(acc)
    sol = ops.xt_solve(acc, exact_order=True)  # the reference's summation order: bit-exact
    ref = xo.fit(d, l, w)
    m = sol.mats.cpu().numpy()
    np.testing.assert_array_equal(m[0].reshape(w, l), ref['scoring_prob'])
    np.testing.assert_array_equal(m[1].reshape(w, l), ref['shot_prob'])
    np.testing.assert_array_equal(m[2].reshape(w, l), ref['move_prob'])
    np.testing.assert_array_equal(sol.trans_t.cpu().numpy().T, ref['transition'])
    assert sol.n_iter + 1 == len(ref['heatmaps'])
    np.testing.assert_array_equal(sol.heatmaps.cpu().numpy().reshape(-1, w, l), ref['heatmaps'])
    np.testing.assert_array_equal(m[3].reshape(w, l), ref['xT'])
    if l * w > 1024:
        # the large-grid solve without the dense transposed matrix: same results, and the
        # drop-in's transition_matrix (formed on first access) equals the oracle's
        lean = ops.xt_solve(acc, transition=False, exact_order=True)
        assert lean.trans_t is None and lean.n_iter == sol.n_iter
        np.testing.assert_array_equal(lean.mats.cpu().numpy(), m)
        np.testing.assert_array_equal(lean.heatmaps.cpu().numpy(), sol.heatmaps.cpu().numpy())
        # the default reordered sums: the same iteration count, iterates within 1e-12 relative
        fast = ops.xt_solve(acc, transition=False)
        assert fast.path == 'reordered' and fast.n_iter == sol.n_iter
        np.testing.assert_array_equal(fast.mats[:3].cpu().numpy(), m[:3])
        h, r = fast.heatmaps.cpu().numpy(), sol.heatmaps.cpu().numpy()
        assert np.all(np.abs(h - r) <= 1e-12 * np.abs(r))
        from socceraction_amd import xthreat
        model = xthreat.ExpectedThreat(l=l, w=w).fit(syn.to_frame(d), exact_order=True)
        assert model._transition is None and model.solve_path == 'sequential'
        np.testing.assert_array_equal(model.xT, ref['xT'])
        np.testing.assert_array_equal(model.transition_matrix, ref['transition'])
        assert model._transition_counts is None
        model = xthreat.ExpectedThreat(l=l, w=w).fit(syn.to_frame(d))
        assert model.solve_path == 'reordered' and len(model.heatmaps) == len(ref['heatmaps'])
        assert np.all(np.abs(model.xT - ref['xT']) <= 1e-12 * np.abs(ref['xT']))


@pytest.mark.parametrize('l,w,games', [(16, 12, 400), (105, 68, 60), (1, 1, 5), (30, 20, 1)])
def test_xt_rate_codes_match_rate(sa, l, w, games):
    """fit + rate of one frame through the count pass's rate codes == the coordinate path:
    counts, error bits, values and NaN pattern bit for bit, incl. NaN / inf coordinates on
    successful moves, failed moves and shots, and a tail shorter than 4 actions."""
    B, ops, syn = sa['batch'], sa['ops'], sa['synthetic']
    d = syn.spadl_games(games, game_id0=5)
    n = len(d['type_id'])
    d = {k: (v[:n - 3].copy() if isinstance(v, np.ndarray) and v.shape == (n,) else v)
         for k, v in d.items()}
    d['game_off'] = np.minimum(d['game_off'], n - 3)
    rng = np.random.default_rng(9)
    for col, val in (('start_x', np.nan), ('end_y', np.inf), ('start_y', -np.inf),
                     ('end_x', np.nan)):
        d[col][rng.choice(n - 3, 7, replace=False)] = val
    ab = B.ActionBatch.from_columns(d)
    ref_acc = ops.xt_count(ab, l, w)
    codes = ops.xt_rate_codes_buffer(ab.n, ab.device)
    acc = ops.xt_count(ab, l, w, codes=codes)
    shared = ops.xt_count(ab, l, w, shared=True)  # co-resident workgroup shape, same counts
    for got_acc in (acc, shared):
        for a, b in ((got_acc.shot, ref_acc.shot), (got_acc.goal, ref_acc.goal),
                     (got_acc.move, ref_acc.move), (got_acc.trans, ref_acc.trans),
                     (got_acc.err, ref_acc.err)):
            assert torch.equal(a, b)
    grid = torch.rand((w, l), dtype=torch.float64, device=ab.device)
    ref, ref_err = ops.xt_rate(ab, grid, l, w)
    got, err = ops.xt_rate_codes(codes, ab.n, grid)
    r, g = ref.cpu().numpy(), got.cpu().numpy()
    np.testing.assert_array_equal(np.isnan(g), np.isnan(r))
    np.testing.assert_array_equal(g[~np.isnan(r)], r[~np.isnan(r)])
    assert int(err.item()) == int(ref_err.item()) == 4
    assert (~np.isnan(r)).sum() > 0


def test_full_size_sampled_games_vs_oracle(sa):
    """cfg2-sized batch (10k games, ~16M actions): sampled games checked against the oracle,
    plus size-independent invariants over the whole batch (one-hot rows sum to 1)."""
    B, ops, syn = sa['batch'], sa['ops'], sa['synthetic']
    d = syn.spadl_games(10000)
    ab = B.ActionBatch.from_columns(d)
    fb = ops.features(ab, vo.SPADL_DEFAULT, 3, bool_tile=1024, num_tile=128)
    lb = ops.labels(ab)
    p = syn.probabilities(ab.n)
    ps = torch.from_numpy(p['scores']).to(ab.device)
    pc = torch.from_numpy(p['concedes']).to(ab.device)
    val = ops.formula(ab, ps, pc)
    torch.cuda.synchronize()
    n = ab.n
    # invariant: each window's type x result one-hot has exactly one True per action
    plan = fb.plan
    tr = [col for name, kind, col in plan.order if name.startswith('type_') and '_result_' in name]
    assert len(tr) == 414
    for i in range(3):
        s = fb.bool_block[:, tr[i * 138]:tr[i * 138] + 138, :].sum(dim=1, dtype=torch.int32)
        s = s.reshape(-1)[:n]
        assert bool((s == 1).all())
    rng = np.random.default_rng(0)
    off = d['game_off']
    names = plan.names
    for g in rng.choice(len(off) - 1, 12, replace=False):
        s, e = int(off[g]), int(off[g + 1])
        cols = {c: d[c][s:e] for c in ('period_id', 'time_seconds', 'team_id', 'start_x',
                                       'start_y', 'end_x', 'end_y', 'type_id', 'result_id',
                                       'bodypart_id')}
        ref = vo.features(cols, 3, vo.SPADL_DEFAULT, home=[d['home_team_id'][g]])
        assert [c[0] for c in ref] == names
        blocks = {k: fb.block(k)[:, s:e].cpu().numpy() for k in 'bfi'}
        for (name, kind, col), (_, _, rv) in zip(plan.order, ref):
            got = blocks[kind][col]
            if kind == 'f':
                assert_close(got, rv, name)
            else:
                np.testing.assert_array_equal(got.astype(np.int64), rv.astype(np.int64), err_msg=name)
        lab = vo.labels(cols)
        np.testing.assert_array_equal(lb.scores[s:e].cpu().numpy().astype(bool), lab['scores'])
        np.testing.assert_array_equal(lb.concedes[s:e].cpu().numpy().astype(bool), lab['concedes'])
        fo = vo.formula(cols, p['scores'][s:e], p['concedes'][s:e])
        for r, c in enumerate(('offensive_value', 'defensive_value', 'vaep_value')):
            assert_close(val[r, s:e].cpu().numpy(), fo[c], c)


@pytest.mark.parametrize('l,w,games', [(16, 12, 300), (30, 20, 60), (64, 64, 40), (1, 1, 5)])
def test_xt_cell_codes_match_coordinate_path(sa, l, w, games):
    """The xT cell codes -- written by the VAEP feature pass (sa_vaep_features_xt, both the k <= 3
    register-window path and the generic path) or alone (sa_xt_cells) -- give the coordinate
    path's counts, error bits, rate values and NaN pattern bit for bit, incl. NaN / inf
    coordinates on successful moves, failed moves and shots, and an odd-length tail."""
    B, ops, syn = sa['batch'], sa['ops'], sa['synthetic']
    d = syn.spadl_games(games, game_id0=9)
    n = len(d['type_id'])
    d = {k: (v[:n - 3].copy() if isinstance(v, np.ndarray) and v.shape == (n,) else v)
         for k, v in d.items()}
    d['game_off'] = np.minimum(d['game_off'], n - 3)
    rng = np.random.default_rng(2)
    for col, val in (('start_x', np.nan), ('end_y', np.inf), ('start_y', -np.inf),
                     ('end_x', np.nan)):
        d[col][rng.choice(n - 3, 9, replace=False)] = val
    ab = B.ActionBatch.from_columns(d)
    cells = ops.xt_cells(ab, l, w)
    for k in (3, 5):
        fb = ops.alloc_feature_blocks(sa['catalog'].build_plan(vo.SPADL_DEFAULT, k), ab.n,
                                      ab.device, 1024, 128)
        c2 = ops.xt_cells_buffer(ab.n, ab.device)
        ops.features_into(ab.struct(), fb, xt_cells=(l, w, c2))
        assert torch.equal(ops.xt_cell_codes(c2, ab.n, l, w), ops.xt_cell_codes(cells, ab.n, l, w)), k
    ref = ops.xt_count(ab, l, w)
    for shared in (False, True):
        acc = ops.xt_count_cells(cells, ab.n, l, w, shared=shared)
        for a, b in ((acc.shot, ref.shot), (acc.goal, ref.goal), (acc.move, ref.move),
                     (acc.trans, ref.trans), (acc.err, ref.err)):
            assert torch.equal(a, b), shared
    assert int(ref.err.item()) != 0
    grid = torch.rand((w, l), dtype=torch.float64, device=ab.device)
    r_ref, e_ref = ops.xt_rate(ab, grid, l, w)
    r, e = ops.xt_rate_cells(cells, ab.n, l, w, grid)
    rr, gg = r_ref.cpu().numpy(), r.cpu().numpy()
    np.testing.assert_array_equal(np.isnan(gg), np.isnan(rr))
    np.testing.assert_array_equal(gg[~np.isnan(rr)], rr[~np.isnan(rr)])
    assert int(e.item()) == int(e_ref.item()) == 4
    with pytest.raises(ValueError):
        ops.xt_cells(ab, 105, 68)  # 7140 cells do not fit the 12-bit fields


def test_atomic_cfg3_slice_sampled_games_vs_oracle(sa):
    """cfg3's per-GPU slice (1,250 synthetic atomic games, ~5M atomic actions -- 40M over 8
    GPUs): Atomic-VAEP features (k=3, default xfns, 154 columns) + labels of the whole batch,
    12 sampled games checked against the oracle column by column, plus the whole-batch
    invariant that every window's atomic type one-hot has exactly one True per action (the
    duplicate 'interception' column is true for ids 10 and 24)."""
    B, ops, syn = sa['batch'], sa['ops'], sa['synthetic']
    d = syn.atomic_games(1250)
    ab = B.ActionBatch.from_columns(d, atomic=True)
    assert ab.n > 4_000_000
    fb = ops.features(ab, vo.ATOMIC_DEFAULT, 3, bool_tile=1024, num_tile=128)
    lb = ops.labels(ab)
    torch.cuda.synchronize()
    plan = fb.plan
    tcols = [col for name, kind, col in plan.order if kind == 'b' and name.startswith('type_')]
    assert len(tcols) == 3 * 32
    for i in range(3):
        s = fb.bool_block[:, tcols[i * 32]:tcols[i * 32] + 32, :].sum(dim=1, dtype=torch.int32)
        assert bool((s.reshape(-1)[:ab.n] == 1).all())
    rng = np.random.default_rng(1)
    off = d['game_off']
    names = ('period_id', 'time_seconds', 'team_id', 'x', 'y', 'dx', 'dy', 'type_id', 'bodypart_id')
    for g in rng.choice(len(off) - 1, 12, replace=False):
        s, e = int(off[g]), int(off[g + 1])
        cols = {c: d[c][s:e] for c in names}
        ref = vo.features(cols, 3, vo.ATOMIC_DEFAULT, atomic=True, home=[d['home_team_id'][g]])
        assert [c[0] for c in ref] == plan.names
        blocks = {k: fb.block(k)[:, s:e].cpu().numpy() for k in 'bfi'}
        for (name, kind, col), (_, _, rv) in zip(plan.order, ref):
            got = blocks[kind][col]
            if kind == 'f':
                assert_close(got, rv, name)
            else:
                np.testing.assert_array_equal(got.astype(np.int64), rv.astype(np.int64), err_msg=name)
        lab = vo.labels(cols, atomic=True)
        for c in ('scores', 'concedes', 'goal_from_shot'):
            np.testing.assert_array_equal(getattr(lb, c)[s:e].cpu().numpy().astype(bool), lab[c])


@pytest.mark.parametrize('atomic', [False, True])
def test_fused_goalscore_matches_scan(sa, atomic):
    """The goalscore columns the numeric feature pass computes in windowed mode (a wave's carry
    counted from its segment's start + ballot counts inside the wave) == the standalone
    one-wave-per-segment scan (``sa_vaep_goalscore``), bit for bit: on a goal-dense batch
    (every 7th action a goal / owngoal credit) of full games + 300 games of 1..40 actions at
    k = 1, 3, 5, and on 2,000 full-size games, where the carries span whole games."""
    B, ops, syn = sa['batch'], sa['ops'], sa['synthetic']
    default = vo.ATOMIC_DEFAULT if atomic else vo.SPADL_DEFAULT
    dense = _small_games(syn, atomic, 17)
    n = int(dense['game_off'][-1])
    rng = np.random.default_rng(5)
    hit = rng.random(n) < 1 / 7
    if atomic:
        dense['type_id'] = np.where(hit, rng.choice([27, 28], n), dense['type_id'])
    else:
        dense['type_id'] = np.where(hit, rng.choice([11, 12, 13], n), dense['type_id'])
        dense['result_id'] = np.where(hit, rng.choice([0, 1, 3], n), dense['result_id'])
    gen = syn.atomic_games if atomic else syn.spadl_games
    for d, kk in ((dense, (1, 3, 5)), (gen(2000, seed=9), (3,))):
        ab = B.ActionBatch.from_columns(d, atomic=atomic)
        for k in kk:
            fb = ops.features(ab, default, k, bool_tile=1024, num_tile=128)
            fused = fb.i64_block.clone()
            fb.i64_block.fill_(-7)
            ops.goalscore_into(ab, fb)
            gc = [col for name, kind, col in fb.plan.order if name.startswith('goalscore')]
            assert len(gc) == 3
            got = fused[:, gc, :].permute(1, 0, 2).reshape(3, -1)[:, :ab.n]
            ref = fb.i64_block[:, gc, :].permute(1, 0, 2).reshape(3, -1)[:, :ab.n]
            assert torch.equal(got, ref), (atomic, k)
            assert int(ref[0].max()) > 0


@pytest.mark.parametrize('atomic', [False, True])
def test_step_matches_separate_launches(sa, atomic):
    """sa_vaep_step_f64 (labels + f64 formula computed by the numeric pass, lane = 2 rows, the
    look-ahead by wave shuffles) == sa_vaep_features (+ the xT cell codes) followed by
    sa_vaep_labels_formula_f64, byte for byte: the goldens (edge sizes 1..300, forced tail goals),
    full games + 300 games of 1..40 actions at nr_actions 1, 2, 10, 11 and 20 (the last runs the
    separate launches), k = 1..4, both layouts, and 2,000 full-size games; and the labels-only
    form (no probabilities) == features + labels."""
    B, ops, syn = sa['batch'], sa['ops'], sa['synthetic']
    default = vo.ATOMIC_DEFAULT if atomic else vo.SPADL_DEFAULT
    prefix = 'atomic' if atomic else 'spadl'
    gen = syn.atomic_games if atomic else syn.spadl_games
    batches = [B.ActionBatch.from_frame(frame(load(prefix, c), atomic), atomic=atomic,
                                        home_team_id=load(prefix, c)['home_team_id'][0])
               for c in cases(prefix)]
    dense = _small_games(syn, atomic, 23)
    hit = np.random.default_rng(3).random(len(dense['type_id'])) < 1 / 9
    if atomic:
        dense['type_id'] = np.where(hit, np.random.default_rng(4).choice([11, 27, 28], hit.size),
                                    dense['type_id'])
    else:
        dense['type_id'] = np.where(hit, 11, dense['type_id'])
        dense['result_id'] = np.where(hit, np.random.default_rng(4).choice([0, 1, 3], hit.size),
                                      dense['result_id'])
    batches += [B.ActionBatch.from_columns(dense, atomic=atomic),
                B.ActionBatch.from_columns(gen(2000, seed=31), atomic=atomic)]
    rng = np.random.default_rng(8)
    for bi, ab in enumerate(batches):
        n = ab.n
        ps = torch.from_numpy(rng.random(n)).to(ab.device)
        pc = torch.from_numpy(rng.random(n)).to(ab.device)
        small = bi == len(batches) - 2
        layouts = ((1024, 128), (None, None)) if small else ((1024, 128),)
        for Rb, Rn in layouts:
            for nr in ((1, 2, 10, 11, 20) if bi >= len(batches) - 2 else (10,)):
                for k in ((1, 2, 3, 4) if small and nr == 10 else (3,)):
                    xt = None if atomic else 16
                    cells_ref = ops.xt_cells_buffer(n, ab.device) if xt else None
                    ref = ops.alloc_feature_blocks(ops.build_plan(default, k, atomic), n, ab.device,
                                                   Rb, Rn)
                    ops.features_into(ab.struct(), ref, xt_cells=(16, 12, cells_ref) if xt else None)
                    lref, vref = ops.labels_formula(ab, ps, pc, nr_actions=nr)
                    out = ops.alloc_feature_blocks(ref.plan, n, ab.device, Rb, Rn)
                    lab, val = ops.labels_formula(ab, ps, pc, nr_actions=nr)  # right-shaped buffers
                    for t in (lab.scores, lab.concedes, lab.goal_from_shot):
                        t.fill_(7)
                    val.fill_(float('nan'))
                    cells = ops.xt_cells_buffer(n, ab.device) if xt else None
                    ops.step_into(ab.struct(), out, ps, pc, nr, lab, val,
                                  xt_cells=(16, 12, cells) if xt else None)
                    for a, b in zip(out.to_numpy(), ref.to_numpy()):
                        np.testing.assert_array_equal(a, b)
                    for c in ('scores', 'concedes', 'goal_from_shot'):
                        assert torch.equal(getattr(lab, c)[:n], getattr(lref, c)[:n]), (bi, nr, k, c)
                    assert torch.equal(val[:, :n], vref[:, :n]), (bi, nr, k)
                    if xt:
                        assert torch.equal(ops.xt_cell_codes(cells, n, 16, 12),
                                           ops.xt_cell_codes(cells_ref, n, 16, 12))
                    if k == 3:  # features + labels only (no probabilities): the cfg3 step
                        out2 = ops.alloc_feature_blocks(ref.plan, n, ab.device, Rb, Rn)
                        lab2, _ = ops.labels_formula(ab, ps, pc, nr_actions=nr)
                        for t in (lab2.scores, lab2.concedes, lab2.goal_from_shot):
                            t.fill_(7)
                        ops.step_into(ab.struct(), out2, None, None, nr, lab2, None)
                        for a, b in zip(out2.to_numpy(), ref.to_numpy()):
                            np.testing.assert_array_equal(a, b)
                        for c in ('scores', 'concedes', 'goal_from_shot'):
                            assert torch.equal(getattr(lab2, c)[:n], getattr(lref, c)[:n]), (bi, nr, c)


@pytest.mark.parametrize('l,w', [(16, 12), (8, 6), (30, 20)])
def test_xt_solve_async_matches_solve(sa, l, w):
    """sa_xt_solve_async (no host round trip; the iteration count stays on the device) == the
    synchronised sa_xt_solve: every matrix, the surface, the heatmaps and the iteration count,
    bit for bit (the register solve at 16 x 12 and 8 x 6, the one-workgroup solve at 30 x 20)."""
    B, ops, syn = sa['batch'], sa['ops'], sa['synthetic']
    ab = B.ActionBatch.from_columns(syn.spadl_games(40, seed=12))
    acc = ops.xt_count(ab, l, w)
    ref = ops.xt_solve(acc)
    got = ops.xt_solve_async(acc)
    torch.cuda.synchronize()
    n = int(got.n_iter.item())
    assert n == ref.n_iter > 0
    assert torch.equal(got.mats, ref.mats)
    assert torch.equal(got.trans_t, ref.trans_t)
    assert torch.equal(got.heatmaps[:n + 1], ref.heatmaps)


def test_contiguous_bool_block_matches(sa):
    """Feature blocks whose bool block lives in physically contiguous VRAM (sa_device_alloc,
    viewed through __cuda_array_interface__) hold the same bytes as caching-allocator blocks, and
    the allocation outlives the DeviceBuffer's last Python reference held by the blocks."""
    import gc
    B, ops, syn = sa['batch'], sa['ops'], sa['synthetic']
    ab = B.ActionBatch.from_columns(syn.spadl_games(30, seed=4))
    plan = ops.build_plan(vo.SPADL_DEFAULT, 3, False)
    ref = ops.alloc_feature_blocks(plan, ab.n, ab.device, 1024, 128)
    got = ops.alloc_feature_blocks(plan, ab.n, ab.device, 1024, 128, contiguous=True)
    assert got._arena is not None and got.bool_block.data_ptr() == got._arena.ptr
    gc.collect()
    for fb in (ref, got):
        ops.features_into(ab.struct(), fb)
    for a, b in zip(got.to_numpy(), ref.to_numpy()):
        np.testing.assert_array_equal(a, b)
    buf = ops.DeviceBuffer(1 << 20, contiguous=False)
    t = buf.tensor((256, 1024), torch.float32)
    t.fill_(2.0)
    assert float(t.sum()) == 2.0 * 256 * 1024


def test_contiguous_action_batch_matches(sa):
    """An ActionBatch whose device buffer is one physically contiguous range holds the same
    bytes, and the features and the whole 'all' block arena computed from it are equal."""
    B, ops, syn = sa['batch'], sa['ops'], sa['synthetic']
    d = syn.atomic_games(20, seed=6)
    ref = B.ActionBatch.from_columns(d, atomic=True)
    got = B.ActionBatch.from_columns(d, atomic=True, contiguous=True)
    assert got._dbuf is not None and got.buffer.data_ptr() == got._dbuf.ptr
    assert torch.equal(got.buffer, ref.buffer)
    plan = ops.build_plan(vo.ATOMIC_DEFAULT, 3, True)
    a = ops.alloc_feature_blocks(plan, ref.n, ref.device, 1024, 128)
    b = ops.alloc_feature_blocks(plan, got.n, got.device, 1024, 128, contiguous='all')
    assert b.bool_alloc in ('contiguous-all', 'caching')
    ops.features_into(ref.struct(), a)
    ops.features_into(got.struct(), b)
    for x, y in zip(a.to_numpy(), b.to_numpy()):
        np.testing.assert_array_equal(x, y)


def test_chunked_step_equals_step(sa):
    """sa_vaep_step_f64_chunked (the numeric step pass in launches of whole 512-row blocks, each
    optionally after a pure-read pass over its inputs; bench.py's --ab probe of the pass's read /
    write turnaround) == sa_vaep_step_f64 byte for byte: f64 / i64 blocks, xT cell codes, labels
    and formula, with a chunk that does not divide n."""
    import copy
    B, ops, syn = sa['batch'], sa['ops'], sa['synthetic']
    ab = B.ActionBatch.from_columns(syn.spadl_games(700, seed=41))
    n = ab.n
    rng = np.random.default_rng(9)
    ps = torch.from_numpy(rng.random(n)).to(ab.device)
    pc = torch.from_numpy(rng.random(n)).to(ab.device)
    plan = ops.build_plan(vo.SPADL_DEFAULT, 3, False)
    num = copy.copy(plan)
    num.struct = copy.deepcopy(plan.struct)
    for x in range(len(num.struct.bool_col)):
        num.struct.bool_col[x] = -1
    outs = []
    for chunk, pf in ((0, False), (131072, False), (131072, True), (512 * 997, True)):
        blk = ops.alloc_feature_blocks(plan, n, ab.device, 1024, 128)
        view = ops.FeatureBlocks(num, n, blk.Rb, blk.Rn, blk.bool_block, blk.f64_block, blk.i64_block)
        blk.f64_block.fill_(float('nan'))
        blk.i64_block.fill_(-7)
        lab, val = ops.labels_formula(ab, ps, pc, nr_actions=10)
        for t in (lab.scores, lab.concedes, lab.goal_from_shot):
            t.fill_(7)
        val.fill_(float('nan'))
        cells = ops.xt_cells_buffer(n, ab.device)
        ops.step_into(ab.struct(), view, ps, pc, 10, lab, val, xt_cells=(16, 12, cells), chunk_rows=chunk,
                      prefetch=pf)
        outs.append((blk.f64_block.clone(), blk.i64_block.clone(), ops.xt_cell_codes(cells, n, 16, 12).clone(),
                     [getattr(lab, c)[:n].clone() for c in ('scores', 'concedes', 'goal_from_shot')],
                     val[:, :n].clone()))
    f0, i0, c0, l0, v0 = outs[0]
    for f, i, c, l, v in outs[1:]:
        assert torch.equal(f.view(torch.int64), f0.view(torch.int64)) and torch.equal(i, i0)
        assert torch.equal(c, c0) and torch.equal(v.view(torch.int64), v0.view(torch.int64))
        assert all(torch.equal(a, b) for a, b in zip(l, l0))
