"""GPU parity of the large-grid xT fit (sa_xt_large.hip): the band-owned count (no global
atomics) against the oracle's counts, and the compact-form value iteration against the dense
count-row iteration (sa_xt_iterate_rows), bit for bit.  Reference: xthreat.py:40-67, 177-218
(counts), 278-320 (value iteration)."""
import numpy as np
import pytest

from oracle import xt_oracle as xo

pytestmark = pytest.mark.gpu

torch = pytest.importorskip('torch')


@pytest.fixture(scope='module')
def sa():
    from socceraction_amd import _native, batch, ops, synthetic
    _native.load_library()
    return dict(_native=_native, batch=batch, ops=ops, synthetic=synthetic)


def _oracle(d, l, w):
    return xo.counts({c: d[c] for c in ('start_x', 'start_y', 'end_x', 'end_y', 'type_id',
                                         'result_id')}, l, w)


def _same_counts(acc, ref, l, w):
    C = l * w
    np.testing.assert_array_equal(acc.shot.cpu().numpy(), ref['shot'].reshape(-1))
    np.testing.assert_array_equal(acc.goal.cpu().numpy(), ref['goal'].reshape(-1))
    np.testing.assert_array_equal(acc.move.cpu().numpy(), ref['move'].reshape(-1))
    np.testing.assert_array_equal(acc.trans.cpu().numpy().reshape(C, C), ref['trans'])


def _cat(parts):
    out = {}
    for k, v in parts[0].items():
        if isinstance(v, np.ndarray) and k not in ('game_off', 'home_team_id'):
            out[k] = np.concatenate([p[k] for p in parts])
    return out


@pytest.mark.parametrize('l,w', [(105, 68), (40, 30), (15, 14), (100, 68), (75, 68), (120, 68)])
def test_band_count_many_batches_vs_oracle(sa, l, w):
    """xt_count_many over three device batches (fresh accumulator: the band count writes the
    table once, never reading it) == the oracle's counts of all their actions; the same batches
    added into an accumulator that already holds counts (one xt_count first) == the sum."""
    B, ops, syn = sa['batch'], sa['ops'], sa['synthetic']
    assert ops.xt_band_shape(l, w) is not None
    ds = [syn.spadl_games(g, game_id0=100 * i + 7) for i, g in enumerate((40, 55, 23))]
    abs_ = [B.ActionBatch.from_columns(d) for d in ds]
    acc = ops.xt_count_many(abs_, l, w)
    ops.xt_check_errors(acc)
    _same_counts(acc, _oracle(_cat(ds), l, w), l, w)
    acc2 = ops.xt_count(abs_[0], l, w)
    ops.xt_count_many(abs_[1:], l, w, acc2)  # accumulate (read-modify-write of the rows)
    _same_counts(acc2, _oracle(_cat(ds), l, w), l, w)


def _xe_slots(k):
    return (k & ~127) | ((k & 31) << 2) | ((k >> 5) & 3)


@pytest.mark.parametrize('l,w,hot', [(105, 68, False), (40, 30, False), (120, 68, False),
                                     (105, 68, True)])
def test_band_count_emits_compact_rows(sa, l, w, hot):
    """The band count's compact rows (sa_xt_count_from_buckets_ex, written from the bins) ==
    sa_xt_compact_rows of the dense table it wrote, entry for entry (incl. escaped counts >=
    65535), and the solve from them == the solve that builds its own (same path, iteration
    count and heatmaps bit for bit); an all-reduce or a further count drops them."""
    B, ops, syn, N = sa['batch'], sa['ops'], sa['synthetic'], sa['_native']
    C = l * w
    ds = [syn.spadl_games(g, game_id0=31 * i + 5) for i, g in enumerate((150 if hot else 60, 45))]
    if hot:
        mv = np.isin(ds[0]['type_id'], (0, 1, 21))
        ds[0]['start_x'][mv], ds[0]['start_y'][mv] = 52.2, 33.3
        ds[0]['end_x'][mv], ds[0]['end_y'][mv] = 104.999, 0.0
    abs_ = [B.ActionBatch.from_columns(d) for d in ds]
    acc = ops.xt_count_many(abs_, l, w)
    assert acc.compact is not None
    ell, rl = acc.compact
    pe = int(N.lib().sa_xt_compact_bytes(C, 1)) // 4
    ref_ell = torch.empty(C * pe, dtype=torch.int32, device=ell.device)
    ref_rl = torch.empty(C, dtype=torch.int32, device=ell.device)
    N.check(N.lib().sa_xt_compact_rows(acc.trans.data_ptr(), C, C, ref_ell.data_ptr(),
                                       ref_rl.data_ptr(), torch.cuda.current_stream().cuda_stream))
    a, b = rl.cpu().numpy(), ref_rl.cpu().numpy()
    np.testing.assert_array_equal(a, b)
    ea, eb = ell.cpu().numpy().reshape(C, pe), ref_ell.cpu().numpy().reshape(C, pe)
    for r in np.flatnonzero(a):
        sl = _xe_slots(np.arange(a[r]))
        np.testing.assert_array_equal(ea[r, sl], eb[r, sl])
    if hot:
        assert (ea.view(np.uint32) >> 16 == 0xFFFF).any()
    sol = ops.xt_solve(acc, transition=False)
    acc.compact = None
    ref = ops.xt_solve(acc, transition=False)
    assert sol.path == ref.path and sol.n_iter == ref.n_iter
    assert torch.equal(sol.heatmaps, ref.heatmaps) and torch.equal(sol.mats, ref.mats)
    acc2 = ops.xt_count_many(abs_, l, w)
    ops.xt_count(abs_[0], l, w, acc2)
    assert acc2.compact is None


def test_band_count_hot_cells_and_edges(sa):
    """Adversarial key distributions: every move between two cells (one bin far above 65535
    counts, one band holding almost every key), actions on the exact pitch edges, NaN / inf
    coordinates (error bytes as sa_xt_count's coordinate path) and a batch shorter than one
    workgroup's chunk."""
    B, ops, syn = sa['batch'], sa['ops'], sa['synthetic']
    l, w = 105, 68
    d = syn.spadl_games(80, game_id0=11)
    n = len(d['type_id'])
    mv = np.isin(d['type_id'], (0, 1, 21))
    d['start_x'][mv], d['start_y'][mv] = 52.2, 33.3
    d['end_x'][mv], d['end_y'][mv] = 104.999, 0.0
    ab = B.ActionBatch.from_columns(d)
    acc = ops.xt_count(ab, l, w)
    ops.xt_check_errors(acc)
    ref = _oracle(d, l, w)
    assert ref['trans'].max() > 65535
    _same_counts(acc, ref, l, w)
    rng = np.random.default_rng(4)
    e = syn.spadl_games(3, game_id0=19)
    m = len(e['type_id'])
    for col, v in (('start_x', 0.0), ('end_x', 105.0), ('start_y', 68.0), ('end_y', 0.0)):
        e[col][rng.choice(m, 40, replace=False)] = v
    ab = B.ActionBatch.from_columns(e)
    _same_counts(ops.xt_count_many([ab], l, w), _oracle(e, l, w), l, w)
    for col, v, bit in (('start_x', np.nan, 0x10000), ('end_y', np.inf, 0x10000)):
        f = {k: (v2.copy() if isinstance(v2, np.ndarray) else v2) for k, v2 in e.items()}
        f[col][np.flatnonzero(np.isin(f['type_id'], (0, 1, 21)))[:5]] = v
        ab = B.ActionBatch.from_columns(f)
        got = ops.xt_count_many([ab], l, w)
        old = ops.xt_count(ab, l, w)  # the one-batch entry point: the same band path
        assert int(got.err.item()) & bit and int(got.err.item()) == int(old.err.item())
        for a, b in ((got.shot, old.shot), (got.goal, old.goal), (got.move, old.move),
                     (got.trans, old.trans)):
            assert torch.equal(a, b)
    # a shot with an infinite start: byte 0x1
    f = {k: (v2.copy() if isinstance(v2, np.ndarray) else v2) for k, v2 in e.items()}
    f['start_x'][np.flatnonzero(f['type_id'] == 11)[:2]] = -np.inf
    got = ops.xt_count_many([B.ActionBatch.from_columns(f)], l, w)
    assert int(got.err.item()) & 0xFF


def _random_rows(rng, C, nrows, zero_rows=3):
    """Count rows shaped like a fit's: ~40 % non-zero, mostly small counts, some >= 64 (the
    division path), a few >= 65535 (the escape to the dense row), some empty rows."""
    cnt = np.zeros((nrows, C), np.int32)
    nz = rng.random((nrows, C)) < 0.4
    cnt[nz] = rng.geometric(0.3, nz.sum())
    big = rng.random((nrows, C)) < 0.002
    cnt[big] = rng.integers(64, 5000, big.sum())
    cnt[rng.integers(0, nrows, 4), rng.integers(0, C, 4)] = rng.integers(65535, 300000, 4)
    cnt[rng.choice(nrows, zero_rows, replace=False)] = 0
    return cnt


@pytest.mark.parametrize('C,r0,nrows', [(7140, 0, 7140), (7140, 1785, 1785), (1200, 1170, 30),
                                        (203, 0, 203), (1201, 7, 100)])
def test_compact_iteration_equals_dense(sa, C, r0, nrows):
    """sa_xt_compact_rows holds each row's non-zero columns and counts in order, and
    sa_xt_iterate_compact over it == sa_xt_iterate_rows (the dense count-row kernel), bit for
    bit, on random count rows (tabulated quotients, divided counts, escaped
    counts >= 65535, empty rows), a sub-range of rows (the row-sharded solve), x with zeros;
    the convergence flag and the no-op when the previous flag is 0."""
    _native, ops = sa['_native'], sa['ops']
    from socceraction_amd.batch import stream_handle
    lib = _native.lib()
    dev = torch.device('cuda')
    rng = np.random.default_rng(C + r0)
    rows = torch.from_numpy(_random_rows(rng, C, nrows)).to(dev)
    move_all = rng.integers(1, 10, C).astype(np.int64)
    move_all[r0:r0 + nrows] += rows.sum(dim=1, dtype=torch.int64).cpu().numpy()
    move = torch.from_numpy(move_all).to(dev)
    gs = torch.rand(C, dtype=torch.float64, device=dev) * 0.1
    pm = torch.rand(C, dtype=torch.float64, device=dev)
    ell = torch.empty(int(lib.sa_xt_compact_bytes(C, nrows)) // 4, dtype=torch.int32, device=dev)
    slen = torch.empty(nrows, dtype=torch.int32, device=dev)
    p = lambda t: t.data_ptr()  # noqa: E731
    _native.check(lib.sa_xt_compact_rows(p(rows), C, nrows, p(ell), p(slen), stream_handle()))
    h = rows.cpu().numpy()
    np.testing.assert_array_equal(slen.cpu().numpy(), (h != 0).sum(axis=1))
    pe = (C + 127) // 128 * 128  # the compact rows' pitch (whole 128-entry chunks)
    e = ell.cpu().numpy().view(np.uint32).reshape(nrows, pe)
    k = np.arange(pe)
    slot = (k & ~127) | (k % 32) << 2 | (k // 32) % 4  # chunk-interleaved: entry k's slot
    assert np.array_equal(np.sort(slot), k)
    for i in rng.choice(nrows, 5, replace=False):  # row i: its non-zero columns in order, counts
        nz = np.flatnonzero(h[i])
        ei = e[i, slot[:len(nz)]]
        np.testing.assert_array_equal(ei & 0xFFFF, nz)
        np.testing.assert_array_equal(ei >> 16, np.minimum(h[i, nz], 0xFFFF))
    for trial in range(3):
        x = torch.rand(C, dtype=torch.float64, device=dev)
        x[torch.from_numpy(rng.random(C) < 0.2).to(dev)] = 0.0
        a = torch.empty(nrows, dtype=torch.float64, device=dev)
        b = torch.empty(nrows, dtype=torch.float64, device=dev)
        fa = torch.zeros(1, dtype=torch.int32, device=dev)
        fb = torch.zeros(1, dtype=torch.int32, device=dev)
        eps = 1e-5 if trial < 2 else 10.0
        _native.check(lib.sa_xt_iterate_rows(p(rows), p(move), p(gs), p(pm), C, r0, nrows, p(x),
                                             eps, p(a), None, p(fa), stream_handle()))
        _native.check(lib.sa_xt_iterate_compact(p(ell), p(slen), p(rows), p(move), p(gs), p(pm), C,
                                                r0, nrows, p(x), eps, p(b), None, p(fb),
                                                stream_handle()))
        assert torch.equal(a, b), trial
        assert int(fa.item()) == int(fb.item()) == (1 if trial < 2 else 0)
    zero = torch.zeros(1, dtype=torch.int32, device=dev)
    b.fill_(-1.0)
    _native.check(lib.sa_xt_iterate_compact(p(ell), p(slen), p(rows), p(move), p(gs), p(pm), C, r0,
                                            nrows, p(x), 1e-5, p(b), p(zero), p(fb), stream_handle()))
    assert bool((b == -1.0).all())


# The reordered solve's iterates against the reference's order: the error bound allows 4e-11
# relative after 26 iterations at 105 x 68 (sa_xt_large.hip); the bar the tests hold is 1e-12.
REORDER_RTOL = 1e-12


def _close_rel(a, b, rtol=REORDER_RTOL):
    a, b = np.asarray(a), np.asarray(b)
    assert a.shape == b.shape
    np.testing.assert_array_equal(np.isnan(a), np.isnan(b))
    assert np.all(np.abs(a - b) <= rtol * np.abs(b) + 1e-300), np.max(np.abs(a - b) / np.maximum(np.abs(b), 1e-300))


def test_full_cfg4_batch_large_grid_solve(sa):
    """One full cfg2/cfg4 batch (10k games, ~16M actions) at 105 x 68: band count == the oracle's
    counts; the solve over the compact rows in the reference's order gives the oracle's iteration
    count and surface bit for bit, the default reordered solve the same count and every heatmap
    within 1e-12 relative."""
    B, ops, syn = sa['batch'], sa['ops'], sa['synthetic']
    d = syn.spadl_games(10000)
    ab = B.ActionBatch.from_columns(d)
    acc = ops.xt_count_many([ab], 105, 68)
    ref = _oracle(d, 105, 68)
    _same_counts(acc, ref, 105, 68)
    fit = xo.solve(ref, 105, 68)
    exact = ops.xt_solve(acc, transition=False, exact_order=True)
    assert exact.path == 'sequential' and exact.n_iter + 1 == len(fit['heatmaps'])
    np.testing.assert_array_equal(exact.mats[3].cpu().numpy().reshape(68, 105), fit['xT'])
    sol = ops.xt_solve(acc, transition=False)
    assert sol.path == 'reordered' and sol.n_iter == exact.n_iter
    _close_rel(sol.heatmaps.cpu().numpy().reshape(-1, 68, 105), fit['heatmaps'])
    again = ops.xt_solve(acc, transition=False)  # run to run: the same bits
    assert torch.equal(again.heatmaps, sol.heatmaps) and torch.equal(again.mats, sol.mats)


def _fit_like_rows(rng, C, dense=0.4, zero_rows=3, hot=0):
    """Count rows of a fit without escapes (every count < 65535) and the vectors of a system
    that converges: move[r] >= the row's transitions, gs and pmove like a fit's."""
    cnt = np.zeros((C, C), np.int32)
    nz = rng.random((C, C)) < dense
    cnt[nz] = rng.geometric(0.3, nz.sum())
    big = rng.random((C, C)) < 0.002
    cnt[big] = rng.integers(64, 5000, big.sum())
    if hot:
        cnt[rng.integers(0, C, hot), rng.integers(0, C, hot)] = rng.integers(65535, 300000, hot)
    cnt[rng.choice(C, zero_rows, replace=False)] = 0
    move = cnt.sum(axis=1, dtype=np.int64) + rng.integers(1, 50, C)
    gs = rng.random(C) * 0.05
    pm = rng.random(C) * 0.95
    return cnt, move, gs, pm


def _compact_solve(sa, cnt, move, gs, pm, eps, max_iter=1000, exact=False):
    _native, ops = sa['_native'], sa['ops']
    from socceraction_amd.batch import stream_handle
    lib = _native.lib()
    dev = torch.device('cuda')
    C = cnt.shape[0]
    rows = torch.from_numpy(cnt).to(dev)
    ell = torch.empty(int(lib.sa_xt_compact_bytes(C, C)) // 4, dtype=torch.int32, device=dev)
    slen = torch.empty(C, dtype=torch.int32, device=dev)
    _native.check(lib.sa_xt_compact_rows(rows.data_ptr(), C, C, ell.data_ptr(), slen.data_ptr(),
                                         stream_handle()))
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    heat, n, path = ops.xt_solve_compact(ell, slen, rows, t(move), t(gs), t(pm), C, eps, max_iter,
                                         exact_order=exact)
    return heat[:max(n, max_iter) + 1 if n < 0 else n + 1].cpu().numpy(), n, path


@pytest.mark.parametrize('C,dense', [(7140, 0.3), (1200, 0.6), (1025, 0.05), (9472, 0.1)])
def test_reordered_solve_vs_sequential(sa, C, dense):
    """sa_xt_solve_compact's reordered solve == the reference-order solve: the same iteration
    count, every iterate within 1e-12 relative, path 'reordered'; two runs give the same bits;
    max_iter reached first (-1) on both paths alike."""
    rng = np.random.default_rng(C)
    cnt, move, gs, pm = _fit_like_rows(rng, C, dense)
    h0, n0, p0 = _compact_solve(sa, cnt, move, gs, pm, 1e-5, exact=True)
    h1, n1, p1 = _compact_solve(sa, cnt, move, gs, pm, 1e-5)
    assert p0 == 'sequential' and p1 == 'reordered'
    assert n0 > 2 and n1 == n0
    _close_rel(h1, h0)
    h2, n2, _ = _compact_solve(sa, cnt, move, gs, pm, 1e-5)
    assert n2 == n1 and np.array_equal(h2, h1)
    m = n0 - 1  # stops one iteration short: not converged on either path
    h3, n3, p3 = _compact_solve(sa, cnt, move, gs, pm, 1e-5, max_iter=m)
    assert n3 == -1 and p3 == 'reordered'
    _close_rel(h3, h0[:m + 1])


def test_reordered_solve_inside_bound_falls_back(sa):
    """eps set to a cell's exact diff at some iteration: the reordered decision for that cell
    lies inside the error bound, so the solve is redone in the reference's order (path
    'inside-bound') and its iteration count and iterates are the reference order's, bit for
    bit."""
    rng = np.random.default_rng(5)
    C = 2000
    cnt, move, gs, pm = _fit_like_rows(rng, C, 0.2)
    h0, n0, _ = _compact_solve(sa, cnt, move, gs, pm, 1e-5, exact=True)
    k = n0 // 2
    eps = float(np.max(h0[k] - h0[k - 1]))  # the largest diff of iteration k: stops there
    he, ne, _ = _compact_solve(sa, cnt, move, gs, pm, eps, exact=True)
    hr, nr, pr = _compact_solve(sa, cnt, move, gs, pm, eps)
    assert pr == 'inside-bound'
    assert nr == ne and np.array_equal(hr, he)


def test_reordered_solve_with_escaped_counts(sa):
    """A count >= 65535 (held in the dense row only): the reordered solve declines (path
    'unavailable') and the reference-order solve runs, bit for bit."""
    rng = np.random.default_rng(6)
    cnt, move, gs, pm = _fit_like_rows(rng, 1500, 0.3, hot=3)
    assert cnt.max() >= 65535
    h0, n0, _ = _compact_solve(sa, cnt, move, gs, pm, 1e-5, exact=True)
    h1, n1, p1 = _compact_solve(sa, cnt, move, gs, pm, 1e-5)
    assert p1 == 'unavailable' and n1 == n0 and np.array_equal(h1, h0)


def test_interp_codes_rate_equals_rate_interp(sa):
    """The bucket pass's per-action interpolated-rate operands + sa_xt_rate_interp_codes ==
    sa_xt_rate_interp on the coordinates, bit for bit: values, NaN pattern and error bit 4
    (NaN / inf coordinates on successful moves, exact pitch edges, an odd-length batch)."""
    B, ops, syn = sa['batch'], sa['ops'], sa['synthetic']
    d = syn.spadl_games(31, game_id0=23)
    n = len(d['type_id'])
    d = {k: (v[:n - 1].copy() if isinstance(v, np.ndarray) and v.shape == (n,) else v)
         for k, v in d.items()}
    d['game_off'] = np.minimum(d['game_off'], n - 1)
    rng = np.random.default_rng(12)
    for col, v in (('start_x', 0.0), ('end_x', 105.0), ('start_y', 68.0), ('end_y', 0.0),
                   ('start_x', 104.99999999999999)):
        d[col][rng.choice(n - 1, 30, replace=False)] = v
    for bad in (False, True):
        if bad:
            for col, v in (('start_x', np.nan), ('end_y', np.inf), ('end_x', -np.inf)):
                d[col][rng.choice(n - 1, 5, replace=False)] = v
        ab = B.ActionBatch.from_columns(d)
        ic = ops.xt_interp_codes_buffer(ab.n, ab.device)
        acc = ops.xt_count_many([ab], 105, 68, interp_codes=[ic])
        xT = torch.rand((68, 105), dtype=torch.float64, device=ab.device)
        ref, e0 = ops.xt_rate_interp(ab, xT, 105, 68)
        got, e1 = ops.xt_rate_interp_codes(ic, ab.n, xT, 105, 68)
        a, b = ref.cpu().numpy(), got.cpu().numpy()
        np.testing.assert_array_equal(np.isnan(a), np.isnan(b))
        np.testing.assert_array_equal(a[~np.isnan(a)], b[~np.isnan(a)])
        assert int(e0.item()) == int(e1.item()) == (4 if bad else 0)
        assert bool(acc.err.item()) == bad


def test_interp_codes_rate_many_equals_per_batch(sa):
    """sa_xt_rate_interp_codes_many over 19 batches (two launches of <= 16 sets; odd, tiny and
    empty batches) == sa_xt_rate_interp_codes of each batch, bit for bit, one error word."""
    B, ops, syn = sa['batch'], sa['ops'], sa['synthetic']
    rng = np.random.default_rng(31)
    ns, ic, bs = [], [], []
    for k in range(19):
        if k % 6 == 4:  # an empty set
            ns.append(0)
            ic.append(ops.xt_interp_codes_buffer(0, 'cuda'))
            continue
        d = syn.spadl_games([1, 3, 7, 40][k % 4], game_id0=100 * k)
        N = len(d['type_id'])
        n = [1, 333, N, N - 1][k % 4] if N > 333 else N
        d = {c: (v[:n].copy() if isinstance(v, np.ndarray) and v.shape == (N,) else v)
             for c, v in d.items()}
        d['game_off'] = np.minimum(d['game_off'], n)
        if k == 5 and n > 10:
            d['start_x'][rng.choice(n, 60, replace=False)] = np.nan
        bs.append(B.ActionBatch.from_columns(d))
        ns.append(bs[-1].n)
        ic.append(ops.xt_interp_codes_buffer(bs[-1].n, bs[-1].device))
    ops.xt_count_many(bs, 105, 68, interp_codes=[c for c, n in zip(ic, ns) if n])
    xT = torch.rand((68, 105), dtype=torch.float64, device='cuda')
    got, err = ops.xt_rate_interp_codes_many(ic, ns, xT, 105, 68)
    want_err = 0
    for n, c, g in zip(ns, ic, got):
        assert g.numel() == n
        if n == 0:
            continue
        ref, e = ops.xt_rate_interp_codes(c, n, xT, 105, 68)
        want_err |= int(e.item())
        a, r = g.cpu().numpy(), ref.cpu().numpy()
        np.testing.assert_array_equal(np.isnan(a), np.isnan(r))
        np.testing.assert_array_equal(a[~np.isnan(r)], r[~np.isnan(r)])
    assert want_err == 4 and int(err.item()) == want_err


def test_fresh_accumulator_overwrite_ignores_stale_memory(sa):
    """xt_count_many's fresh accumulator is not zero-filled (the count overwrites every row):
    counts equal the oracle's even when the allocator hands back memory full of junk."""
    B, ops, syn = sa['batch'], sa['ops'], sa['synthetic']
    l, w = 105, 68
    C = l * w
    junk = torch.full((3 * C * 8 + 512 + C * C * 4 + 4096,), 0x5A, dtype=torch.uint8, device='cuda')
    del junk  # back to the caching allocator, bytes intact
    d = syn.spadl_games(25)
    ab = B.ActionBatch.from_columns(d)
    acc = ops.xt_count_many([ab], l, w)
    ops.xt_check_errors(acc)
    _same_counts(acc, _oracle(d, l, w), l, w)


def test_coresident_16x12_count_full_batch_vs_oracle(sa):
    """The co-resident count (shared=True: the workgroup shape the bench step's side stream
    uses next to the VAEP passes) over cfg2's whole 10k-game batch (~16M actions) == the
    oracle's counts, and == the default launch shape's."""
    B, ops, syn = sa['batch'], sa['ops'], sa['synthetic']
    l, w = 16, 12
    d = syn.spadl_games(10000)
    ab = B.ActionBatch.from_columns(d)
    acc = ops.xt_count(ab, l, w, shared=True)
    ops.xt_check_errors(acc)
    _same_counts(acc, _oracle(d, l, w), l, w)
    ref = ops.xt_count(ab, l, w)
    for a, b in ((acc.shot, ref.shot), (acc.goal, ref.goal), (acc.move, ref.move), (acc.trans, ref.trans)):
        assert torch.equal(a, b)


@pytest.mark.parametrize('l,w,hot', [(105, 68, False), (105, 68, True), (40, 30, True)])
def test_compact_only_count_skips_the_dense_table(sa, l, w, hot):
    """xt_count_many(dense=False) (SA_XT_COUNT_COMPACT_ONLY): the same shot / goal / move counts
    and compact rows as the dense count, entry for entry; the dense rows written ONLY for the
    bands holding a count >= 65535 (the rows the compact solve reads; every other row keeps the
    sentinel it held); the transition entries read back from the compact rows == the dense
    table's non-zero bins; the solve == the dense count's solve bit for bit (incl. the escaped
    case's fallback to the reference order); ops that read the dense table refuse the count."""
    B, ops, syn = sa['batch'], sa['ops'], sa['synthetic']
    C = l * w
    ds = [syn.spadl_games(g, game_id0=17 * i + 3) for i, g in enumerate((150 if hot else 60, 45))]
    if hot:  # one bin far above 65535 counts: its band's dense rows must be written
        mv = np.isin(ds[0]['type_id'], (0, 1, 21))
        ds[0]['start_x'][mv], ds[0]['start_y'][mv] = 52.2, 33.3
        ds[0]['end_x'][mv], ds[0]['end_y'][mv] = 104.999, 0.0
    abs_ = [B.ActionBatch.from_columns(d) for d in ds]
    ref = ops.xt_count_many(abs_, l, w)
    acc = ops.xt_zero_counts(l, w, abs_[0].device, zero_counts=False)
    acc.trans.fill_(-7)
    ops.xt_count_many(abs_, l, w, acc=acc, overwrite=True, dense=False)
    assert not acc.dense and acc.compact is not None and ref.dense
    for a, b in ((acc.shot, ref.shot), (acc.goal, ref.goal), (acc.move, ref.move), (acc.err, ref.err)):
        assert torch.equal(a, b)
    (ea, ra), (eb, rb) = acc.compact, ref.compact
    assert torch.equal(ra, rb)
    pe = ea.numel() // C
    xa, xb = ea.cpu().numpy().reshape(C, pe), eb.cpu().numpy().reshape(C, pe)
    lens = ra.cpu().numpy()
    for r in np.flatnonzero(lens):
        sl = _xe_slots(np.arange(lens[r]))
        np.testing.assert_array_equal(xa[r, sl], xb[r, sl])
    R, NB = ops.xt_band_shape(l, w)
    dense_ref = ref.trans.cpu().numpy().reshape(C, C)
    got = acc.trans.cpu().numpy().reshape(C, C)
    esc_rows = np.flatnonzero(dense_ref.max(axis=1) >= 65535)
    esc_bands = set((esc_rows // R).tolist())
    assert bool(esc_bands) == hot
    for band in range(NB):
        rows = slice(band * R, min(C, band * R + R))
        if band in esc_bands:
            np.testing.assert_array_equal(got[rows], dense_ref[rows])
        else:
            assert (got[rows] == -7).all(), band
    idx, cnt = ops.xt_transition_entries(acc)
    nz = np.flatnonzero(dense_ref.reshape(-1))
    np.testing.assert_array_equal(idx.cpu().numpy(), nz)
    np.testing.assert_array_equal(cnt.cpu().numpy(), dense_ref.reshape(-1)[nz])
    sol = ops.xt_solve(acc, transition=False)
    want = ops.xt_solve(ref, transition=False)
    assert sol.path == want.path == ('unavailable' if hot else 'reordered')
    assert sol.n_iter == want.n_iter
    assert torch.equal(sol.heatmaps, want.heatmaps) and torch.equal(sol.mats, want.mats)
    for bad in (lambda: ops.xt_normalize(acc), lambda: ops.xt_solve(acc, transition=True),
                lambda: ops.xt_count(abs_[0], l, w, acc)):
        with pytest.raises(ValueError, match='dense'):
            bad()


def test_cell_code_bucket_count_small_grid(sa):
    """sa_xt_count_bucket from 16-bit cell codes (grids of <= SA_XT_CELLS16_MAX_C cells, 16 x 12;
    ADVICE r05): K1 loads and decodes them like the small-grid count, so the band-owned count
    from the codes == sa_xt_count of the coordinates; 32-bit codes (40 x 30) the same."""
    import ctypes

    B, ops, syn, N = sa['batch'], sa['ops'], sa['synthetic'], sa['_native']
    from socceraction_amd.batch import stream_handle
    d = syn.spadl_games(30, game_id0=71)
    ab = B.ActionBatch.from_columns(d)
    lib = N.lib()
    for l, w in ((16, 12), (40, 30)):
        rr, nn = ctypes.c_int32(0), ctypes.c_int32(0)
        N.check(lib.sa_xt_band_shape(l, w, ctypes.byref(rr), ctypes.byref(nn)))
        cells = ops.xt_cells(ab, l, w)
        err = torch.zeros(1, dtype=torch.int32, device=ab.device)
        keys = torch.empty(max(ab.n, 16), dtype=torch.int32, device=ab.device)
        off = torch.empty(nn.value + 1, dtype=torch.int64, device=ab.device)
        N.check(lib.sa_xt_count_bucket(None, cells.data_ptr(), ab.n, l, w, keys.data_ptr(),
                                       off.data_ptr(), err.data_ptr(), None, None, 1050, 680,
                                       stream_handle()))
        acc = ops.xt_zero_counts(l, w, ab.device)
        kp = (ctypes.c_void_p * 1)(keys.data_ptr())
        op = (ctypes.c_void_p * 1)(off.data_ptr())
        N.check(lib.sa_xt_count_from_buckets(1, kp, op, l, w, acc.shot.data_ptr(), acc.goal.data_ptr(),
                                             acc.move.data_ptr(), acc.trans.data_ptr(),
                                             N.SA_XT_COUNT_OVERWRITE, stream_handle()))
        ref = ops.xt_count(ab, l, w)
        for a, b in ((acc.shot, ref.shot), (acc.goal, ref.goal), (acc.move, ref.move),
                     (acc.trans, ref.trans)):
            assert torch.equal(a, b), (l, w)
        assert int(err.item()) == int(ref.err.item())


@pytest.mark.parametrize('hot', [False, True])
def test_fused_fit_rate_equals_solve_then_rate(sa, hot):
    """sa_xt_fit_rate_interp_codes (the rate queued behind the one-launch solve, before its host
    round trip) == xt_solve(transition=False) then xt_rate_interp_codes_many: iteration count,
    path, matrices, heatmaps and every rate bit for bit; with an escaped count (hot) the solve
    takes the reference's order after the speculative rate ran, and the rate is redone over the
    rewritten surface."""
    B, ops, syn = sa['batch'], sa['ops'], sa['synthetic']
    ds = [syn.spadl_games(g, game_id0=41 * i + 7) for i, g in enumerate((120 if hot else 90, 37))]
    if hot:  # one bin far above 65535 counts: the compact solve cannot take it
        mv = np.isin(ds[0]['type_id'], (0, 1, 21))
        ds[0]['start_x'][mv], ds[0]['start_y'][mv] = 52.2, 33.3
        ds[0]['end_x'][mv], ds[0]['end_y'][mv] = 104.999, 0.0
    bs = [B.ActionBatch.from_columns(d) for d in ds]
    ns = [b.n for b in bs]
    ic = [ops.xt_interp_codes_buffer(b.n, b.device) for b in bs]
    acc = ops.xt_count_many(bs, 105, 68, interp_codes=ic, dense=hot)
    sol = ops.xt_solve(acc, transition=False)
    ref, ref_err = ops.xt_rate_interp_codes_many(ic, ns, sol.mats[3].reshape(68, 105), 105, 68)
    sol2, got, err = ops.xt_fit_rate_interp_codes(acc, ic, ns)
    assert sol2.path == sol.path == ('unavailable' if hot else 'reordered')
    assert sol2.n_iter == sol.n_iter
    assert torch.equal(sol2.mats, sol.mats) and torch.equal(sol2.heatmaps, sol.heatmaps)
    for g, r in zip(got, ref):
        assert torch.equal(g.view(torch.int64), r.view(torch.int64))  # NaN patterns included
    assert int(err.item()) == int(ref_err.item())
    with pytest.raises(ValueError):
        ops.xt_fit_rate_interp_codes(ops.xt_count_many(bs, 16, 12), ic, ns)
