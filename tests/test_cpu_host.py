"""CPU-only tests: C-ABI library surface, host-side logic (catalogue, plans, batches,
sharding) and the host helpers the reference's own tests pin. No GPU needed."""
import json
import os
import re

import numpy as np
import pandas as pd
import pytest

from golden_io import cases, inputs, ks, load

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


# ----------------------------------------------------------------------------- C ABI
def _declared_functions():
    with open(os.path.join(ROOT, 'include', 'socceraction_amd.h')) as f:
        src = f.read()
    src = re.sub(r'/\*.*?\*/', '', src, flags=re.S)
    return sorted(set(re.findall(r'\b(sa_[a-z0-9_]+)\s*\(', src)))


def test_library_builds_and_exports_every_declared_symbol():
    from socceraction_amd import _native, build
    build.build(force=False, verbose=False)
    lib = _native.load_library()
    declared = _declared_functions()
    assert 'sa_vaep_features' in declared and 'sa_xt_solve' in declared
    for sym in declared:
        assert hasattr(lib, sym), sym
    assert set(declared) == set(_native.EXPORTED_SYMBOLS)
    assert lib.sa_abi_version() == 3
    assert lib.sa_debug_enabled() == 0
    assert lib.sa_debug_check() == 0  # default build: no device checks, no device call


def test_build_id_ties_the_library_to_its_sources(tmp_path):
    """sa_build_id() is the hash of the sources + flags; build.py rebuilds on a hash change (not
    file times) and the loader refuses a library whose id differs from the sources next to it."""
    from socceraction_amd import _native, build
    build.build(force=False, verbose=False)
    lib = _native.load_library()
    bid = build.build_id()
    assert lib.sa_build_id().decode() == bid == build.file_build_id(build.OUT)
    assert build.build_id(build.DEBUG_DEFINES) != bid
    # a stale copy (other defines) is refused when loaded as the default library
    stale = tmp_path / 'libstale.so'
    build.build(force=True, verbose=False, defines=('SA_NT_STORES=0',), out=str(stale))
    assert build.file_build_id(str(stale)) == build.build_id(('SA_NT_STORES=0',))
    other = _native.load_library(str(stale))  # an explicit variant path is not checked
    with pytest.raises(ImportError):
        _native._check_build_id(other, _native.DEFAULT_LIB)


def test_debug_library_builds_with_device_checks():
    from socceraction_amd import _native, build
    path = build.build_debug(verbose=False)
    lib = _native.load_library(path)
    _native._check_build_id(lib, _native.DEBUG_LIB)
    assert lib.sa_debug_enabled() == 1
    assert lib.sa_build_id().decode() == build.build_id(build.DEBUG_DEFINES)
    for sym in _native.EXPORTED_SYMBOLS:
        assert hasattr(lib, sym), sym


def test_shutdown_without_scratch_is_a_no_op():
    from socceraction_amd import _native
    lib = _native.load_library()
    assert lib.sa_shutdown() == 0


def test_ctypes_struct_layout_matches_header():
    """Struct sizes the kernels see: sa_frame = 10 pointers, sa_actions = 40 B + 8 frames."""
    import ctypes

    from socceraction_amd import _native
    assert ctypes.sizeof(_native.SaFrame) == 80
    assert ctypes.sizeof(_native.SaActions) == 40 + 8 * 80 + 8
    assert ctypes.sizeof(_native.SaFeaturePlan) == 4 * (1 + 3 * _native.SA_XFN_COUNT)
    assert ctypes.sizeof(_native.SaBlock) == 24
    assert ctypes.sizeof(_native.SaTreeModel) == 4 * 8 + 2 * 4 + 8 + 8  # sa_tree_model
    with open(os.path.join(ROOT, 'include', 'socceraction_amd.h')) as f:
        enum = f.read().split('enum sa_xfn {')[1].split('};')[0]
    names = re.findall(r'SA_XFN_([A-Z_]+)', enum)
    assert [n.lower() for n in names[:-1]] == _native.XFN_NAMES and names[-1] == 'COUNT'


def test_invalid_arguments_are_rejected_without_a_gpu():
    """Argument validation happens before any HIP call (returns SA_EINVAL)."""
    import ctypes

    from socceraction_amd import _native
    lib = _native.load_library()
    s = _native.SaActions()
    s.n, s.n_segments, s.n_frames = 10, 1, 0
    plan = _native.SaFeaturePlan()
    rc = lib.sa_vaep_features(ctypes.byref(s), ctypes.byref(plan), None, None, None, None)
    assert rc == _native.SA_EINVAL
    assert b'n_frames' in lib.sa_last_error()
    with pytest.raises(ValueError):
        _native.check(rc)
    # round-5 entry points: their argument checks too come before any HIP call
    fake = ctypes.c_void_p(256)  # never dereferenced on the host
    none_p = ctypes.POINTER(ctypes.c_void_p)()
    rc = lib.sa_xt_count_from_buckets_ex(0, none_p, none_p, 105, 68, fake, fake, fake, fake,
                                         _native.SA_XT_COUNT_OVERWRITE, fake, None, None)
    assert rc == _native.SA_EINVAL and b'together' in lib.sa_last_error()
    rc = lib.sa_xt_count_from_buckets_ex(0, none_p, none_p, 105, 68, fake, fake, fake, fake, 0,
                                         fake, fake, None)
    assert rc == _native.SA_EINVAL and b'OVERWRITE' in lib.sa_last_error()
    n_iter, path = ctypes.c_int32(0), ctypes.c_int32(0)
    rc = lib.sa_xt_solve_ex(fake, fake, fake, fake, 16, 12, 1e-5, 100, 0, fake, fake, fake,
                            ctypes.byref(n_iter), ctypes.byref(path), fake, fake, None)
    assert rc == _native.SA_EINVAL and b'compact' in lib.sa_last_error()
    rc = lib.sa_xt_solve_ex(fake, fake, fake, fake, 105, 68, 1e-5, 100, 4, fake, None, fake,
                            ctypes.byref(n_iter), ctypes.byref(path), None, None, None)
    assert rc == _native.SA_EINVAL and b'flags' in lib.sa_last_error()
    rc = lib.sa_xt_rate_interp_codes_many(-1, none_p, None, fake, fake, fake, 105, 68, fake, 1050,
                                          fake, 680, none_p, fake, None)
    assert rc == _native.SA_EINVAL
    # round 6: the fused fit + rate checks its grid and the rate's arguments before launching
    fit_rate = lambda l, w, nsets, L: lib.sa_xt_fit_rate_interp_codes(  # noqa: E731
        fake, fake, fake, fake, l, w, 1e-5, 100, 0, fake, fake, ctypes.byref(n_iter),
        ctypes.byref(path), fake, fake, nsets, none_p, None, fake, fake, fake, L, fake, 680, none_p,
        fake, None)
    assert fit_rate(16, 12, 0, 1050) == _native.SA_EINVAL and b'above' in lib.sa_last_error()
    assert fit_rate(105, 68, -1, 1050) == _native.SA_EINVAL and b'rate' in lib.sa_last_error()
    assert fit_rate(105, 68, 0, 0) == _native.SA_EINVAL and b'rate' in lib.sa_last_error()


# ----------------------------------------------------------------------------- catalogue
@pytest.mark.parametrize('prefix', ['spadl', 'atomic'])
def test_catalogue_names_match_reference(prefix):
    from socceraction_amd import catalog
    from socceraction_amd.atomic.vaep import base as abase
    from socceraction_amd.vaep import base as vbase
    atomic = prefix == 'atomic'
    xfns = [f._sa_xfn for f in (abase.xfns_default if atomic else vbase.xfns_default)]
    for name in cases(prefix):
        g = load(prefix, name)
        for k in ks(g):
            plan = catalog.build_plan(xfns, k, atomic)
            assert plan.names == list(g[f'k{k}_names_all'])
            assert [c[1] for c in plan.order] == list(g[f'k{k}_kinds_all'])


def test_default_plan_block_sizes():
    from socceraction_amd import catalog
    from socceraction_amd.atomic.vaep import base as abase
    from socceraction_amd.vaep import base as vbase
    p = catalog.build_plan([f._sa_xfn for f in vbase.xfns_default], 3)
    assert (p.n_bool, p.n_f64, p.n_i64) == (515, 47, 6)
    p = catalog.build_plan([f._sa_xfn for f in abase.xfns_default], 3, atomic=True)
    assert (p.n_bool, p.n_f64, p.n_i64) == (110, 32, 12)
    with pytest.raises(ValueError):
        catalog.build_plan(['location'], 3, atomic=False)
    with pytest.raises(ValueError):
        catalog.build_plan(['movement'], 3, atomic=True)
    # any nb_prev_actions (vaep/features.py:62-88); 0 gives the one frame of gamestates(a, 0)
    p = catalog.build_plan(list(catalog.SPADL_XFNS[:1]) + ['time', 'team', 'space_delta'], 17)
    assert p.struct.nb_prev_actions == 17 and p.names[-1] == 'mov_a016'
    assert catalog.build_plan(['time'], 0).names == catalog.build_plan(['time'], 1).names


def test_feature_column_names_with_user_transformer():
    from socceraction_amd.vaep import base as vbase
    from socceraction_amd.vaep import features as fs

    @fs.simple
    def myfeat(actions):
        return pd.DataFrame({'double_x': actions['start_x'] * 2})

    names = fs.feature_column_names(vbase.xfns_default + [myfeat], 2)
    assert names[-2:] == ['double_x_a0', 'double_x_a1']
    g = load('spadl', 'fixture')
    assert fs.feature_column_names(vbase.xfns_default, 3) == list(g['k3_names_all'])


def test_host_gamestates_and_flip_match_oracle():
    from oracle import vaep_oracle as vo
    from socceraction_amd.vaep import features as fs
    g = load('spadl', 'n40')
    cols = inputs(g)
    df = pd.DataFrame(cols)
    gs = fs.play_left_to_right(fs.gamestates(df, 3), g['home_team_id'][0])
    for i, a in enumerate(gs):
        rows = vo.window_rows(len(df), np.array([0, len(df)]), i)
        away = cols['team_id'] != g['home_team_id'][0]
        exp = np.where(away, 105.0 - cols['start_x'][rows], cols['start_x'][rows])
        np.testing.assert_array_equal(a['start_x'].to_numpy(), exp)


# ----------------------------------------------------------------------------- batches
def test_encode_teams_preserves_equality():
    from socceraction_amd.batch import encode_teams
    ids = np.array(['b', 'a', 'b', 'c'], dtype=object)
    codes, home = encode_teams(ids, ['c', 'zz'])
    assert (codes[0] == codes[2]) and len(set(codes.tolist())) == 3
    assert home[0] == codes[3] and home[1] == -1
    big = np.array([2**40, 5, 2**40])
    codes, home = encode_teams(big, [5])
    assert codes[0] == codes[2] != codes[1] and home[0] == codes[1]
    with pytest.raises(ValueError):
        encode_teams(np.array([1.0, np.nan]))


def test_encode_columns_validates_like_the_schema():
    from socceraction_amd.batch import encode_columns
    g = load('spadl', 'fixture')
    df = pd.DataFrame(inputs(g))
    cols = encode_columns(df, atomic=False)
    assert cols['type_id'].dtype == np.uint8 and cols['c0'].dtype == np.float64
    bad = df.copy()
    bad.loc[3, 'type_id'] = 23
    with pytest.raises(ValueError):
        encode_columns(bad, atomic=False)
    bad = df.copy()
    bad.loc[3, 'result_id'] = 6
    with pytest.raises(ValueError):
        encode_columns(bad, atomic=False)
    names = df.drop(columns=['type_id']).assign(type_name=['pass'] * len(df))
    assert (encode_columns(names, atomic=False)['type_id'] == 0).all()


def test_segment_offsets():
    from socceraction_amd.batch import segment_offsets
    np.testing.assert_array_equal(segment_offsets(np.array([7, 7, 3, 3, 3, 9])), [0, 2, 5, 6])
    np.testing.assert_array_equal(segment_offsets(np.array([], dtype=np.int64)), [0])


# ----------------------------------------------------------------------------- sharding
def test_partition_games_covers_every_game_once():
    from socceraction_amd import shard, synthetic
    d = synthetic.spadl_games(101)
    off = d['game_off']
    for world in (1, 2, 3, 4, 8):
        parts = shard.partition_games(off, world)
        assert parts[0][0] == 0 and parts[-1][1] == 101
        assert all(a[1] == b[0] for a, b in zip(parts, parts[1:]))
        sizes = [off[b] - off[a] for a, b in parts]
        assert max(sizes) - min(sizes) <= 2 * 2000  # within two games of balance


def _gloo_worker(rank, world, port, q):
    import torch
    import torch.distributed as dist

    from oracle import xt_oracle as xo
    from socceraction_amd import shard, synthetic
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    d = synthetic.spadl_games(6, seed=9)
    off = d['game_off']
    g0, g1 = shard.partition_games(off, world)[rank]
    s, e = int(off[g0]), int(off[g1])
    l, w = 8, 6
    C = l * w
    cols = {c: d[c][s:e] for c in ('start_x', 'start_y', 'end_x', 'end_y', 'type_id', 'result_id')}
    t = cols['type_id']
    shot = t == 11
    move = (t == 0) | (t == 21) | (t == 1)
    succ = move & (cols['result_id'] == 1)
    cnt = lambda m, x, y: np.bincount(xo.flat_indexes(x[m], y[m], l, w), minlength=C)  # noqa: E731
    from socceraction_amd import ops
    acc = ops.xt_zero_counts(l, w, 'cpu')  # the device layout, on the host for gloo
    acc.shot.copy_(torch.tensor(cnt(shot, cols['start_x'], cols['start_y'])))
    acc.goal.copy_(torch.tensor(cnt(shot & (cols['result_id'] == 1), cols['start_x'], cols['start_y'])))
    acc.move.copy_(torch.tensor(cnt(move, cols['start_x'], cols['start_y'])))
    tr = np.zeros(C * C, np.int32)
    np.add.at(tr, xo.flat_indexes(cols['start_x'][succ], cols['start_y'][succ], l, w) * C +
              xo.flat_indexes(cols['end_x'][succ], cols['end_y'][succ], l, w), 1)
    acc.trans.copy_(torch.tensor(tr))
    # rank 0 flags an infinite shot start, rank 1 that and an infinite move start: the byte
    # lanes add up without touching each other
    acc.err.fill_(ops.XT_ERR_SHOT & 0x1 if rank == 0 else 0x101)
    acc.compact = (torch.zeros(4, dtype=torch.int32), torch.zeros(1, dtype=torch.int32))
    shard.allreduce_xt_counts(acc)  # ONE all-reduce
    assert acc.compact is None  # this rank's compact rows describe its own counts only
    if rank == 0:
        q.put((acc.shot.numpy().copy(), acc.goal.numpy().copy(), acc.move.numpy().copy(),
               acc.trans.numpy().copy(), int(acc.err.item())))
    dist.destroy_process_group()


def test_xt_counts_drop_compact_rows_when_the_counts_change():
    """XTCounts.compact (the compact rows a band count wrote for the solve) never outlives the
    counts it describes: zeroing drops it (the all-reduce case is in the gloo test)."""
    import torch

    from socceraction_amd import ops
    acc = ops.xt_zero_counts(105, 68, 'cpu')
    assert acc.compact is None
    acc.compact = (torch.zeros(4, dtype=torch.int32), torch.zeros(1, dtype=torch.int32))
    acc.zero_()
    assert acc.compact is None


def test_xt_count_allreduce_gloo_world2():
    """World-size-2 gloo run of the xT exchange step: sharded counts sum to the global ones."""
    import multiprocessing as mp
    import socket

    from oracle import xt_oracle as xo
    from socceraction_amd import synthetic
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        port = s.getsockname()[1]
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    procs = [ctx.Process(target=_gloo_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    sh, go, mv, tr, err = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert err == 0x102  # shot flag from both ranks (2), move-start flag from rank 1 (1)
    from socceraction_amd import ops
    assert err & ops.XT_ERR_SHOT and err & ops.XT_ERR_MOVE_START and not err & ops.XT_ERR_MOVE_OTHER
    d = synthetic.spadl_games(6, seed=9)
    f = xo.fit({c: d[c] for c in ('start_x', 'start_y', 'end_x', 'end_y', 'type_id',
                                  'result_id')}, 8, 6)
    total = mv.astype(np.float64) + sh
    np.testing.assert_array_equal(np.divide(sh, total, out=np.zeros(48), where=total != 0),
                                  f['shot_prob'].reshape(-1))
    T = np.zeros((48, 48))
    t2 = tr.reshape(48, 48)
    nz = t2 != 0
    T[nz] = t2[nz] / mv.astype(np.float64)[np.nonzero(nz)[0]]
    np.testing.assert_array_equal(T, f['transition'])


def _band_keys(rank, part, R, NB):
    """Synthetic bucketed keys of one local batch, int16 like sa_xt_count_bucket's bins, sorted
    by band; for the test each key also names its band (band * 1000 + bin, bin < 1000)."""
    rng = np.random.default_rng([rank, part, 5])
    n = int(rng.integers(0, 400))
    cs = rng.integers(0, NB * R - 2, n)  # the last band is partial (C = NB R - 2)
    band = cs // R
    keys = (band * 1000 + (cs - band * R) * 100 + rng.integers(0, 50, n)).astype(np.int64)
    order = np.argsort(band, kind='stable')
    off = np.concatenate([[0], np.cumsum(np.bincount(band, minlength=NB))])
    return keys[order].astype(np.int16), off.astype(np.int64)


_BAND_PARTS = {2: (2, 1), 3: (2, 0, 1)}  # local batches per rank: uneven, one rank with none


def _band_exchange_worker(rank, world, port, q):
    import torch
    import torch.distributed as dist

    from socceraction_amd import shard
    dist.init_process_group('gloo', init_method=f'tcp://127.0.0.1:{port}', rank=rank,
                            world_size=world)
    R, NB = 3, 11
    nparts = _BAND_PARTS[world][rank]  # the ranks run different numbers of local batches
    parts = [tuple(torch.from_numpy(a) for a in _band_keys(rank, k, R, NB)) for k in range(nparts)]
    stats = {}
    keys, offs = shard.exchange_band_keys(parts, NB, dev=torch.device('cpu'), stats=stats)
    assert stats['host_reads'] == 1, stats  # one host read for every round's splits
    b0, b1 = shard.band_ranges(NB, world)[rank]
    got = []
    for k, o in zip(keys, offs):
        o = o.numpy()
        kk = k.numpy().astype(np.int64)
        for lb in range(b1 - b0):  # every key of local band lb belongs to band b0 + lb
            seg = kk[o[lb]:o[lb + 1]]
            assert (seg // 1000 == b0 + lb).all()
            got.append(seg)
    q.put((rank, np.sort(np.concatenate(got)) if got else np.zeros(0, np.int64), len(keys)))
    dist.destroy_process_group()


@pytest.mark.parametrize('world', [2, 3])
def test_band_key_exchange_gloo(world):
    """shard.exchange_band_keys (the band-sharded xT fit's all-to-all) over gloo, world 2 and 3
    (3: uneven band ownership 4 / 4 / 3 bands, a rank with no local batch), with a different
    number of local batches per rank: each rank receives exactly the keys of its own bands from
    every rank's every batch, with band offsets relative to its first band, after ONE host read
    of the split sizes (stats['host_reads'])."""
    import multiprocessing as mp
    import socket

    from socceraction_amd import shard
    assert shard.band_ranges(11, 2) == [(0, 6), (6, 11)]
    assert shard.band_ranges(11, 3) == [(0, 4), (4, 8), (8, 11)]
    assert shard.band_ranges(3, 4) == [(0, 1), (1, 2), (2, 3), (3, 3)]
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        port = s.getsockname()[1]
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    procs = [ctx.Process(target=_band_exchange_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict((r, (keys, n)) for r, keys, n in (q.get(timeout=120) for _ in range(world)))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    R, NB = 3, 11
    every = np.concatenate([_band_keys(r, k, R, NB)[0].astype(np.int64)
                            for r, nparts in enumerate(_BAND_PARTS[world]) for k in range(nparts)])
    for r, (b0, b1) in enumerate(shard.band_ranges(NB, world)):
        band = every // 1000
        want = np.sort(every[(band >= b0) & (band < b1)])
        np.testing.assert_array_equal(res[r][0], want)
        assert res[r][1] == 2 * world  # two rounds (rank 0's batches) x every source rank


def _band_exchange_limit_worker(rank, world, port, q):
    import torch
    import torch.distributed as dist

    from socceraction_amd import shard
    dist.init_process_group('gloo', init_method=f'tcp://127.0.0.1:{port}', rank=rank,
                            world_size=world)
    R, NB = 3, 11
    nparts = shard._MAX_ROUNDS + 1 if rank == 0 else 1  # only rank 0 is over the limit
    parts = [tuple(torch.from_numpy(a) for a in _band_keys(rank, k, R, NB)) for k in range(nparts)]
    try:
        shard.exchange_band_keys(parts, NB, dev=torch.device('cpu'))
        q.put((rank, 'no error'))
    except ValueError as e:
        q.put((rank, 'ValueError' if 'local batches' in str(e) else repr(e)))
    dist.destroy_process_group()


def test_band_key_exchange_over_limit_raises_on_every_rank():
    """A rank with more local batches than one band exchange takes: every rank
    raises ValueError after the header all-to-all -- none is left waiting in a collective."""
    import multiprocessing as mp
    import socket
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        port = s.getsockname()[1]
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    procs = [ctx.Process(target=_band_exchange_limit_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res == {0: 'ValueError', 1: 'ValueError'}


def _compact_pack_worker(rank, world, port, q):
    import torch
    import torch.distributed as dist

    from socceraction_amd import shard
    dist.init_process_group('gloo', init_method=f'tcp://127.0.0.1:{port}', rank=rank,
                            world_size=world)
    C, pe = 23, 384  # 3 chunks per row slot
    B = -(-C // world)
    lens = np.random.default_rng(7).integers(0, pe + 1, C)  # every rank knows every length
    r0, nrows = rank * B, max(0, min(B, C - rank * B))
    ell = torch.from_numpy(np.random.default_rng([rank, 8]).integers(0, 2 ** 31, max(nrows, 1) * pe)
                           .astype(np.int32))
    nch = torch.from_numpy((lens + 127) // 128)
    rank_chunks = np.array([((lens[qq * B:min(C, (qq + 1) * B)] + 127) // 128).sum()
                            for qq in range(world)], np.int64)
    mx = int(rank_chunks.max())
    send = torch.zeros(mx * 128, dtype=torch.int32)
    mine = shard.pack_compact_rows(ell, nch[r0:r0 + nrows], pe, int(rank_chunks[rank]))
    send[:mine.numel()] = mine
    recv = torch.empty(world * mx * 128, dtype=torch.int32)
    shard._all_gather(recv, send)
    full = torch.full((C * pe,), -1, dtype=torch.int32)
    shard.unpack_compact_rows(recv, mx, rank_chunks, nch, B, pe, full)
    q.put((rank, ell.numpy(), full.numpy()))
    dist.destroy_process_group()


def test_compact_row_pack_unpack_gloo_world3():
    """The band-sharded solve's compact-row exchange (shard.pack_compact_rows -> all-gather ->
    shard.unpack_compact_rows) over gloo with 3 ranks and uneven row blocks (23 rows: 8 / 8 / 7):
    every row's used 128-slot chunks land where the single-GPU compact form holds them, and the
    slots past them are untouched."""
    import multiprocessing as mp
    import socket
    world = 3
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        port = s.getsockname()[1]
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    procs = [ctx.Process(target=_compact_pack_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {r: (e, f) for r, e, f in (q.get(timeout=120) for _ in range(world))}
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    C, pe = 23, 384
    B = -(-C // world)
    lens = np.random.default_rng(7).integers(0, pe + 1, C)
    for r in range(world):
        full = res[r][1].reshape(C, pe)
        for i in range(C):
            owner, li = i // B, i % B
            used = (lens[i] + 127) // 128 * 128
            src = res[owner][0].reshape(-1, pe)[li]
            np.testing.assert_array_equal(full[i, :used], src[:used])
            assert (full[i, used:] == -1).all()


# ----------------------------------------------------------------------------- synthetic data
def test_synthetic_generator_shape_and_determinism():
    from socceraction_amd import synthetic
    a = synthetic.spadl_games(20)
    b = synthetic.spadl_games(20)
    for k in a:
        np.testing.assert_array_equal(a[k], b[k])
    sizes = np.diff(a['game_off'])
    assert sizes.min() >= 1200 and sizes.max() <= 2000
    assert a['start_x'].min() >= 0 and a['start_x'].max() <= 105
    assert a['end_y'].min() >= 0 and a['end_y'].max() <= 68
    df = synthetic.to_frame(a)
    assert len(df) == a['game_off'][-1] and df['type_id'].dtype == np.int64
    gaps = df.groupby('game_id').time_seconds.diff().dropna()
    assert 0.01 < (gaps.abs() > 10).mean() < 0.2
    at = synthetic.atomic_games(3)
    assert (at['type_id'] == 27).any() and at['type_id'].max() <= 32


# ----------------------------------------------------------------------------- xT host helpers
class TestGridCount:
    """Known-answer tests of reference tests/test_xthreat.py:44-78 (host index helpers)."""

    N = 2
    M = 2

    def test_get_cell_indexes(self):
        from socceraction_amd import xthreat as xt
        x = pd.Series([0, 105 / 2 - 1, 105.0])
        y = pd.Series([0, 68 / 2 + 1, 68.0])
        xi, yi = xt._get_cell_indexes(x, y, self.N, self.M)
        pd.testing.assert_series_equal(xi, pd.Series([0, 0, 1]))
        pd.testing.assert_series_equal(yi, pd.Series([0, 1, 1]))

    def test_get_cell_indexes_out_of_bounds(self):
        from socceraction_amd import xthreat as xt
        xi, yi = xt._get_cell_indexes(pd.Series([-10.0, 115.0]), pd.Series([-10.0, 78.0]),
                                      self.N, self.M)
        pd.testing.assert_series_equal(xi, pd.Series([0, 1]))
        pd.testing.assert_series_equal(yi, pd.Series([0, 1]))

    def test_get_flat_indexes(self):
        from socceraction_amd import xthreat as xt
        x = pd.Series([0, 105 / 2 - 1, 105 / 2 + 1, 105.0])
        y = pd.Series([0, 68 / 2 + 1, 68 / 2 - 1, 68.0])
        pd.testing.assert_series_equal(xt._get_flat_indexes(x, y, self.N, self.M),
                                       pd.Series([2, 0, 3, 1]))


class TestModelPersistency:
    """reference tests/test_xthreat.py:88-129 (host JSON I/O, NotFittedError)."""

    def test_save_and_load_model(self, tmp_path):
        from socceraction_amd import xthreat as xt
        p = tmp_path / 'xt_model.json'
        model = xt.ExpectedThreat()
        model.xT = np.ones((model.w, model.l))
        model.save_model(str(p))
        assert p.read_text() == json.dumps(model.xT.tolist())
        p.write_text(json.dumps([[0.1, 0.2], [0.1, 0.0]]))
        m2 = xt.load_model(str(p))
        assert (m2.w, m2.l) == (2, 2)
        np.testing.assert_array_equal(m2.xT, [[0.1, 0.2], [0.1, 0.0]])

    def test_save_model_not_fitted_and_exists(self, tmp_path):
        from sklearn.exceptions import NotFittedError

        from socceraction_amd import xthreat as xt
        p = tmp_path / 'xt_model.json'
        model = xt.ExpectedThreat()
        with pytest.raises(NotFittedError):
            model.save_model(str(p))
        p.write_text('create file')
        model.xT = np.ones((model.w, model.l))
        with pytest.raises(ValueError):
            model.save_model(str(p), overwrite=False)
        model.save_model(str(p), overwrite=True)

    def test_init_and_rate_not_fitted(self):
        from sklearn.exceptions import NotFittedError

        from socceraction_amd import xthreat as xt
        m = xt.ExpectedThreat(l=8, w=6, eps=1e-3)
        assert (m.l, m.w, m.eps) == (8, 6, 1e-3) and np.sum(m.xT) == 0
        assert m.transition_matrix is None and len(m.heatmaps) == 0
        with pytest.raises(NotFittedError):
            m.rate(pd.DataFrame({'type_id': [0]}))

    @pytest.mark.parametrize('kind,k', [('cubic', 3), ('quintic', 5)])
    def test_interpolator_spline_kinds(self, kind, k):
        """interpolator(kind='cubic' | 'quintic') (xthreat.py:347-378): interp2d's regular-grid
        spline as scipy < 1.14 computed it -- RectBivariateSpline(kx=ky=k, s=0), sorted query
        axes, out-of-hull points clamped, (len(ys), len(xs)) -- incl. interpolation at the nodes.
        Parity against interp2d itself is unpinned (scipy here no longer has it)."""
        from scipy.interpolate import RectBivariateSpline

        from socceraction_amd import xthreat as xt
        m = xt.ExpectedThreat(l=16, w=12)
        rng = np.random.default_rng(3)
        m.xT = rng.random((12, 16)) * 0.3
        f = m.interpolator(kind)
        cx = np.arange(0.0, 105.0, 105.0 / 16) + 0.5 * 105.0 / 16
        cy = np.arange(0.0, 68.0, 68.0 / 12) + 0.5 * 68.0 / 12
        np.testing.assert_allclose(f(cx, cy), m.xT, rtol=1e-10, atol=1e-12)  # through the nodes
        xs, ys = np.array([104.0, -3.0, 50.2, 7.5]), np.array([30.0, 70.0, 1.0])
        got = f(xs, ys)
        spl = RectBivariateSpline(cx, cy, m.xT.T, kx=k, ky=k, s=0)
        ref = spl(np.clip(np.sort(xs), cx[0], cx[-1]), np.clip(np.sort(ys), cy[0], cy[-1])).T
        assert got.shape == (3, 4)
        np.testing.assert_array_equal(got, ref)
        with pytest.raises(ValueError):
            m.interpolator('nearest')

    def test_interpolate_without_interp2d(self, monkeypatch):
        from socceraction_amd import xthreat as xt
        monkeypatch.setattr(xt, 'interp2d', None)
        with pytest.raises(ImportError, match='Interpolation requires scipy to be installed.'):
            xt.ExpectedThreat().interpolator()


def test_move_filters_on_reference_fixture():
    """reference tests/test_xthreat.py:132-154 (pandas filters)."""
    from socceraction_amd import xthreat as xt
    g = load('spadl', 'fixture')
    df = pd.DataFrame(inputs(g))
    mv = xt.get_move_actions(df)
    assert mv.type_id.isin([0, 21, 1]).all() and len(mv) > 0
    sm = xt.get_successful_move_actions(df)
    assert (sm.result_id == 1).all()


def test_single_hip_runtime_after_load():
    """The library must bind to torch's HIP runtime, never load a second copy."""
    import subprocess
    import sys
    code = ("import socceraction_amd._native as n; n.load_library(); "
            "import os; print(len({l.split()[-1] for l in open('/proc/self/maps') "
            "if 'libamdhip64' in l}))")
    out = subprocess.run([sys.executable, '-c', code], capture_output=True, text=True,
                         check=True, cwd=os.path.dirname(os.path.dirname(__file__)))
    assert out.stdout.strip().splitlines()[-1] == '1'


def test_play_left_to_right_sa_two_argument_form():
    """spadl/utils.py:31-57: rows of the away team are mirrored, home rows unchanged."""
    import pandas as pd
    from socceraction_amd.spadl.utils import play_left_to_right, play_left_to_right_sa
    df = pd.DataFrame({'team_id': [1, 2, 2], 'start_x': [1., 2., 105.], 'end_x': [3., 4., 0.],
                       'start_y': [5., 6., 68.], 'end_y': [7., 8., 0.]})
    out = play_left_to_right_sa(df, 1)
    assert out.start_x.tolist() == [1., 103., 0.] and out.end_x.tolist() == [3., 101., 105.]
    assert out.start_y.tolist() == [5., 62., 0.] and out.end_y.tolist() == [7., 60., 68.]
    assert df.start_x.tolist() == [1., 2., 105.]  # input untouched
    pd.testing.assert_frame_equal(out, play_left_to_right(df.assign(home_team_id=1)).drop(
        columns='home_team_id'))


class _FakeBooster:
    def __init__(self, raw):
        self.raw = raw

    def save_raw(self, fmt):
        assert fmt == 'json'
        return bytearray(json.dumps(self.raw).encode())


class _FakeXGBClassifier:
    """The two members of xgboost.XGBClassifier that TreeEnsemble.from_model reads."""

    def __init__(self, raw, best_iteration=None):
        self._b = _FakeBooster(raw)
        if best_iteration is not None:
            self.best_iteration = best_iteration

    def get_booster(self):
        return self._b


def test_xgb_classifier_keeps_only_the_early_stopping_rounds():
    """After the reference's default fit (early_stopping_rounds=10 with an eval set,
    vaep/base.py:199-235) XGBClassifier.predict_proba evaluates rounds 0..best_iteration only:
    the device model must hold exactly those trees -- from the estimator's attribute or from the
    booster attribute in the JSON dump -- and the full model otherwise."""
    from oracle import tree_oracle as to
    from socceraction_amd import trees
    raw = trees.synthetic_xgboost_json(12, n_trees=30, depth=3, seed=4)
    full = trees.TreeEnsemble.from_model(_FakeXGBClassifier(raw))
    assert full.n_trees == 30
    cut = trees.TreeEnsemble.from_model(_FakeXGBClassifier(raw, best_iteration=19))
    assert cut.n_trees == 20
    hand = dict(raw)
    hand['learner'] = dict(raw['learner'])
    gb = dict(raw['learner']['gradient_booster'])
    gb['model'] = dict(gb['model'], trees=raw['learner']['gradient_booster']['model']['trees'][:20])
    hand['learner']['gradient_booster'] = gb
    ref = trees.TreeEnsemble.from_xgboost_json(hand)
    np.testing.assert_array_equal(cut.nodes, ref.nodes)
    np.testing.assert_array_equal(cut.roots, ref.roots)
    # the booster attribute inside the JSON dump (xgboost stores attributes as strings)
    attr = dict(raw)
    attr['learner'] = dict(raw['learner'], attributes={'best_iteration': '7'})
    assert trees.TreeEnsemble.from_model(_FakeXGBClassifier(attr)).n_trees == 8
    # a raw Booster / dict predicts with every tree (Booster.predict's default range)
    assert trees.TreeEnsemble.from_model(attr).n_trees == 30
    # the dropped rounds change the probabilities (oracle restatement of the prediction rule)
    X = np.random.default_rng(1).normal(0, 30, (50, 12))
    assert not np.array_equal(to.predict_xgboost_json(hand, X), to.predict_xgboost_json(raw, X))


def test_unsupported_model_layouts_fall_back_to_the_host():
    """A model dump this flattening does not know (missing keys, odd values) gives None, so
    VAEP.rate runs the learner's own predict_proba instead of failing."""
    from socceraction_amd import trees
    raw = trees.synthetic_xgboost_json(4, n_trees=2, depth=2, seed=1)
    broken = dict(raw)
    broken['learner'] = dict(raw['learner'])
    broken['learner'].pop('learner_model_param')
    assert trees.TreeEnsemble.from_model(broken) is None
    odd = dict(raw)
    odd['learner'] = dict(raw['learner'], learner_model_param={'base_score': '[5E-1]',
                                                               'num_feature': '4'})
    assert trees.TreeEnsemble.from_model(odd) is None
    assert trees.TreeEnsemble.from_model(object()) is None


def test_bench_launches_one_rank_per_gpu(monkeypatch):
    """bench.py --gpus N outside torch.distributed.run starts the N ranks as a child torchrun
    (never exec) and forwards its exit status; under torchrun a world that is not --gpus is
    refused, so a --gpus 8 run cannot print an N = 1 line."""
    import sys

    import bench
    calls = []

    class _Done:
        returncode = 3

    def fake_run(cmd, env):
        calls.append((cmd, env))
        return _Done()
    assert bench.launch_ranks(2, ['--gpus', '2', '--steps', '3'], run=fake_run) == 3
    cmd, env = calls[0]
    assert cmd[:4] == [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1']
    assert '--nproc-per-node=2' in cmd and cmd[cmd.index('--master-addr') + 1] == '127.0.0.1'
    assert cmd[-4:] == ['--gpus', '2', '--steps', '3'] and cmd[-5].endswith('bench.py')
    assert env['MASTER_ADDR'] == '127.0.0.1' and 'HSA_ENABLE_IPC_MODE_LEGACY' in env
    monkeypatch.delenv('WORLD_SIZE', raising=False)
    monkeypatch.setattr(bench, 'launch_ranks', lambda n, argv: 5 if n == 2 else 0)
    monkeypatch.setattr(sys, 'argv', ['bench.py', '--gpus', '2', '--steps', '1'])
    with pytest.raises(SystemExit) as e:
        bench.main()
    assert e.value.code == 5
    monkeypatch.setenv('WORLD_SIZE', '4')
    monkeypatch.setattr(sys, 'argv', ['bench.py', '--gpus', '2'])
    with pytest.raises(SystemExit) as e:
        bench.main()
    assert e.value.code == 2
    monkeypatch.setenv('WORLD_SIZE', '1')
    monkeypatch.setattr(sys, 'argv', ['bench.py', '--gpus', '1'])
    bench.check_world(1)  # the driver's N = 1 line under a 1-rank torchrun


def _eval_staged_layout(lay, roots, depth, slot_feature, X, f32, le, base):
    """numpy restatement of sa_tree_predict_staged over the host-built layout: condition bits
    per row, then every tree walked `depth` levels over {condition, left | right << 16}."""
    A = np.float32 if f32 else np.float64
    nrow = X.shape[0]
    nb = len(lay['bool_cols'])
    bits = np.zeros((1 + nb + len(lay['num_slots']), nrow), bool)
    for i, col in enumerate(lay['bool_cols']):
        bits[1 + i] = X[:, slot_feature[int(col)]] != 0
    for c, (sl, thr, dl) in enumerate(zip(lay['num_slots'], lay['num_thr'], lay['num_dl'])):
        x = X[:, slot_feature[int(sl)]].astype(A)
        left = np.where(np.isnan(x), dl == 1, (x <= thr) if le else (x < thr))
        bits[1 + nb + c] = ~left
    cond = (lay['nodes'] & 0xFFFF).astype(np.int64)
    first = (lay['nodes'] >> 16).astype(np.int64)
    m = np.full(nrow, A(base), A)
    rows = np.arange(nrow)
    for t, r in enumerate(lay['roots']):
        k = np.full(nrow, int(r), np.int64)
        for _ in range(int(depth[t])):
            k = first[k] + bits[cond[k], rows]
        m = (m + lay['leaf'][k].astype(A)).astype(A)
    return (A(1) / (A(1) + np.exp(-m))).astype(A)


@pytest.mark.parametrize('depth', [1, 2, 3, 5])
def test_staged_layout_restates_the_walk(depth):
    """The condition layout of sa_tree_predict_staged (host-built, trees.staged_layout) sends
    every row to the walk's leaf: xgboost-shaped models over bool and numeric features with NaN,
    bool thresholds that send 0 and 1 the same way (constant splits) or 0 right (swapped
    children), repeated numeric thresholds (one condition) and unbalanced trees."""
    from oracle import tree_oracle as to
    from socceraction_amd import trees
    rng = np.random.default_rng(depth)
    nf = 40
    kinds = ['b' if f % 3 else 'f' for f in range(nf)]
    model = trees.synthetic_xgboost_json(nf, n_trees=30, depth=depth, seed=depth, feature_kinds=kinds)
    tl = model['learner']['gradient_booster']['model']['trees']
    for t in tl[::4]:  # the root's left child becomes a leaf: an unbalanced tree
        if depth > 1:
            t['left_children'][1] = -1
            t['right_children'][1] = -1
    for q, t in enumerate(tl[1::5]):  # bool thresholds outside (0, 1]
        for k, f in enumerate(t['split_indices']):
            if kinds[f] == 'b' and t['left_children'][k] >= 0:
                t['split_conditions'][k] = (1.5, -0.5)[(k + q) % 2]
    for t in tl[2::6]:  # a numeric split repeated elsewhere: one shared condition
        t['split_indices'][0], t['split_conditions'][0] = 0, 3.0
    X = np.where(np.array(kinds) == 'b', rng.random((700, nf)) < 0.3,
                 rng.normal(0, 30, (700, nf))).astype(np.float64)
    X[rng.random(X.shape) < 0.05 * (np.array(kinds) == 'f')] = np.nan
    te = trees.TreeEnsemble.from_xgboost_json(model)
    # block layout: bool feature f -> bool column f, numeric -> f64 column f
    slots = np.array([f if k == 'b' else (1 << 24 | f) for f, k in enumerate(kinds)], np.int32)
    slot_feature = {int(s_) if (int(s_) >> 24) else int(s_) & 0xFFFFFF: f for f, s_ in enumerate(slots)}
    lay = te.staged_layout(slots)
    lay.update(lay['models'][0])
    assert len(lay['nodes']) <= len(te.nodes) and lay['num_slots'].tolist() == sorted(lay['num_slots'])
    got = _eval_staged_layout(lay, te.roots, te.depths(), slot_feature, X, True, False, te.base_margin)
    with np.errstate(over='ignore'):
        np.testing.assert_array_equal(got, to.predict_xgboost_json(model, X))


def test_phase_times_on_the_host():
    """shard.PhaseTimes (the multi-rank fit's per-phase timer): wall clock per phase on the
    host, summed over repeats; _phase is a no-op without a timer in the stats."""
    import time as _t

    from socceraction_amd import shard
    pt = shard.PhaseTimes('cpu')
    for _ in range(2):
        with shard._phase({'timer': pt}, 'a'):
            _t.sleep(0.01)
    with shard._phase({'timer': pt}, 'b'):
        pass
    with shard._phase(None, 'c'), shard._phase({}, 'd'):
        pass
    ms = pt.ms()
    assert set(ms) == {'a', 'b'} and ms['a'] >= 19 and ms['b'] >= 0


def test_pipeline_chunks_cut_at_games_on_aligned_rows():
    """socceraction_amd.pipeline._chunks: game-aligned chunks covering every game once, of about
    the asked size, each cut at a row that is a multiple of 4 when one lies within reach (the
    DMA's fast path), else at the plain game boundary."""
    from socceraction_amd import pipeline
    rng = np.random.default_rng(3)
    sizes = rng.integers(1000, 2200, 400)
    off = np.concatenate([[0], np.cumsum(sizes)])
    cuts = pipeline._chunks(off, 50_000)
    assert cuts[0][0] == 0 and cuts[-1][1] == len(sizes)
    assert all(a[1] == b[0] for a, b in zip(cuts, cuts[1:]))
    assert all(off[s1] % 4 == 0 for _, s1 in cuts[:-1])
    want = [12_500, 25_000] + [50_000] * len(cuts)  # the ramp: chunk_rows / 4, / 2, then chunk_rows
    assert all(abs((off[s1] - off[s0]) - w) < 10_000 for (s0, s1), w in zip(cuts[:-1], want))
    flat = pipeline._chunks(off, 50_000, ramp=())
    assert all(abs((off[s1] - off[s0]) - 50_000) < 10_000 for s0, s1 in flat[:-1])
    odd = np.concatenate([[0], np.cumsum(np.full(50, 1001))])  # no row but 0 mod 4 every 4 games
    cuts = pipeline._chunks(odd, 5000, look=0)
    assert cuts[-1][1] == 50 and all(a[1] == b[0] for a, b in zip(cuts, cuts[1:]))
