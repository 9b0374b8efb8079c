"""Per-game feature / label stores (socceraction_amd/store.py; the notebooks' ``X.to_hdf(path,
f"game_{game_id}")`` / ``pd.read_hdf``).

CPU: the store itself (put / get / keys / modes / row ranges spanning row groups). GPU: the
device bitmaps equal numpy's little-endian packbits, and the batched writers store, per game,
exactly the DataFrames ``compute_features`` / ``compute_labels`` return.
"""
import numpy as np
import pandas as pd
import pytest

pa = pytest.importorskip('pyarrow')


def _frame(n, seed):
    rng = np.random.default_rng(seed)
    return pd.DataFrame({'type_pass_a0': rng.random(n) < 0.5,
                         'start_x_a0': rng.random(n) * 105,
                         'period_id_a0': rng.integers(1, 3, n).astype(np.int64),
                         'angle': np.where(rng.random(n) < 0.1, np.nan, rng.random(n))})


def test_store_put_get_roundtrip(tmp_path):
    from socceraction_amd.store import FeatureStore, read_store
    p = str(tmp_path / 'features')
    frames = {g: _frame(50 + g, g) for g in range(5)}
    with FeatureStore(p, mode='w') as st:
        for g, df in frames.items():
            st.put(f'game_{g}', df)
        st['extra'] = frames[0]
        assert 'game_3' in st and '/game_3' in st and len(st) == 6
    with FeatureStore(p, mode='r') as st:
        assert sorted(st.keys()) == sorted(['/extra'] + [f'/game_{g}' for g in range(5)])
        for g, df in frames.items():
            pd.testing.assert_frame_equal(st.get(f'/game_{g}'), df)
        with pytest.raises(KeyError):
            st.get('game_99')
        with pytest.raises(ValueError):
            st.put('x', frames[0])
    pd.testing.assert_frame_equal(read_store(p, 'game_2'), frames[2])
    with pytest.raises(FileNotFoundError):
        FeatureStore(str(tmp_path / 'missing'), mode='r')


def test_store_put_many_row_ranges(tmp_path, monkeypatch):
    """Keys spanning several row groups and part files come back exactly."""
    from socceraction_amd import store as S
    monkeypatch.setattr(S, 'ROW_GROUP_ROWS', 64)
    df = _frame(1000, 7)
    off = np.array([0, 10, 10, 200, 333, 640, 1000])
    keys = [f'game_{i}' for i in range(len(off) - 1)]
    p = str(tmp_path / 'many')
    with S.FeatureStore(p, mode='w', compression='snappy') as st:
        st.put_many(pa.Table.from_pandas(df, preserve_index=False), keys, off, parts=3)
    with S.FeatureStore(p, mode='a') as st:
        for i, k in enumerate(keys):
            got = st.get(k)
            exp = df.iloc[off[i]:off[i + 1]].reset_index(drop=True)
            pd.testing.assert_frame_equal(got, exp)
        with pytest.raises(ValueError):
            st.put_many(pa.Table.from_pandas(df), keys, off[:-1])


def _packbits_ref(b: np.ndarray, n: int) -> np.ndarray:
    return np.packbits(b[:n].astype(bool), bitorder='little')


@pytest.mark.gpu
def test_pack_bits_matches_numpy():
    torch = pytest.importorskip('torch')
    from socceraction_amd import _native, store
    _native.load_library()
    rng = np.random.default_rng(3)
    for n, R, tiles in ((1, 16, 1), (37, 48, 1), (5000, 1024, 5), (1000, 1008, 1)):
        C = 7
        blk = (rng.random((tiles, C, R)) < 0.3).astype(np.uint8)
        bits = store.pack_bits(torch.from_numpy(blk).cuda(), R, n).cpu().numpy()
        cols = blk.transpose(1, 0, 2).reshape(C, -1)
        for c in range(C):
            ref = _packbits_ref(cols[c], n)
            np.testing.assert_array_equal(bits[c, :len(ref)], ref, err_msg=f'n={n} c={c}')


@pytest.mark.gpu
def test_store_features_and_labels_batch(tmp_path):
    """Device writers == compute_features / compute_labels per game (values, names, dtypes)."""
    pytest.importorskip('torch')
    from socceraction_amd import _native, store, synthetic
    import socceraction_amd.vaep as vaep
    _native.load_library()
    d = synthetic.spadl_games(5, seed=31)
    actions = synthetic.to_frame(d)
    games = synthetic.games_frame(d)
    model = vaep.VAEP()
    fx, lx = str(tmp_path / 'features'), str(tmp_path / 'labels')
    with store.FeatureStore(fx, mode='w') as st:
        assert store.store_features_batch(model, games, actions, st, parts=3) == len(actions)
    with store.FeatureStore(lx, mode='w') as st:
        store.store_labels_batch(model, games, actions, st)
    for g in games.itertuples():
        ga = actions[actions.game_id == g.game_id].reset_index(drop=True)
        X = model.compute_features(g, ga)
        Y = model.compute_labels(g, ga)
        pd.testing.assert_frame_equal(store.read_store(fx, f'game_{g.game_id}'), X)
        pd.testing.assert_frame_equal(store.read_store(lx, f'game_{g.game_id}'), Y)
