"""Per-game feature and label stores.

The reference's notebooks write one HDF5 key per game (public-notebooks/
2-compute-features-and-labels.ipynb: ``X.to_hdf(features_h5, f"game_{game.game_id}")``, the
labels likewise) and read them back per game (3-estimate-scoring-and-conceding-probabilities
.ipynb: ``pd.read_hdf(features_h5, f"game_{game_id}")``). PyTables is not installed in this
image, so the store here is Parquet (pyarrow): :class:`FeatureStore` keeps the subset of
``pandas.HDFStore`` those notebooks use (``put`` / ``get`` / ``[]`` / ``keys`` / ``in`` /
``close``, context manager) over a directory of Parquet part files plus a JSON index of each
key's row range.

The batched writers (:func:`store_features_batch`, :func:`store_labels_batch`) never build a
DataFrame: the feature blocks leave HBM as Arrow columns -- bool columns as bitmaps packed on
the device (``sa_pack_bits``, 1/8 of the bytes over PCIe, no host packing pass), f64 / i64
columns as zero-copy views of the pinned host copy -- and the games are written as several
part files in parallel (pyarrow releases the GIL while encoding).
"""
from __future__ import annotations

import ctypes
import json
import os
import shutil
from concurrent.futures import ThreadPoolExecutor
from typing import Dict, List, Optional, Sequence

import numpy as np
import pandas as pd
import torch

from . import _native
from .batch import ActionBatch, stream_handle

try:
    import pyarrow as pa
    import pyarrow.parquet as pq
except ImportError:  # pragma: no cover - pyarrow ships with this image
    pa = pq = None

ROW_GROUP_ROWS = 1 << 16
INDEX = 'index.json'


def _need_arrow():
    if pa is None:
        raise ImportError('the feature store needs pyarrow')


# ------------------------------------------------------------------ device -> Arrow
def pack_bits(block: torch.Tensor, tile_rows: int, n: int) -> torch.Tensor:
    """Arrow bitmaps of a tiled uint8 block ``[tiles, C, tile_rows]`` (or ``[C, tile_rows]``):
    a device tensor ``[C, stride]`` of bytes, LSB first, rows >= n zero."""
    if block.dim() == 2:
        block = block.unsqueeze(0)
    C = block.shape[1]
    stride = max(64, -(-2 * (-(-n // 16)) // 64) * 64)
    bits = torch.empty((C, stride), dtype=torch.uint8, device=block.device)
    b = _native.SaBlock()
    b.data = block.data_ptr()
    b.n_cols = C
    b.tile_rows = int(tile_rows)
    _native.check(_native.lib().sa_pack_bits(ctypes.byref(b), int(n), bits.data_ptr(), stride,
                                             stream_handle()))
    return bits


def _to_pinned(t: torch.Tensor) -> torch.Tensor:
    h = torch.empty(t.shape, dtype=t.dtype, pin_memory=True)
    h.copy_(t, non_blocking=True)
    return h


def _bool_array(bitmap_row: np.ndarray, n: int):
    return pa.Array.from_buffers(pa.bool_(), n, [None, pa.py_buffer(bitmap_row)])


def features_to_arrow(blocks) -> 'pa.Table':
    """The feature blocks (``ops.FeatureBlocks``) as an Arrow table with the reference's column
    names and order (bool / float64 / int64, like ``compute_features``)."""
    _need_arrow()
    n = blocks.n
    plan = blocks.plan
    bits = pack_bits(blocks.bool_block, blocks.Rb, n) if plan.n_bool else None
    hb = _to_pinned(bits) if bits is not None else None
    hosts = {}
    for k in 'fi':
        t = blocks._blk(k)
        src = t[0] if t.shape[0] == 1 else t.permute(1, 0, 2).reshape(t.shape[1], -1)
        hosts[k] = _to_pinned(src)
    torch.cuda.current_stream().synchronize()
    hbn = hb.numpy() if hb is not None else None
    hn = {k: v.numpy() for k, v in hosts.items()}
    arrays = []
    for _, kind, col in plan.order:
        if kind == 'b':
            arrays.append(_bool_array(hbn[col], n))
        else:
            arrays.append(pa.array(hn[kind][col, :n]))
    return pa.Table.from_arrays(arrays, names=list(plan.names))


def labels_to_arrow(lab, columns: Sequence[str] = ('scores', 'concedes')) -> 'pa.Table':
    """Label columns (``ops.LabelBlocks`` fields) as an Arrow table of bools."""
    _need_arrow()
    n = lab.n
    bits = [pack_bits(getattr(lab, c).view(1, -1), getattr(lab, c).numel(), n) for c in columns]
    hosts = [_to_pinned(b) for b in bits]
    torch.cuda.current_stream().synchronize()
    return pa.Table.from_arrays([_bool_array(h.numpy()[0], n) for h in hosts],
                                names=list(columns))


# ------------------------------------------------------------------ the store
class FeatureStore:
    """A per-key Parquet store with the ``pandas.HDFStore`` calls the notebooks use.

    ``mode``: 'a' (create or append, default), 'w' (truncate), 'r' (read only). Keys are stored
    without the leading '/'; :meth:`keys` returns them with it, like ``HDFStore.keys()``.
    ``compression``: any Parquet codec pyarrow knows ('snappy', 'lz4', 'zstd', 'none', ...).
    """

    def __init__(self, path: str, mode: str = 'a', compression: str = 'lz4') -> None:
        _need_arrow()
        if mode not in ('a', 'w', 'r'):
            raise ValueError(f'mode must be one of a, w, r (got {mode!r})')
        self.path = path
        self.mode = mode
        self.compression = compression
        if mode == 'w' and os.path.exists(path):
            shutil.rmtree(path)
        if mode == 'r' and not os.path.exists(os.path.join(path, INDEX)):
            raise FileNotFoundError(f'no feature store at {path}')
        os.makedirs(path, exist_ok=True)
        self._index: Dict[str, List] = {}
        self._parts: List[str] = []
        ip = os.path.join(path, INDEX)
        if os.path.exists(ip):
            with open(ip) as f:
                meta = json.load(f)
            self._parts = list(meta['parts'])
            self._index = {k: list(v) for k, v in meta['keys'].items()}
        self._files: Dict[int, 'pq.ParquetFile'] = {}
        self._dirty = False

    # -- context manager / lifetime
    def __enter__(self) -> 'FeatureStore':
        return self

    def __exit__(self, *exc) -> None:
        self.close()

    def flush(self) -> None:
        if not self._dirty:
            return
        tmp = os.path.join(self.path, INDEX + '.tmp')
        with open(tmp, 'w') as f:
            json.dump({'parts': self._parts, 'keys': self._index}, f)
        os.replace(tmp, os.path.join(self.path, INDEX))
        self._dirty = False

    def close(self) -> None:
        if self.mode != 'r':
            self.flush()
        self._files.clear()

    # -- keys
    @staticmethod
    def _norm(key: str) -> str:
        return key.lstrip('/')

    def keys(self) -> List[str]:
        return ['/' + k for k in self._index]

    def __contains__(self, key: str) -> bool:
        return self._norm(key) in self._index

    def __len__(self) -> int:
        return len(self._index)

    # -- writing
    def _check_writable(self) -> None:
        if self.mode == 'r':
            raise ValueError('the store is open read-only')

    def _new_part(self) -> int:
        i = len(self._parts)
        self._parts.append(f'part-{i:05d}.parquet')
        return i

    def _write_part(self, part: int, table: 'pa.Table') -> None:
        pq.write_table(table, os.path.join(self.path, self._parts[part]),
                       row_group_size=ROW_GROUP_ROWS, compression=self.compression,
                       use_dictionary=False, write_statistics=False)

    def put(self, key: str, value) -> None:
        """Store one DataFrame (or Arrow table) under ``key`` (replacing an earlier one)."""
        self._check_writable()
        table = value if isinstance(value, pa.Table) else pa.Table.from_pandas(value)
        part = self._new_part()
        self._write_part(part, table)
        self._index[self._norm(key)] = [part, 0, table.num_rows]
        self._dirty = True

    def put_many(self, table: 'pa.Table', keys: Sequence[str], offsets: Sequence[int],
                 parts: int = 8) -> None:
        """Store rows ``[offsets[i], offsets[i + 1])`` of ``table`` under ``keys[i]``, as up to
        ``parts`` part files of whole keys written in parallel."""
        self._check_writable()
        off = np.asarray(offsets, dtype=np.int64)
        if len(off) != len(keys) + 1 or off[0] != 0 or off[-1] != table.num_rows:
            raise ValueError('offsets must have len(keys) + 1 entries from 0 to the row count')
        nk = len(keys)
        if nk == 0:
            return
        parts = max(1, min(int(parts), nk))
        # split the keys into contiguous chunks of about equal row counts
        cuts = np.searchsorted(off, np.linspace(0, off[-1], parts + 1)[1:-1])
        bounds = [0] + sorted(set(int(c) for c in cuts if 0 < c < nk)) + [nk]
        jobs = []
        for a, b in zip(bounds[:-1], bounds[1:]):
            part = self._new_part()
            jobs.append((part, a, b))
            for i in range(a, b):
                self._index[self._norm(keys[i])] = [part, int(off[i] - off[a]),
                                                    int(off[i + 1] - off[i])]

        def write(job):
            part, a, b = job
            self._write_part(part, table.slice(int(off[a]), int(off[b] - off[a])))

        with ThreadPoolExecutor(max_workers=len(jobs)) as ex:
            list(ex.map(write, jobs))
        self._dirty = True

    # -- reading
    def _file(self, part: int) -> 'pq.ParquetFile':
        f = self._files.get(part)
        if f is None:
            f = pq.ParquetFile(os.path.join(self.path, self._parts[part]))
            self._files[part] = f
        return f

    def get_table(self, key: str) -> 'pa.Table':
        k = self._norm(key)
        if k not in self._index:
            raise KeyError(f'No object named {key} in the file')
        part, start, length = self._index[k]
        f = self._file(part)
        md = f.metadata
        groups, first, row = [], None, 0
        for g in range(md.num_row_groups):
            m = md.row_group(g).num_rows
            if row + m > start and row < start + length:
                groups.append(g)
                if first is None:
                    first = row
            row += m
        if not groups:
            return f.schema_arrow.empty_table()
        t = f.read_row_groups(groups)
        return t.slice(start - first, length)

    def get(self, key: str) -> pd.DataFrame:
        return self.get_table(key).to_pandas()

    __getitem__ = get

    def __setitem__(self, key: str, value) -> None:
        self.put(key, value)


def read_store(path: str, key: str) -> pd.DataFrame:
    """``pd.read_hdf(path, key)`` for a :class:`FeatureStore`."""
    with FeatureStore(path, mode='r') as st:
        return st.get(key)


# ------------------------------------------------------------------ batched writers
def _games_batch(model, games: pd.DataFrame, actions: pd.DataFrame):
    home_of = games.set_index('game_id')['home_team_id']
    ab = ActionBatch.from_frame(actions, atomic=model._atomic, home_team_id=home_of,
                                segments='game')
    off = ab.cols['seg_off'].cpu().numpy()
    gids = actions['game_id'].to_numpy()[off[:-1]] if len(actions) else []
    return ab, off, gids


def store_features_batch(model, games: pd.DataFrame, actions: pd.DataFrame,
                         store: FeatureStore, key: str = 'game_{game_id}',
                         parts: int = 8) -> int:
    """``X = model.compute_features(game, actions_of_game); X.to_hdf(store, key)`` for every
    game of ``actions`` (contiguous per game) in one launch; returns the rows written.
    Games whose transformers the device does not know go through ``compute_features_batch``."""
    from . import ops
    known, unknown = model._split_xfns()
    ab, off, gids = _games_batch(model, games, actions)
    if unknown or not known:
        table = pa.Table.from_pandas(model.compute_features_batch(games, actions),
                                     preserve_index=False)
    else:
        table = features_to_arrow(ops.features(ab, known, model.nb_prev_actions))
    store.put_many(table, [key.format(game_id=g) for g in gids], off, parts=parts)
    return table.num_rows


def store_labels_batch(model, games: pd.DataFrame, actions: pd.DataFrame, store: FeatureStore,
                       key: str = 'game_{game_id}', parts: int = 8) -> int:
    """``Y = model.compute_labels(game, actions_of_game); Y.to_hdf(store, key)`` for every game,
    in one launch (device labels packed as bitmaps when the label functions are the
    reference's)."""
    from . import ops
    lab = model._lab
    known = {lab.scores: 'scores', lab.concedes: 'concedes', lab.goal_from_shot: 'goal_from_shot'}
    ab, off, gids = _games_batch(model, games, actions)
    if len(actions) and all(f in known for f in model.yfns):
        lb = ops.labels(ab)
        cols = [known[f] for f in model.yfns]
        table = labels_to_arrow(lb, cols)
        if model._atomic and 'goal_from_shot' in cols:
            table = table.rename_columns(['goal' if c == 'goal_from_shot' else c for c in cols])
    else:
        table = pa.Table.from_pandas(model.compute_labels_batch(games, actions),
                                     preserve_index=False)
    store.put_many(table, [key.format(game_id=g) for g in gids], off, parts=parts)
    return table.num_rows


__all__ = ['FeatureStore', 'read_store', 'features_to_arrow', 'labels_to_arrow', 'pack_bits',
           'store_features_batch', 'store_labels_batch']
