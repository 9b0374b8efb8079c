"""SPADL -> Atomic-SPADL conversion on MI355X (drop-in for ``socceraction.atomic.spadl.base``).

``convert_to_atomic`` (reference atomic/spadl/base.py:15-35) runs as one device expansion:
the SPADL frame is flattened once into HBM columns (ids as int32 equality codes), one
kernel counts how many Atomic-SPADL rows each input row becomes, one scans those counts and
one writes the rows (``sa_atomic_count`` / ``sa_atomic_emit``, socceraction_amd/csrc/
sa_atomic.hip). The host only factorises the id columns, decodes the output codes and
builds the DataFrame. The reference's four concat + sort passes collapse into this single
expansion because every inserted row lands directly after the row that produced it (see
the kernel's header comment); the numpy restatement of the four passes in
``oracle/atomic_convert_oracle.py`` and the reference's own outputs
(``tests/golden/convert_*.npz``) are the parity checks.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass
from typing import Dict, Optional, Tuple

import numpy as np
import pandas as pd
import torch

from ... import _native

_REQUIRED = ('game_id', 'original_event_id', 'action_id', 'period_id', 'time_seconds',
             'team_id', 'player_id', 'start_x', 'start_y', 'end_x', 'end_y', 'type_id',
             'result_id', 'bodypart_id')
_OUT = ('game_id', 'original_event_id', 'action_id', 'period_id', 'time_seconds', 'team_id',
        'player_id', 'x', 'y', 'dx', 'dy', 'type_id', 'bodypart_id')
_ALIGN = 256


def device():
    from ...batch import device as _device  # lazy: batch imports this package's config
    return _device()


def stream_handle() -> int:
    return torch.cuda.current_stream().cuda_stream


def _pack(arrays: Dict[str, np.ndarray], dev) -> Tuple[torch.Tensor, Dict[str, torch.Tensor]]:
    """One device allocation holding every array at 256-byte aligned offsets (one H2D copy)."""
    offs, total = {}, 0
    for k, a in arrays.items():
        offs[k] = total
        total += (max(a.nbytes, 16) + _ALIGN - 1) // _ALIGN * _ALIGN
    host = np.zeros(max(total, _ALIGN), dtype=np.uint8)
    for k, a in arrays.items():
        host[offs[k]:offs[k] + a.nbytes] = np.ascontiguousarray(a).view(np.uint8).reshape(-1)
    buf = torch.from_numpy(host).to(dev)
    views = {k: buf[offs[k]:offs[k] + max(a.nbytes, a.itemsize)].view(torch.from_numpy(a[:0]).dtype)
             for k, a in arrays.items()}
    return buf, views


def _alloc(spec: Dict[str, type], n: int, dev) -> Tuple[torch.Tensor, Dict[str, torch.Tensor]]:
    """One uninitialised device allocation carved into length-n columns (256-B aligned)."""
    offs, total = {}, 0
    for k, dt in spec.items():
        offs[k] = total
        total += (max(n * np.dtype(dt).itemsize, 16) + _ALIGN - 1) // _ALIGN * _ALIGN
    buf = torch.empty(total, dtype=torch.uint8, device=dev)
    tdt = {np.float64: torch.float64, np.int32: torch.int32, np.uint8: torch.uint8}
    cols = {k: buf[offs[k]:offs[k] + n * np.dtype(dt).itemsize].view(tdt[dt])
            for k, dt in spec.items()}
    return buf, cols


def _codes(values, sort: bool = False) -> Tuple[np.ndarray, pd.Index]:
    codes, uniques = pd.factorize(pd.Series(values), sort=sort, use_na_sentinel=True)
    return codes.astype(np.int32), pd.Index(uniques)


def _ids(df: pd.DataFrame, col: str, lo: int, hi: int) -> np.ndarray:
    v = df[col].to_numpy()
    if v.dtype.kind == 'f':
        if np.isnan(v).any() or (v != np.floor(v)).any():
            raise ValueError(f'{col} must hold integers')
    if len(v) and (v.min() < lo or v.max() > hi):
        raise ValueError(f'{col} values must lie in [{lo}, {hi}] (SPADL schema isin check)')
    return v.astype(np.uint8)


def _key_layout(g: np.ndarray, per: np.ndarray, aid) -> Tuple[Optional[np.ndarray], bool]:
    """(order, general) for the rows' (game, period, action_id) keys.  ``order`` is None when the
    rows already are in that order, else the stable sort permutation the reference's
    sort_values applies (base.py:110).  ``general`` is True when the single expansion's layout
    -- every row _extra_from_passes inserts (key action_id + 0.1, base.py:82) sorts directly
    after its parent -- may not be the reference's order: keys that repeat, or two consecutive
    keys of one game and period no more than 0.1 apart.  Such frames take the general path
    (the first pass on its own, placed by the host's stable lexsort; ``convert_device``)."""
    n = len(g)
    if n < 2:
        return None, False
    aid = np.asarray(aid)
    if aid.dtype.kind not in 'iuf':
        raise ValueError('action_id must be numeric')

    def tight(gg, pp, aa):  # any consecutive pair of one game and period with a + 0.1 >= next
        same = (np.diff(gg.astype(np.int64)) == 0) & (np.diff(pp.astype(np.int64)) == 0)
        a = aa.astype(np.float64)
        return bool((same & ~(a[:-1] + 0.1 < a[1:])).any())

    def strictly_increasing(gg, pp, aa):
        d_g, d_p, d_a = np.diff(gg.astype(np.int64)), np.diff(pp.astype(np.int64)), np.diff(aa)
        return bool(((d_g > 0) | ((d_g == 0) & ((d_p > 0) | ((d_p == 0) & (d_a > 0))))).all())

    if strictly_increasing(g, per, aid):
        return None, tight(g, per, aid)
    order = np.lexsort((aid, per, g)).astype(np.int64)
    return order, tight(g[order], per[order], aid[order])


@dataclass
class SpadlFrame:
    """A SPADL frame in HBM (``sa_spadl_frame``) plus the host tables decoding its codes."""

    n: int
    buffer: torch.Tensor
    cols: Dict[str, torch.Tensor]
    uniques: Dict[str, pd.Index]
    dtypes: Dict[str, np.dtype]
    # general path (see _key_layout): the host keys (game codes, period, action_id as f64) the
    # first pass sorts on; None on the single-expansion path
    keys: Optional[Tuple[np.ndarray, np.ndarray, np.ndarray]] = None
    # True for the first pass's sorted output (sa_atomic_passes_emit): converted without it
    after_passes: bool = False

    @classmethod
    def from_frame(cls, actions: pd.DataFrame, dev=None, sort: bool = True) -> 'SpadlFrame':
        """``sort=False``: rows stay in input order (no ``order`` permutation)."""
        for c in _REQUIRED:
            if c not in actions.columns:
                raise AttributeError(f"'DataFrame' object has no attribute '{c}'")
        dev = dev or device()
        n = len(actions)
        g, gu = _codes(actions['game_id'].to_numpy(), sort=True)  # order-preserving codes
        if (g < 0).any():
            raise ValueError('game_id contains missing values')
        t, tu = _codes(actions['team_id'].to_numpy())
        p, pu = _codes(actions['player_id'].to_numpy())
        e, eu = _codes(actions['original_event_id'].to_numpy())  # missing -> -1
        per = _ids(actions, 'period_id', 1, 5)
        arrays = {
            'time_seconds': actions['time_seconds'].to_numpy(np.float64),
            'start_x': actions['start_x'].to_numpy(np.float64),
            'start_y': actions['start_y'].to_numpy(np.float64),
            'end_x': actions['end_x'].to_numpy(np.float64),
            'end_y': actions['end_y'].to_numpy(np.float64),
            'game': g, 'team': t, 'player': p, 'event': e,
            'period_id': per,
            'type_id': _ids(actions, 'type_id', 0, 22),
            'result_id': _ids(actions, 'result_id', 0, 5),
            'bodypart_id': _ids(actions, 'bodypart_id', 0, 3),
        }
        aid = actions['action_id'].to_numpy()
        order, general = _key_layout(g, per, aid) if sort else (None, False)
        if order is not None and not general:
            arrays['order'] = order
        buf, views = _pack(arrays, dev)
        dtypes = {c: actions[c].dtype for c in ('game_id', 'team_id', 'player_id')}
        keys = (g, per, aid.astype(np.float64)) if general else None
        return cls(n, buf, views, {'game': gu, 'team': tu, 'player': pu, 'event': eu}, dtypes, keys)

    @classmethod
    def from_columns(cls, d: Dict[str, np.ndarray], dev=None) -> 'SpadlFrame':
        """From the flat, game-sorted numpy columns of :mod:`socceraction_amd.synthetic`
        (integer ids; no original_event_id: every event code is missing)."""
        dev = dev or device()
        n = len(d['type_id'])
        g, gu = _codes(d['game_id'], sort=True)
        t, tu = _codes(d['team_id'])
        player = d['player_id'] if 'player_id' in d else \
            (np.asarray(d['team_id']) * 100 + np.asarray(d['pos']) % 11)
        p, pu = _codes(player)
        arrays = {'time_seconds': np.asarray(d['time_seconds'], np.float64)}
        for c in ('start_x', 'start_y', 'end_x', 'end_y'):
            arrays[c] = np.asarray(d[c], np.float64)
        arrays.update(game=g, team=t, player=p, event=np.full(n, -1, np.int32))
        for c in ('period_id', 'type_id', 'result_id', 'bodypart_id'):
            arrays[c] = np.asarray(d[c]).astype(np.uint8)
        aid = np.asarray(d['pos'] if 'pos' in d else np.arange(n))
        order, general = _key_layout(g, arrays['period_id'], aid)
        if order is not None and not general:
            arrays['order'] = order
        buf, views = _pack(arrays, dev)
        dtypes = {'game_id': np.dtype(np.int64), 'team_id': np.dtype(np.int64),
                  'player_id': np.dtype(np.int64)}
        keys = (g, arrays['period_id'], aid.astype(np.float64)) if general else None
        return cls(n, buf, views, {'game': gu, 'team': tu, 'player': pu,
                                   'event': pd.Index([])}, dtypes, keys)

    def struct(self) -> _native.SaSpadlFrame:
        s = _native.SaSpadlFrame()
        s.n = self.n
        for name in ('time_seconds', 'start_x', 'start_y', 'end_x', 'end_y', 'game', 'team',
                     'player', 'event', 'period_id', 'type_id', 'result_id', 'bodypart_id'):
            setattr(s, name, self.cols[name].data_ptr())
        s.order = self.cols['order'].data_ptr() if 'order' in self.cols else None
        return s


@dataclass
class AtomicColumns:
    """Atomic-SPADL rows in HBM (``sa_atomic_frame``), codes as in the source SpadlFrame."""

    n: int
    buffer: torch.Tensor
    cols: Dict[str, torch.Tensor]

    def to_batch(self, frame: 'SpadlFrame', home_team_ids=None):
        """The rows as an atomic :class:`~socceraction_amd.batch.ActionBatch` (one segment per
        game, no copy), ready for the Atomic-VAEP feature / label / formula kernels.
        ``home_team_ids``: one home team id per game, in game_id order (None: no flip)."""
        from ...batch import ActionBatch
        dev = self.buffer.device
        G = len(frame.uniques['game'])
        seg_off = torch.empty(G + 1, dtype=torch.int64, device=dev)
        _native.check(_native.lib().sa_segment_offsets(self.cols['game'].data_ptr(), self.n, G,
                                                       seg_off.data_ptr(), stream_handle()))
        home = None
        if home_team_ids is not None:
            hc = frame.uniques['team'].get_indexer(pd.Index(home_team_ids)).astype(np.int32)
            home = torch.from_numpy(hc).to(dev)
        c = self.cols
        cols = {'c0': c['x'], 'c1': c['y'], 'c2': c['dx'], 'c3': c['dy'],
                'time_seconds': c['time_seconds'], 'team': c['team'], 'type_id': c['type_id'],
                'bodypart_id': c['bodypart_id'], 'period_id': c['period_id']}
        return ActionBatch.from_device(cols, self.n, seg_off, home, atomic=True)

    def struct(self) -> _native.SaAtomicFrame:
        s = _native.SaAtomicFrame()
        for name in ('time_seconds', 'x', 'y', 'dx', 'dy', 'game', 'team', 'player', 'event',
                     'period_id', 'type_id', 'bodypart_id'):
            setattr(s, name, self.cols[name].data_ptr())
        return s


def first_pass_device(frame: SpadlFrame) -> SpadlFrame:
    """The general path's first pass (``_extra_from_passes``, base.py:38-112) on its own: the
    device flags the rows that get an inserted row (input-order successor), the host places the
    reference's concat [inputs, inserted rows] by the stable lexsort of their keys
    (base.py:109-110), and the device writes the sorted rows.  Returns them as a frame in sorted
    order (no ``order``) for the remaining passes."""
    from ...spadl.base import SpadlRows, _F64, _U8
    lib = _native.lib()
    dev = frame.buffer.device
    n = frame.n
    s = frame.struct()
    flags = torch.empty(max(n, 1), dtype=torch.uint8, device=dev)
    _native.check(lib.sa_atomic_passes_flags(ctypes.byref(s), flags.data_ptr(), stream_handle()))
    j = np.flatnonzero(flags[:n].cpu().numpy()).astype(np.int64)
    m = len(j)
    g, per, aid = frame.keys
    kg = np.concatenate([g, g[j]]).astype(np.int64)
    kp = np.concatenate([per, per[j]]).astype(np.int64)
    ka = np.concatenate([aid, aid[j] + 0.1])
    order = np.lexsort((ka, kp, kg))  # stable, like sort_values on several keys
    pos = np.empty(n + m, np.int64)
    pos[order] = np.arange(n + m, dtype=np.int64)
    dest = torch.from_numpy(pos).to(dev)
    parents = torch.from_numpy(j if m else np.zeros(1, np.int64)).to(dev)
    spec = {c: np.float64 for c in _F64}
    spec.update(game=np.int32, team=np.int32, player=np.int32, event=np.int32)
    spec.update({c: np.uint8 for c in _U8})
    buf, cols = _alloc(spec, n + m, dev)
    cols['src'] = torch.empty(n + m, dtype=torch.int64, device=dev)
    rows = SpadlRows(n + m, m, buf, cols)
    o = rows.struct()
    _native.check(lib.sa_atomic_passes_emit(ctypes.byref(s), parents.data_ptr(), m, dest.data_ptr(),
                                            ctypes.byref(o), stream_handle()))
    keep = dict(cols, _dest=dest, _parents=parents)  # alive until the stream has used them
    return SpadlFrame(n + m, buf, keep, frame.uniques, frame.dtypes, None, True)


def convert_device(frame: SpadlFrame) -> AtomicColumns:
    """Run the conversion on device; the result stays in HBM."""
    lib = _native.lib()
    if frame.keys is not None and not frame.after_passes:
        frame = first_pass_device(frame)
    count, emit = ((lib.sa_atomic_count_after_passes, lib.sa_atomic_emit_after_passes)
                   if frame.after_passes else (lib.sa_atomic_count, lib.sa_atomic_emit))
    dev = frame.buffer.device
    s = frame.struct()
    scratch = torch.empty(max(int(lib.sa_atomic_scratch_bytes(frame.n)), 16), dtype=torch.uint8,
                          device=dev)
    n_out = ctypes.c_int64(0)
    _native.check(count(ctypes.byref(s), scratch.data_ptr(), ctypes.byref(n_out), stream_handle()))
    m = int(n_out.value)
    spec = {'time_seconds': np.float64, 'x': np.float64, 'y': np.float64, 'dx': np.float64,
            'dy': np.float64, 'game': np.int32, 'team': np.int32, 'player': np.int32,
            'event': np.int32, 'period_id': np.uint8, 'type_id': np.uint8, 'bodypart_id': np.uint8}
    buf, cols = _alloc(spec, max(m, 1), dev)
    out = AtomicColumns(m, buf, cols)
    if m:
        o = out.struct()
        _native.check(emit(ctypes.byref(s), scratch.data_ptr(), ctypes.byref(o), stream_handle()))
    return out


def _decode(codes: np.ndarray, uniques: pd.Index, dtype, missing=None) -> np.ndarray:
    """Ids back from their codes (code -1 -> ``missing``)."""
    neg = codes < 0
    if len(uniques) == 0:
        return np.full(len(codes), missing, dtype=object)
    vals = uniques.take(np.where(neg, 0, codes)).to_numpy()
    if neg.any():
        vals = vals.astype(object)
        vals[neg] = missing
    elif dtype is not None and vals.dtype != dtype:
        vals = vals.astype(dtype)
    return vals


def convert_to_atomic(actions: pd.DataFrame) -> pd.DataFrame:
    """Convert regular SPADL actions to Atomic-SPADL actions (reference base.py:15-35)."""
    for c in _REQUIRED:
        if c not in actions.columns:
            raise AttributeError(f"'DataFrame' object has no attribute '{c}'")
    if len(actions) == 0:
        cols = {c: np.zeros(0, np.int64) for c in _OUT}
        for c in ('game_id', 'team_id', 'player_id'):
            cols[c] = actions[c].to_numpy()[:0]
        for c in ('time_seconds', 'x', 'y', 'dx', 'dy'):
            cols[c] = np.zeros(0, np.float64)
        cols['original_event_id'] = np.zeros(0, dtype=object)
        return pd.DataFrame(cols, columns=list(_OUT))
    frame = SpadlFrame.from_frame(actions)
    out = convert_device(frame)
    host = {k: v[:out.n].cpu().numpy() for k, v in out.cols.items()}
    u = frame.uniques
    res = {
        'game_id': _decode(host['game'], u['game'], frame.dtypes['game_id']),
        'original_event_id': _decode(host['event'], u['event'], None, missing=np.nan).astype(object),
        'action_id': np.arange(out.n, dtype=np.int64),
        'period_id': host['period_id'].astype(np.int64),
        'time_seconds': host['time_seconds'],
        'team_id': _decode(host['team'], u['team'], frame.dtypes['team_id']),
        'player_id': _decode(host['player'], u['player'], frame.dtypes['player_id']),
        'x': host['x'], 'y': host['y'], 'dx': host['dx'], 'dy': host['dy'],
        'type_id': host['type_id'].astype(np.int64),
        'bodypart_id': host['bodypart_id'].astype(np.int64),
    }
    return pd.DataFrame(res, columns=list(_OUT))
