"""``_add_dribbles`` on MI355X (drop-in for ``socceraction.spadl.base._add_dribbles``).

The reference (spadl/base.py:54-93) compares every action with its input-order successor
(``shift(-1, fill_value=0)``), inserts a dribble between the two when they belong to the same
team and period, lie 3-60 m apart and less than 10 s apart, then concatenates, sorts on
(game_id, period_id, action_id) and resets action_id. Here one kernel counts the inserted rows
per 256-row block (``sa_dribble_count``), one scan turns the counts into offsets and one kernel
writes every output row at its sorted position (``sa_dribble_emit``, csrc/sa_atomic.hip); the
host only factorises the id columns, checks that the fast layout is the reference's sort
order (else passes the stable lexsort of the concatenated keys) and builds the DataFrame.
The thresholds are read from this module's globals at call time, like the reference's.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass
from typing import Dict, Optional

import numpy as np
import pandas as pd
import torch

from .. import _native

min_dribble_length: float = 3.0
max_dribble_length: float = 60.0
max_dribble_duration: float = 10.0

_F64 = ('time_seconds', 'start_x', 'start_y', 'end_x', 'end_y')
_U8 = ('period_id', 'type_id', 'result_id', 'bodypart_id')
_DRIBBLE_TYPE = 21  # spadl/config.py actiontypes.index('dribble')


@dataclass
class SpadlRows:
    """SPADL rows in HBM (``sa_spadl_out``): codes as in the source SpadlFrame, ``src`` the
    input row (>= 0) or ``~q`` for a dribble inserted before input row q."""

    n: int
    n_dribbles: int
    buffer: torch.Tensor
    cols: Dict[str, torch.Tensor]

    def struct(self) -> _native.SaSpadlOut:
        s = _native.SaSpadlOut()
        for name, _ in _native.SaSpadlOut._fields_:
            setattr(s, name, self.cols[name].data_ptr())
        return s


def _rule():
    return (float(min_dribble_length) ** 2, float(max_dribble_length) ** 2,
            float(max_dribble_duration))


def add_dribbles_device(frame, action_id: np.ndarray) -> SpadlRows:
    """Run ``_add_dribbles`` on a device :class:`~socceraction_amd.atomic.spadl.base.SpadlFrame`
    (input order, no ``order``); ``action_id`` are the input's action ids (numpy or a device
    tensor; the sort keys). The result stays in HBM."""
    from ..atomic.spadl.base import _alloc, stream_handle
    lib = _native.lib()
    dev = frame.buffer.device
    n = frame.n
    s = frame.struct()
    rule = _rule()
    scratch = torch.empty(max(int(lib.sa_atomic_scratch_bytes(n)), 16), dtype=torch.uint8,
                          device=dev)
    flags = torch.empty(max(n, 1), dtype=torch.uint8, device=dev)
    if isinstance(action_id, torch.Tensor):
        aid_dev = action_id.to(device=dev, dtype=torch.float64).contiguous()
    else:
        aid_dev = torch.from_numpy(np.ascontiguousarray(action_id, dtype=np.float64)).to(dev)
    aid_dev = aid_dev if n else None
    n_out, n_bad = ctypes.c_int64(0), ctypes.c_int64(0)
    _native.check(lib.sa_dribble_count(ctypes.byref(s), *rule,
                                       aid_dev.data_ptr() if aid_dev is not None else None,
                                       scratch.data_ptr(), flags.data_ptr(), ctypes.byref(n_out),
                                       ctypes.byref(n_bad), stream_handle()))
    m = int(n_out.value)
    nd = m - n
    dest = None
    if nd > 0 and n_bad.value != 0:
        # general placement: the stable lexsort of the concatenated keys (the reference's
        # sort_values over its concat, spadl/base.py:91)
        g = frame.cols['game'][:n].cpu().numpy()
        per = frame.cols['period_id'][:n].cpu().numpy()
        j = np.flatnonzero(flags[:n].cpu().numpy())
        aid = aid_dev.cpu().numpy()
        kg = np.concatenate([g, g[j + 1]]).astype(np.int64)
        kp = np.concatenate([per, per[j + 1]]).astype(np.int64)
        ka = np.concatenate([aid, aid[j] + 0.1])
        order = np.lexsort((ka, kp, kg))  # stable, like sort_values on several keys
        pos = np.empty(m, np.int64)
        pos[order] = np.arange(m, dtype=np.int64)
        dest = torch.from_numpy(pos).to(dev)
    spec = {c: np.float64 for c in _F64}
    spec.update(game=np.int32, team=np.int32, player=np.int32, event=np.int32)
    spec.update({c: np.uint8 for c in _U8})
    buf, cols = _alloc(spec, max(m, 1), dev)
    cols['src'] = torch.empty(max(m, 1), dtype=torch.int64, device=dev)
    out = SpadlRows(m, nd, buf, cols)
    if m:
        o = out.struct()
        _native.check(lib.sa_dribble_emit(ctypes.byref(s), *rule, scratch.data_ptr(),
                                          dest.data_ptr() if dest is not None else None,
                                          ctypes.byref(o), stream_handle()))
    return out


def _passthrough(col: pd.Series, take: np.ndarray, missing: Optional[np.ndarray]) -> np.ndarray:
    """``col`` at input rows ``take``; rows in ``missing`` become NaN with the dtype pandas'
    concat gives a column the dribble rows lack (int -> float64, bool -> object, ...)."""
    s = pd.Series(col.to_numpy())
    if missing is None or not missing.any():
        return s.take(take).to_numpy()
    return s.reindex(np.where(missing, -1, take)).to_numpy()


def _add_dribbles(actions: pd.DataFrame) -> pd.DataFrame:
    """Insert dribbles between consecutive actions (reference spadl/base.py:54-93)."""
    from ..atomic.spadl.base import _REQUIRED, SpadlFrame, _decode
    for c in _REQUIRED:
        if c not in actions.columns:
            raise AttributeError(f"'DataFrame' object has no attribute '{c}'")
    n = len(actions)
    if n == 0:
        return actions.reset_index(drop=True).assign(action_id=np.arange(0, dtype=np.int64))
    frame = SpadlFrame.from_frame(actions, sort=False)
    out = add_dribbles_device(frame, actions['action_id'].to_numpy())
    host = {k: v[:out.n].cpu().numpy() for k, v in out.cols.items()}
    src = host['src']
    drib = src < 0
    take = np.where(drib, ~src, src)  # a dribble's columns come from its successor row
    u = frame.uniques
    res = {}
    for c in actions.columns:
        col = actions[c]
        if c == 'action_id':
            res[c] = np.arange(out.n, dtype=np.int64)
        elif c in _F64:
            v = host[c]
            res[c] = v if out.n_dribbles or col.dtype.kind == 'f' else v.astype(col.dtype)
        elif c in _U8:
            res[c] = host[c].astype(col.dtype if col.dtype.kind in 'iuf' else np.int64)
        elif c in ('game_id', 'team_id', 'player_id'):
            key = {'game_id': 'game', 'team_id': 'team', 'player_id': 'player'}[c]
            res[c] = _decode(host[key], u[key], frame.dtypes[c])
        elif c == 'timestamp':
            res[c] = _passthrough(col, take, None)
        else:  # original_event_id and any extra column: missing on the dribble rows
            res[c] = _passthrough(col, take, drib)
    return pd.DataFrame(res, columns=list(actions.columns))


__all__ = ['_add_dribbles', 'add_dribbles_device', 'SpadlRows', 'min_dribble_length',
           'max_dribble_length', 'max_dribble_duration']
