"""Feature-column catalogue: names, dtypes and block layout of every known transformer.

The names and their order reproduce what the reference transformers emit
(vaep/features.py:119-539, atomic/vaep/features.py:114-260): a ``@simple``
transformer emits its per-frame columns for a0, then a1, ... with an ``_a{i}``
suffix (features.py:135-143); state features emit one group per previous action.

Each column is ``(name, kind, slot)`` where kind is ``'b'`` (bool), ``'f'`` (float64)
or ``'i'`` (int64) and ``slot`` is the column's offset inside the transformer's run in
that dtype's output block. The HIP kernel (``csrc/sa_vaep.hip``) writes exactly these
slots, so this table and the kernel must change together.
"""
from __future__ import annotations

from dataclasses import dataclass
from functools import lru_cache
from typing import Dict, List, Sequence, Tuple

import numpy as np
import pandas as pd

from ._native import SA_XFN_COUNT, XFN, SaFeaturePlan
from .atomic.spadl import config as atomicconfig
from .spadl import config as spadlconfig

Column = Tuple[str, str, int]

SPADL_XFNS = ('actiontype', 'actiontype_onehot', 'result', 'result_onehot',
              'actiontype_result_onehot', 'bodypart', 'bodypart_onehot', 'time',
              'startlocation', 'endlocation', 'startpolar', 'endpolar', 'movement', 'team',
              'time_delta', 'space_delta', 'goalscore')
ATOMIC_XFNS = ('actiontype', 'actiontype_onehot', 'bodypart', 'bodypart_onehot', 'time', 'team',
               'time_delta', 'location', 'polar', 'movement_polar', 'direction', 'goalscore')


def atomic_type_names() -> List[str]:
    """Unique atomic type names in first-occurrence order (32; 'interception' once)."""
    seen: Dict[str, None] = {}
    for name in atomicconfig.actiontypes:
        seen.setdefault(name, None)
    return list(seen)


def _per_frame(k: int, fields: Sequence[Tuple[str, str]]) -> List[Column]:
    """Columns of a @simple transformer: fields for a0, then a1, ... (suffix _a{i})."""
    cols: List[Column] = []
    count: Dict[str, int] = {'b': 0, 'f': 0, 'i': 0}
    for i in range(k):
        for name, kind in fields:
            cols.append((f'{name}_a{i}', kind, count[kind]))
            count[kind] += 1
    return cols


def xfn_columns(xfn: str, k: int, atomic: bool = False) -> List[Column]:
    """Columns emitted by transformer ``xfn`` at ``nb_prev_actions = k``."""
    if xfn == 'actiontype':
        return _per_frame(k, [('type_id', 'i')])
    if xfn == 'actiontype_onehot':
        names = atomic_type_names() if atomic else spadlconfig.actiontypes
        return _per_frame(k, [(f'type_{t}', 'b') for t in names])
    if xfn == 'result':
        return _per_frame(k, [('result_id', 'i')])
    if xfn == 'result_onehot':
        return _per_frame(k, [(f'result_{r}', 'b') for r in spadlconfig.results])
    if xfn == 'actiontype_result_onehot':
        return _per_frame(k, [(f'type_{t}_result_{r}', 'b') for t in spadlconfig.actiontypes
                              for r in spadlconfig.results])
    if xfn == 'bodypart':
        return _per_frame(k, [('bodypart_id', 'i')])
    if xfn == 'bodypart_onehot':
        return _per_frame(k, [(f'bodypart_{b}', 'b') for b in spadlconfig.bodyparts])
    if xfn == 'time':
        return _per_frame(k, [('period_id', 'i'), ('time_seconds', 'f'),
                              ('time_seconds_overall', 'f')])
    if xfn == 'startlocation':
        return _per_frame(k, [('start_x', 'f'), ('start_y', 'f')])
    if xfn == 'endlocation':
        return _per_frame(k, [('end_x', 'f'), ('end_y', 'f')])
    if xfn == 'startpolar':
        return _per_frame(k, [('start_dist_to_goal', 'f'), ('start_angle_to_goal', 'f')])
    if xfn == 'endpolar':
        return _per_frame(k, [('end_dist_to_goal', 'f'), ('end_angle_to_goal', 'f')])
    if xfn == 'movement':
        return _per_frame(k, [('dx', 'f'), ('dy', 'f'), ('movement', 'f')])
    if xfn == 'location':
        return _per_frame(k, [('x', 'f'), ('y', 'f')])
    if xfn == 'polar':
        return _per_frame(k, [('dist_to_goal', 'f'), ('angle_to_goal', 'f')])
    if xfn == 'movement_polar':
        return _per_frame(k, [('mov_d', 'f'), ('mov_angle', 'f')])
    if xfn == 'direction':
        return _per_frame(k, [('dx', 'f'), ('dy', 'f')])
    if xfn == 'team':
        return [(f'team_{i}', 'b', i - 1) for i in range(1, k)]
    if xfn == 'time_delta':
        return [(f'time_delta_{i}', 'f', i - 1) for i in range(1, k)]
    if xfn == 'space_delta':
        cols = []
        for i in range(1, k):
            cols += [(f'dx_a0{i}', 'f', 3 * (i - 1)), (f'dy_a0{i}', 'f', 3 * (i - 1) + 1),
                     (f'mov_a0{i}', 'f', 3 * (i - 1) + 2)]
        return cols
    if xfn == 'goalscore':
        return [('goalscore_team', 'i', 0), ('goalscore_opponent', 'i', 1),
                ('goalscore_diff', 'i', 2)]
    raise KeyError(xfn)


@dataclass
class FeaturePlan:
    """Block layout for an ordered list of known transformers.

    ``order`` lists, in output order, ``(name, kind, block_column)`` for every column of
    every transformer in ``xfns`` (a transformer listed twice repeats its columns, as
    ``pd.concat`` in the reference would).
    """

    xfns: Tuple[str, ...]
    k: int
    atomic: bool
    n_bool: int
    n_f64: int
    n_i64: int
    order: List[Tuple[str, str, int]]
    struct: SaFeaturePlan

    @property
    def names(self) -> List[str]:
        return [c[0] for c in self.order]


def build_plan(xfns: Sequence[str], k: int, atomic: bool = False) -> FeaturePlan:
    """The block layout of ``xfns`` (cached: callers treat plans as read-only)."""
    return _build_plan(tuple(xfns), int(k), bool(atomic))


@lru_cache(maxsize=128)
def _build_plan(xfns: Tuple[str, ...], k: int, atomic: bool) -> FeaturePlan:
    valid = ATOMIC_XFNS if atomic else SPADL_XFNS
    if k < 1:
        # the reference's gamestates(actions, 0) is [actions]: one frame, as k = 1
        k = 1
    base = {'b': {}, 'f': {}, 'i': {}}
    count = {'b': 0, 'f': 0, 'i': 0}
    order = []
    for x in xfns:
        if x not in valid:
            raise ValueError(f'transformer {x!r} is not defined for '
                             f'{"atomic" if atomic else "SPADL"} actions')
        cols = xfn_columns(x, k, atomic)
        for kind in 'bfi':
            if x not in base[kind]:
                nk = sum(1 for c in cols if c[1] == kind)
                if nk:
                    base[kind][x] = count[kind]
                    count[kind] += nk
        for name, kind, slot in cols:
            order.append((name, kind, base[kind][x] + slot))
    s = SaFeaturePlan()
    s.nb_prev_actions = k
    for kind, arr in (('b', s.bool_col), ('f', s.f64_col), ('i', s.i64_col)):
        for j in range(SA_XFN_COUNT):
            arr[j] = -1
        for x, c in base[kind].items():
            arr[XFN[x]] = c
    return FeaturePlan(tuple(xfns), k, atomic, count['b'], count['f'], count['i'], order, s)


def _frame_from_blocks(plan: FeaturePlan, blocks: dict, n: int) -> pd.DataFrame:
    """Zero-copy DataFrame over the host blocks: one pandas block per dtype, placed at the
    reference's column positions (no per-column Series, no consolidation copy)."""
    from pandas.core.internals import BlockManager
    from pandas.core.internals.api import make_block
    sizes = {'b': plan.n_bool, 'f': plan.n_f64, 'i': plan.n_i64}
    pos = {k: np.full(sizes[k], -1, np.intp) for k in sizes}
    for p, (_, kind, col) in enumerate(plan.order):
        pos[kind][col] = p
    mblocks = []
    for kind in 'bfi':
        if sizes[kind] == 0:
            continue
        if (pos[kind] < 0).any():
            raise ValueError('block column without a name')
        v = blocks[kind][:sizes[kind], :n]
        mblocks.append(make_block(v.view(np.bool_) if kind == 'b' else v, placement=pos[kind],
                                  ndim=2))
    mgr = BlockManager(mblocks, [pd.Index(plan.names), pd.RangeIndex(n)])
    return pd.DataFrame._from_mgr(mgr, mgr.axes)


def assemble_frame(plan: FeaturePlan, bool_block: np.ndarray, f64_block: np.ndarray,
                   i64_block: np.ndarray, n: int, index=None) -> pd.DataFrame:
    """Build the feature DataFrame from column-major host blocks ``[cols, >= n]``."""
    blocks = {'b': bool_block, 'f': f64_block, 'i': i64_block}
    df = None
    if len(set(plan.names)) == len(plan.names):
        try:
            df = _frame_from_blocks(plan, blocks, n)
        except (ImportError, AttributeError, TypeError, ValueError):  # pandas internals moved
            df = None
    if df is None:
        if len(set(plan.names)) != len(plan.names):  # a transformer listed twice: keep duplicates
            series = []
            for name, kind, col in plan.order:
                v = blocks[kind][col, :n]
                series.append(pd.Series(v.view(np.bool_) if kind == 'b' else v, name=name,
                                        copy=False))
            df = pd.concat(series, axis=1)
        else:
            data = {}
            for name, kind, col in plan.order:
                v = blocks[kind][col, :n]
                data[name] = v.view(np.bool_) if kind == 'b' else v
            df = pd.DataFrame(data, copy=False)
    if index is not None:
        df.index = index
    return df
