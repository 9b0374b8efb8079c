"""CPU oracle (numpy restatement) of the reference's Expected Threat path.

TEST INFRASTRUCTURE ONLY (see ``oracle/vaep_oracle.py``). Parity pinned against
goldens generated from the reference (``tests/golden/xt_*.npz``) and the
reference's own known-answer tests (``tests/test_xthreat.py:44-193``).

Follows socceraction/xthreat.py: binning ``_get_cell_indexes`` (:25-37), ``_count``
(:40-67), ``scoring_prob`` (:74-98), ``action_prob`` (:144-174),
``move_transition_matrix`` (:177-218), ``__solve`` (:278-320), ``rate`` (:408-465) and
the ``interp2d(kind='linear')`` surface (:347-378), restated as clamped bilinear
interpolation through the cell centres.
"""
from __future__ import annotations

from typing import Dict, Tuple

import numpy as np

FIELD_L, FIELD_W = 105.0, 68.0


def _to_int64(v: np.ndarray) -> np.ndarray:
    """numpy float64 -> int64 cast as on x86 (NaN / out of range -> INT64_MIN)."""
    v = np.asarray(v, dtype=np.float64)
    out = np.full(v.shape, np.iinfo(np.int64).min, dtype=np.int64)
    ok = (v >= -9.2233720368547758e18) & (v < 9.2233720368547758e18)
    out[ok] = v[ok].astype(np.int64)
    return out


def cell_indexes(x, y, l: int, w: int) -> Tuple[np.ndarray, np.ndarray]:
    xi = np.clip(_to_int64(np.asarray(x, np.float64) / FIELD_L * l), 0, l - 1)
    yj = np.clip(_to_int64(np.asarray(y, np.float64) / FIELD_W * w), 0, w - 1)
    return xi, yj


def flat_indexes(x, y, l: int, w: int) -> np.ndarray:
    xi, yj = cell_indexes(x, y, l, w)
    return (w - 1 - yj) * l + xi


def count(x, y, l: int, w: int) -> np.ndarray:
    x = np.asarray(x, np.float64)
    y = np.asarray(y, np.float64)
    keep = ~np.isnan(x) & ~np.isnan(y)
    v = np.bincount(flat_indexes(x[keep], y[keep], l, w), minlength=w * l).astype(np.float64)
    return v.reshape((w, l))


def _safe_divide(a, b):
    return np.divide(a, b, out=np.zeros_like(a), where=b != 0)


def counts(cols: Dict[str, np.ndarray], l: int = 16, w: int = 12) -> dict:
    """The fit's integer counts (xthreat.py:74-218): shots, goals and moves per start cell,
    moves per start cell for the transition rows, and the C x C successful-move counts
    (int64). Counts of disjoint action sets add, so shards can be summed before ``solve``."""
    t, r = cols['type_id'], cols['result_id']
    sx, sy, ex, ey = cols['start_x'], cols['start_y'], cols['end_x'], cols['end_y']
    shot = t == 11
    goal = shot & (r == 1)
    move = (t == 0) | (t == 21) | (t == 1)
    C = l * w
    s_cell = flat_indexes(sx[move], sy[move], l, w)
    e_cell = flat_indexes(ex[move], ey[move], l, w)
    succ = r[move] == 1
    tc = np.bincount(s_cell[succ] * C + e_cell[succ], minlength=C * C).astype(np.int64)
    return dict(shot=count(sx[shot], sy[shot], l, w).astype(np.int64),
                goal=count(sx[goal], sy[goal], l, w).astype(np.int64),
                move=count(sx[move], sy[move], l, w).astype(np.int64),
                start=np.bincount(s_cell, minlength=C).astype(np.int64),
                trans=tc.reshape(C, C))


def solve(cnt: dict, l: int = 16, w: int = 12, eps: float = 1e-5) -> dict:
    """Probabilities, transition matrix and value iteration from ``counts`` (xthreat.py:74-218,
    278-320): the same float64 operations as the reference on its float64 count matrices."""
    shotm, goalm, movem = (cnt[k].astype(np.float64).reshape((w, l)) for k in ('shot', 'goal', 'move'))
    scoring = _safe_divide(goalm, shotm)
    total = movem + shotm
    pshot, pmove = _safe_divide(shotm, total), _safe_divide(movem, total)
    C = l * w
    start_counts = cnt['start'].astype(np.float64).reshape(-1)
    tc = cnt['trans'].reshape(C, C)
    T = np.zeros((C, C))
    nz = tc != 0
    rows = np.nonzero(nz)[0]
    T[nz] = tc[nz] / start_counts[rows]
    # value iteration, summed left to right in the reference's loop order (:306-312)
    gs = scoring * pshot
    xT = np.zeros((w, l))
    heat = [xT.copy()]
    Tt = np.ascontiguousarray(T.T)  # Tt[c] = T[:, c]: same products, contiguous rows
    while True:
        x = xT.reshape(-1)
        tot = np.zeros(C)
        for c in range(C):  # sequential accumulation over the flat column index
            tot += Tt[c] * x[c]
        newxT = gs + pmove * tot.reshape((w, l))
        diff = newxT - xT
        xT = newxT
        heat.append(xT.copy())
        if not np.any(diff > eps):
            break
    return dict(scoring_prob=scoring, shot_prob=pshot, move_prob=pmove, transition=T, xT=xT,
                heatmaps=np.stack(heat))


def fit(cols: Dict[str, np.ndarray], l: int = 16, w: int = 12, eps: float = 1e-5) -> dict:
    """ExpectedThreat.fit (xthreat.py:322-345): ``solve(counts(cols))``."""
    return solve(counts(cols, l, w), l, w, eps)


def centres(extent: float, cells: int) -> np.ndarray:
    size = extent / cells
    return np.arange(0.0, extent, size) + 0.5 * size


def _bracket(c: np.ndarray, q: np.ndarray):
    q = np.clip(q, c[0], c[-1])
    i = np.clip(np.searchsorted(c, q, side='right') - 1, 0, len(c) - 2)
    return i, (q - c[i]) / (c[i + 1] - c[i])


def interp_grid(xT: np.ndarray, L: int = 1050, W: int = 680) -> np.ndarray:
    """interp2d(x=cx, y=cy, z=xT, kind='linear')(linspace(0,105,L), linspace(0,68,W))."""
    w, l = xT.shape
    cx, cy = centres(FIELD_L, l), centres(FIELD_W, w)
    xs, ys = np.linspace(0, FIELD_L, L), np.linspace(0, FIELD_W, W)
    i, tx = _bracket(cx, xs)
    j, ty = _bracket(cy, ys)
    z00 = xT[j][:, i]
    z01 = xT[j][:, i + 1]
    z10 = xT[j + 1][:, i]
    z11 = xT[j + 1][:, i + 1]
    ux, uy = 1 - tx, 1 - ty
    return (ux * z00 + tx * z01) * uy[:, None] + (ux * z10 + tx * z11) * ty[:, None]


def rate(cols: Dict[str, np.ndarray], xT: np.ndarray, use_interpolation: bool = False) -> np.ndarray:
    if use_interpolation:
        grid = interp_grid(xT)
        W, L = grid.shape
    else:
        grid = xT
        W, L = xT.shape
    t, r = cols['type_id'], cols['result_id']
    ok = ((t == 0) | (t == 21) | (t == 1)) & (r == 1)
    out = np.full(len(t), np.nan)
    sxi, syj = cell_indexes(cols['start_x'][ok], cols['start_y'][ok], L, W)
    exi, eyj = cell_indexes(cols['end_x'][ok], cols['end_y'][ok], L, W)
    out[ok] = grid[W - 1 - eyj, exi] - grid[W - 1 - syj, sxi]
    return out
