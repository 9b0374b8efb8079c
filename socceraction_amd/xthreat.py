"""Expected Threat (xT) on MI355X (drop-in for ``socceraction.xthreat``).

``ExpectedThreat.fit`` = one count launch over all actions (``sa_xt_count``: binning,
shot/goal/move histograms and the C x C successful-move transition counts), then one
solve (``sa_xt_solve``: normalisation + value iteration with the reference's exact
summation order, so the iteration count and surface are bit-identical). ``rate`` is one
gather launch over a cell grid or the 1050 x 680 interpolated surface. For multi-GPU
fits, :meth:`ExpectedThreat.fit` takes a ``process_group``: every rank counts its own
game shard and the counts are summed with one RCCL all-reduce before the (replicated)
solve — the path's only collective.
"""
from __future__ import annotations

import json
import os
import warnings
from typing import Callable, List, Optional, Tuple

import numpy as np
import pandas as pd
import torch
from sklearn.exceptions import NotFittedError

from . import ops
from .batch import ActionBatch
from .spadl import config as spadlconfig

M: int = 12
N: int = 16

_MOVE_TYPES = (spadlconfig.actiontypes.index('pass'), spadlconfig.actiontypes.index('dribble'),
               spadlconfig.actiontypes.index('cross'))


def _get_cell_indexes(x: pd.Series, y: pd.Series, l: int = N, w: int = M
                      ) -> Tuple[pd.Series, pd.Series]:
    """Cell indexes (reference xthreat.py:25-32): (x/105)*l truncated, clipped to the grid.

    Host index arithmetic (the kernels use the identical device function)."""
    xi = x.divide(spadlconfig.field_length).multiply(l)
    yj = y.divide(spadlconfig.field_width).multiply(w)
    xi = xi.astype('int64').clip(0, l - 1)
    yj = yj.astype('int64').clip(0, w - 1)
    return xi, yj


def _get_flat_indexes(x: pd.Series, y: pd.Series, l: int = N, w: int = M) -> pd.Series:
    """Row-major flat index with row 0 = top (max y) (reference xthreat.py:35-37)."""
    xi, yj = _get_cell_indexes(x, y, l, w)
    return yj.rsub(w - 1).mul(l).add(xi)


def _xy_batch(x, y, type_id: int, result_id: int = 1, ex=None, ey=None) -> ActionBatch:
    x = np.asarray(x, dtype=np.float64)
    y = np.asarray(y, dtype=np.float64)
    n = len(x)
    cols = {'c0': x, 'c1': y,
            'c2': x if ex is None else np.asarray(ex, np.float64),
            'c3': y if ey is None else np.asarray(ey, np.float64),
            'time_seconds': np.zeros(n), 'type_id': np.full(n, type_id, np.uint8),
            'result_id': np.full(n, result_id, np.uint8), 'bodypart_id': np.zeros(n, np.uint8),
            'period_id': np.ones(n, np.uint8), 'team': np.zeros(n, np.int32)}
    return ActionBatch(cols, np.array([0, n], np.int64), None, False)


def _count(x: pd.Series, y: pd.Series, l: int = N, w: int = M) -> np.ndarray:
    """Actions per grid cell, NaN rows dropped (reference xthreat.py:40-67)."""
    if len(x) == 0:
        return np.zeros((w, l))
    acc = ops.xt_count(_xy_batch(x, y, spadlconfig.actiontypes.index('shot')), l, w)
    ops.xt_check_errors(acc)
    return acc.shot.cpu().numpy().astype(np.float64).reshape((w, l))


def _device():
    from .batch import device
    return device()


def _safe_divide(a, b) -> np.ndarray:
    return np.divide(a, b, out=np.zeros_like(a), where=b != 0)


def _fit_counts(actions: pd.DataFrame, l: int, w: int, process_group=None,
                mask: int = ops.XT_ERR_FIT, dense: bool = True) -> ops.XTCounts:
    if len(actions):
        # the many-batch entry (one batch): a fresh accumulator the band-owned count writes
        # whole, and for 1025 - 9472 cells the solve's compact rows from the same pass
        # (dense=False: those rows alone, no C x C table -- a fit without an all-reduce)
        acc = ops.xt_count_many([ActionBatch.from_frame(actions)], l, w,
                                dense=dense or process_group is not None)
    else:
        from .batch import device
        acc = ops.xt_zero_counts(l, w, device())
    if process_group is not None:
        from .shard import allreduce_xt_counts
        allreduce_xt_counts(acc, process_group)
    ops.xt_check_errors(acc, mask)
    return acc


def scoring_prob(actions: pd.DataFrame, l: int = N, w: int = M) -> np.ndarray:
    """P(goal | shot) per cell (reference xthreat.py:74-98)."""
    mats, _ = ops.xt_normalize(_fit_counts(actions, l, w, mask=ops.XT_ERR_SHOT))
    return mats[0].cpu().numpy().reshape((w, l))


def get_move_actions(actions: pd.DataFrame) -> pd.DataFrame:
    """Passes, dribbles and crosses (reference xthreat.py:101-122)."""
    return actions[actions.type_id.isin(_MOVE_TYPES)]


def get_successful_move_actions(actions: pd.DataFrame) -> pd.DataFrame:
    """Successful passes, dribbles and crosses (reference xthreat.py:125-141)."""
    move_actions = get_move_actions(actions)
    return move_actions[move_actions.result_id == spadlconfig.results.index('success')]


def action_prob(actions: pd.DataFrame, l: int = N, w: int = M) -> Tuple[np.ndarray, np.ndarray]:
    """P(shoot) and P(move) per cell (reference xthreat.py:144-174)."""
    mats, _ = ops.xt_normalize(_fit_counts(actions, l, w,
                                           mask=ops.XT_ERR_SHOT | ops.XT_ERR_MOVE_START))
    m = mats.cpu().numpy()
    return m[1].reshape((w, l)), m[2].reshape((w, l))


def move_transition_matrix(actions: pd.DataFrame, l: int = N, w: int = M) -> np.ndarray:
    """P(successful move s -> e | move from s) (reference xthreat.py:177-218)."""
    _, tt = ops.xt_normalize(_fit_counts(
        actions, l, w, mask=ops.XT_ERR_MOVE_START | ops.XT_ERR_MOVE_OTHER))
    return np.ascontiguousarray(tt.cpu().numpy().T)


_SPLINE_DEGREE = {'linear': 1, 'cubic': 3, 'quintic': 5}


def _spline_interp2d(x, y, z, k):
    """``interp2d(x, y, z, kind='cubic' | 'quintic')`` on a regular grid, as scipy < 1.14 computes
    it: the interpolating tensor-product spline of degree k (FITPACK ``regrid_smth`` with s = 0,
    i.e. ``RectBivariateSpline(x, y, z.T, kx=k, ky=k, s=0)``) evaluated by ``bisplev`` on the
    sorted query axes, points outside the node hull clamped to it (bounds_error=False,
    fill_value=None), result shape (len(ys), len(xs)).  A host delegation to scipy like the
    reference's own (xthreat.py:347-378); off the rating path (``rate`` interpolates linearly on
    the device).  scipy >= 1.14 dropped interp2d itself, so this is pinned to the same
    RectBivariateSpline stand-in the linear golden was produced with."""
    from scipy.interpolate import RectBivariateSpline
    z = np.asarray(z, dtype=np.float64)
    x = np.asarray(x, np.float64).reshape(-1)
    y = np.asarray(y, np.float64).reshape(-1)
    if len(x) <= k or len(y) <= k:
        raise ValueError(f'{k + 1} nodes per axis are needed for a degree-{k} spline')
    spl = RectBivariateSpline(x, y, z.T, kx=k, ky=k, s=0)

    def f(xs, ys):
        xs = np.clip(np.sort(np.atleast_1d(np.asarray(xs, np.float64))), x[0], x[-1])
        ys = np.clip(np.sort(np.atleast_1d(np.asarray(ys, np.float64))), y[0], y[-1])
        return spl(xs, ys).T

    return f


def _gpu_interp2d(x, y, z, kind='linear', bounds_error=False):
    """GPU stand-in for ``scipy.interpolate.interp2d(x, y, z, kind='linear')`` on a regular
    grid: z[j, i] sits at (x[i], y[j]); queries are clamped to the node hull.  ``kind`` 'cubic'
    and 'quintic' delegate to scipy's spline (:func:`_spline_interp2d`)."""
    if kind not in _SPLINE_DEGREE:
        raise ValueError(f'Unsupported interpolation type {kind!r}.')
    if kind != 'linear':
        return _spline_interp2d(x, y, z, _SPLINE_DEGREE[kind])
    z = np.asarray(z, dtype=np.float64)
    w, l = z.shape
    x = np.asarray(x, np.float64).reshape(-1)
    y = np.asarray(y, np.float64).reshape(-1)
    if len(x) != l or len(y) != w:
        raise ValueError('x and y must have the lengths of the xT surface')
    if l < 2 or w < 2:
        raise ValueError('linear interpolation needs at least 2 nodes per axis')
    if (np.diff(x) <= 0).any() or (np.diff(y) <= 0).any() or \
            not (np.isfinite(x).all() and np.isfinite(y).all()):
        raise ValueError('x and y must be finite and strictly increasing')
    zt = torch.from_numpy(np.ascontiguousarray(z))

    def f(xs, ys):
        from .batch import device
        g = ops.xt_interp_grid(zt.to(device()), l, w, np.atleast_1d(xs), np.atleast_1d(ys),
                               cx=x, cy=y)
        return g.cpu().numpy()

    return f


interp2d = _gpu_interp2d  # module attribute, like the reference's optional scipy import


class ExpectedThreat:
    """Expected Threat model (reference xthreat.py:221-504).

    Parameters
    ----------
    l, w : int
        Grid cells along x (length) and y (width).
    eps : float
        Convergence threshold of the value iteration.
    """

    def __init__(self, l: int = N, w: int = M, eps: float = 1e-5) -> None:
        self.l = l
        self.w = w
        self.eps = eps
        self.heatmaps: List[np.ndarray] = []
        self.xT: np.ndarray = np.zeros((self.w, self.l))
        self.scoring_prob_matrix: Optional[np.ndarray] = None
        self.shot_prob_matrix: Optional[np.ndarray] = None
        self.move_prob_matrix: Optional[np.ndarray] = None
        self.transition_matrix: Optional[np.ndarray] = None
        self._grid_cache = None

    # The C x C transition matrix (reference attribute, xthreat.py:276, 337). Grids above
    # LAZY_TRANSITION_CELLS leave it on the device after fit -- the solve never forms it, and
    # at 105 x 68 it is 408 MB -- and it is normalised and copied to the host on first access.
    LAZY_TRANSITION_CELLS = 1024

    @property
    def transition_matrix(self) -> Optional[np.ndarray]:
        if self._transition is None and getattr(self, '_transition_counts', None) is not None:
            # host-side from the compact counts fit kept: T[s, e] = count(s -> e) / moves from s,
            # the reference's `vc2 / start_counts[i]` (one f64 division per non-zero bin)
            move, idx, cnt = self._transition_counts
            C = self.l * self.w
            t = np.zeros(C * C)
            t[idx] = cnt.astype(np.float64) / move[idx // C].astype(np.float64)
            self._transition = t.reshape(C, C)
            self._transition_counts = None
        return self._transition

    @transition_matrix.setter
    def transition_matrix(self, value: Optional[np.ndarray]) -> None:
        self._transition = value
        self._transition_counts = None

    def fit(self, actions: pd.DataFrame, process_group=None, max_iter: int = 1000,
            shard_solve: bool = False, exact_order: bool = False) -> 'ExpectedThreat':
        """Fit the model (reference xthreat.py:322-345).

        With ``process_group`` each rank passes its own shard of games; counts are summed
        with one RCCL all-reduce and every rank solves the same system. ``shard_solve=True``
        instead splits the count rows and the value iteration over the ranks (one all-gather of x
        per iteration; bit-identical results) for large grids -- grids the band-owned count holds
        (``ops.xt_band_shape``, e.g. 105 x 68) exchange the ranks' counted actions by one
        all-to-all, others reduce-scatter the count table; the C x C ``transition_matrix`` is
        then not materialised (left ``None``).

        Grids above 1024 cells sum each row of the value iteration in a fixed parallel order
        under an error bound that keeps every convergence decision, and so the iteration count,
        the reference's; the surface is then within 4e-11 relative of the reference's (105 x 68;
        ``ops.xt_solve``).  ``exact_order=True`` sums in the reference's order (bit-exact).
        ``self.solve_path`` records which path ran.
        """
        w, l = self.w, self.l
        if shard_solve and process_group is not None and ops.xt_band_shape(l, w) is not None:
            # band-owned grids: the ranks exchange their counted actions (an all-to-all of 4-B
            # keys) instead of reduce-scattering the C x C count table
            import types

            from .shard import xt_fit_bands_sharded
            batches = [ActionBatch.from_frame(actions)] if len(actions) else []
            mats, heat_t, n_iter, err = xt_fit_bands_sharded(batches, l, w, self.eps, max_iter,
                                                             process_group, exact_order=exact_order)
            self.solve_path = 'exchanged'
            ops.xt_check_errors(types.SimpleNamespace(err=err))
            trans = None
        elif shard_solve and process_group is not None:
            import torch.distributed as dist

            from .shard import xt_solve_sharded
            world = dist.get_world_size(process_group)
            if len(actions):
                acc = ops.xt_zero_counts(l, w, _device(), row_blocks=world)
                ops.xt_count(ActionBatch.from_frame(actions), l, w, acc)
            else:
                acc = ops.xt_zero_counts(l, w, _device(), row_blocks=world)
            mats, heat_t, n_iter = xt_solve_sharded(acc, self.eps, max_iter, process_group)
            self.solve_path = 'sequential'
            ops.xt_check_errors(acc)
            trans = None
        else:
            lazy = l * w > self.LAZY_TRANSITION_CELLS
            acc = _fit_counts(actions, l, w, process_group, dense=not lazy)
            sol = ops.xt_solve(acc, self.eps, max_iter, transition=not lazy,
                               exact_order=exact_order)
            mats, heat_t, n_iter = sol.mats, sol.heatmaps, sol.n_iter
            self.solve_path = sol.path
            trans = None if lazy else np.ascontiguousarray(sol.trans_t.cpu().numpy().T)
        m = mats.cpu().numpy()
        self.scoring_prob_matrix = m[0].reshape((w, l))
        self.shot_prob_matrix = m[1].reshape((w, l))
        self.move_prob_matrix = m[2].reshape((w, l))
        self.transition_matrix = trans
        if trans is None and not (shard_solve and process_group is not None):
            # normalised on first access from a compact HOST copy (move counts + the non-zero
            # transition bins, read from the count's compact rows when it wrote them), so the
            # 4*C*C-byte device count buffer is not kept alive
            nz, cnt = ops.xt_transition_entries(acc)
            self._transition_counts = (acc.move.cpu().numpy(), nz.cpu().numpy(),
                                       cnt.cpu().numpy())
        self.xT = m[3].reshape((w, l)).copy()
        heat = heat_t.cpu().numpy().reshape((-1, w, l))
        self.heatmaps = [h.copy() for h in heat]
        self._grid_cache = None
        print('# iterations: ', n_iter)
        return self

    def interpolator(self, kind: str = 'linear') -> Callable[[np.ndarray, np.ndarray], np.ndarray]:
        """Bilinear interpolation over the pitch (reference xthreat.py:347-378)."""
        if interp2d is None:
            raise ImportError('Interpolation requires scipy to be installed.')
        cell_length = spadlconfig.field_length / self.l
        cell_width = spadlconfig.field_width / self.w
        x = np.arange(0.0, spadlconfig.field_length, cell_length) + 0.5 * cell_length
        y = np.arange(0.0, spadlconfig.field_width, cell_width) + 0.5 * cell_width
        return interp2d(x=x, y=y, z=self.xT, kind=kind, bounds_error=False)

    def predict(self, actions: pd.DataFrame, use_interpolation: bool = False) -> np.ndarray:
        """Deprecated alias of :meth:`rate` (reference xthreat.py:380-406)."""
        warnings.warn('predict is deprecated, use rate instead', DeprecationWarning)
        return self.rate(actions, use_interpolation)

    def _grid(self, use_interpolation: bool) -> Tuple[torch.Tensor, int, int]:
        from .batch import device
        key = (use_interpolation, self.xT.tobytes())
        if self._grid_cache is not None and self._grid_cache[0] == key:
            return self._grid_cache[1]
        xT = torch.from_numpy(np.ascontiguousarray(self.xT, dtype=np.float64)).to(device())
        w, l = self.xT.shape
        if not use_interpolation:
            res = (xT, l, w)
        else:
            if interp2d is None:
                raise ImportError('Interpolation requires scipy to be installed.')
            L = int(spadlconfig.field_length * 10)
            W = int(spadlconfig.field_width * 10)
            # the surface + its node positions: the rate evaluates each node in place
            # (sa_xt_rate_interp), the 1050 x 680 grid is never formed
            res = (xT, L, W, ops.xt_interp_axes(l, w, device(), L, W))
        self._grid_cache = (key, res)
        return res

    def rate(self, actions: pd.DataFrame, use_interpolation: bool = False) -> np.ndarray:
        """xT value of every successful move, NaN elsewhere (reference xthreat.py:408-465)."""
        if not np.any(self.xT):
            raise NotFittedError()
        g = self._grid(use_interpolation)
        if len(actions) == 0:
            return np.empty(0)
        ab = ActionBatch.from_frame(actions)
        if use_interpolation:
            xT, L, W, axes = g
            out, err = ops.xt_rate_interp(ab, xT, self.l, self.w, L, W, axes=axes)
        else:
            out, err = ops.xt_rate(ab, *g)
        if int(err.item()):
            raise ValueError('Cannot convert non-finite values (NA or inf) to integer')
        return out.cpu().numpy()

    def save_model(self, filepath: str, overwrite: bool = True) -> None:
        """Save the xT surface as JSON (reference xthreat.py:467-504)."""
        if not np.any(self.xT):
            raise NotFittedError()
        if not overwrite and os.path.isfile(filepath):
            raise ValueError(
                'save_xt got overwrite="False", but a file '
                f'({filepath}) exists already. No data was saved.'
            )
        with open(filepath, 'w') as f:
            json.dump(self.xT.tolist(), f)


def load_model(path: str) -> ExpectedThreat:
    """Model from a JSON xT surface (reference xthreat.py:507-529)."""
    grid = pd.read_json(path)
    model = ExpectedThreat()
    model.xT = grid.values
    model.w, model.l = model.xT.shape
    return model
