"""Gradient-boosted tree ensembles evaluated on the device feature blocks.

``VAEP.rate`` (reference vaep/base.py:296-333) is features -> ``predict_proba`` of one fitted
classifier per label (``_estimate_probabilities``, :284-294) -> ``formula.value``. The learners
the reference trains are xgboost (default), catboost and lightgbm; this module flattens a
fitted binary model into device arrays so ``sa_tree_predict`` (csrc/sa_trees.hip) evaluates it
where the features already are, and ``rate`` never copies the ~940 B/action of features to the
host. Supported producers:

* xgboost ``binary:logistic`` gbtree models, from their JSON model dump (``Booster.save_raw
  ('json')`` / ``save_model('*.json')``): float32 arithmetic, ``x < threshold`` goes left,
  missing values follow ``default_left`` (xgboost 1.6.2, the reference's pinned version
  (poetry.lock), is not installed here: this restates its documented prediction rule; the
  restatement in ``oracle/tree_oracle.py`` is the checker);
* scikit-learn ``HistGradientBoostingClassifier`` (binary, numeric splits): float64,
  ``x <= threshold`` goes left, NaN follows ``missing_go_to_left`` -- pinned against
  scikit-learn's own ``predict_proba``.
"""
from __future__ import annotations

import ctypes
import json
import os
from dataclasses import dataclass
from typing import List, Optional, Sequence

import numpy as np
import torch

from . import _native

NODE_DTYPE = np.dtype([('thr', '<f8'), ('feature', '<i4'), ('left', '<i4'), ('right', '<i4'),
                       ('pad', '<i4')])
assert NODE_DTYPE.itemsize == 24


@dataclass
class TreeEnsemble:
    """A binary gradient-boosted tree model in the flat node format of ``sa_tree_predict``."""

    nodes: np.ndarray            # NODE_DTYPE, absolute child indices, bit 31 of right = default_left
    roots: np.ndarray            # int32 [n_trees]
    n_features: int
    feature_names: Optional[List[str]]
    base_margin: float
    le: bool                     # True: x <= threshold goes left (scikit-learn)
    f32: bool                    # True: float32 arithmetic and output (xgboost)
    _dev: Optional[dict] = None

    # ------------------------------------------------------------------ constructors
    @classmethod
    def from_xgboost_json(cls, model, n_iterations: Optional[int] = None) -> 'TreeEnsemble':
        """From an xgboost JSON model (dict, JSON text/bytes, or a path to a .json file).
        ``n_iterations``: keep only the trees of the first n boosting rounds (what
        ``predict_proba`` evaluates after early stopping: ``iteration_range = (0,
        best_iteration + 1)``); None = every tree (``Booster.predict``'s default)."""
        if isinstance(model, (bytes, bytearray)):
            model = json.loads(model.decode())
        elif isinstance(model, str):
            if os.path.exists(model):
                with open(model) as f:
                    model = json.load(f)
            else:
                model = json.loads(model)
        learner = model['learner']
        obj = learner['objective']['name']
        if obj != 'binary:logistic':
            raise NotImplementedError(f'xgboost objective {obj!r} (binary:logistic only)')
        gb = learner['gradient_booster']
        if gb.get('name') != 'gbtree':
            raise NotImplementedError(f"xgboost booster {gb.get('name')!r} (gbtree only)")
        trees = gb['model']['trees']
        if n_iterations is not None:
            gparam = gb['model'].get('gbtree_model_param', {})
            per_iter = int(gparam.get('num_parallel_tree', 1) or 1)
            trees = trees[:max(0, int(n_iterations)) * per_iter]
        parts, roots, off = [], [], 0
        for t in trees:
            left = np.asarray(t['left_children'], np.int64)
            right = np.asarray(t['right_children'], np.int64)
            if any(int(s) != 0 for s in t.get('split_type', [])):
                raise NotImplementedError('categorical xgboost splits')
            m = len(left)
            nd = np.zeros(m, NODE_DTYPE)
            leaf = left < 0
            nd['thr'] = np.asarray(t['split_conditions'], np.float32).astype(np.float64)
            nd['feature'] = np.where(leaf, -1, np.asarray(t['split_indices'], np.int64))
            nd['left'] = np.where(leaf, 0, left + off)
            dl = np.asarray(t['default_left'], np.int64).astype(bool)
            r = np.where(leaf, 0, right + off).astype(np.int64)
            nd['right'] = np.where(dl & ~leaf, r | (1 << 31), r).astype(np.uint32).view(np.int32)
            parts.append(nd)
            roots.append(off)
            off += m
        param = learner['learner_model_param']
        p = np.float32(float(param['base_score']))
        base = float(np.float32(-np.log(np.float32(1.0) / p - np.float32(1.0))))
        names = learner.get('feature_names') or None
        nf = int(param.get('num_feature', 0))
        nodes = np.concatenate(parts) if parts else np.zeros(1, NODE_DTYPE)
        return cls(nodes, np.asarray(roots, np.int32), nf, list(names) if names else None, base,
                   le=False, f32=True)

    @classmethod
    def from_sklearn(cls, clf) -> 'TreeEnsemble':
        """From a fitted binary ``HistGradientBoostingClassifier``."""
        preds = getattr(clf, '_predictors', None)
        if preds is None or getattr(clf, 'n_trees_per_iteration_', 1) != 1:
            raise NotImplementedError('binary HistGradientBoostingClassifier models only')
        parts, roots, off = [], [], 0
        for it in preds:
            src = it[0].nodes
            if src['is_categorical'].any():
                raise NotImplementedError('categorical splits')
            m = len(src)
            nd = np.zeros(m, NODE_DTYPE)
            leaf = src['is_leaf'].astype(bool)
            nd['thr'] = np.where(leaf, src['value'], src['num_threshold'])
            nd['feature'] = np.where(leaf, -1, src['feature_idx'])
            nd['left'] = np.where(leaf, 0, src['left'].astype(np.int64) + off)
            r = np.where(leaf, 0, src['right'].astype(np.int64) + off).astype(np.int64)
            dl = src['missing_go_to_left'].astype(bool) & ~leaf
            nd['right'] = np.where(dl, r | (1 << 31), r).astype(np.uint32).view(np.int32)
            parts.append(nd)
            roots.append(off)
            off += m
        names = getattr(clf, 'feature_names_in_', None)
        return cls(np.concatenate(parts), np.asarray(roots, np.int32), int(clf.n_features_in_),
                   [str(x) for x in names] if names is not None else None,
                   float(np.asarray(clf._baseline_prediction).reshape(-1)[0]), le=True, f32=False)

    @classmethod
    def from_model(cls, model) -> Optional['TreeEnsemble']:
        """Any supported fitted learner -> TreeEnsemble; None when it is not supported (the
        caller then runs the learner's own host ``predict_proba``)."""
        try:
            if type(model).__name__ == 'HistGradientBoostingClassifier':
                return cls.from_sklearn(model)
            if hasattr(model, 'get_booster'):          # xgboost.XGBClassifier
                raw = json.loads(bytes(model.get_booster().save_raw('json')).decode())
                return cls.from_xgboost_json(raw, xgb_classifier_iterations(model, raw))
            if hasattr(model, 'save_raw'):             # xgboost.Booster
                return cls.from_xgboost_json(model.save_raw('json'))
            if isinstance(model, dict) and 'learner' in model:
                return cls.from_xgboost_json(model)
        except (NotImplementedError, KeyError, ValueError, TypeError, IndexError):
            return None  # a model layout this flattening does not know: host predict_proba
        return None

    # ------------------------------------------------------------------ evaluation
    @property
    def n_trees(self) -> int:
        return len(self.roots)

    def depths(self) -> np.ndarray:
        """Split levels on each tree's longest root-to-leaf path (int32 [n_trees])."""
        nd = self.nodes
        out = np.zeros(len(self.roots), np.int32)
        for t, r in enumerate(self.roots):
            stack, best = [(int(r), 0)], 0
            while stack:
                k, d = stack.pop()
                if nd['feature'][k] < 0:
                    best = max(best, d)
                else:
                    stack.append((int(nd['left'][k]), d + 1))
                    stack.append((int(nd['right'][k]) & 0x7FFFFFFF, d + 1))
            out[t] = best
        return out

    def _device(self, dev) -> dict:
        if self._dev is None or self._dev['dev'] != dev:
            self._dev = {'dev': dev,
                         'nodes': torch.from_numpy(self.nodes.view(np.uint8).copy()).to(dev),
                         'roots': torch.from_numpy(self.roots).to(dev),
                         'depth': torch.from_numpy(self.depths()).to(dev)}
        return self._dev

    def feature_slots(self, plan, feature_names: Optional[Sequence[str]] = None) -> np.ndarray:
        """(kind << 24) | column of every model feature in the blocks of ``plan``. The model's
        features are matched by name when it carries names, else by position in
        ``feature_names`` (default: the plan's own column order = the reference's
        ``feature_column_names``, vaep/features.py:20-59)."""
        where = {name: (kind, col) for name, kind, col in plan.order}
        names = self.feature_names or list(feature_names if feature_names is not None
                                           else plan.names)[:self.n_features]
        if len(names) < self.n_features:
            raise ValueError('the model has more features than the feature blocks')
        kinds = {'b': 0, 'f': 1, 'i': 2}
        slots = np.empty(len(names), np.int32)
        for f, name in enumerate(names):
            if name not in where:
                raise ValueError(f'{name} is not available in the features')
            kind, col = where[name]
            slots[f] = (kinds[kind] << 24) | col
        return slots

    def staged_layout(self, slots: np.ndarray):
        """The staged walk's model (sa_tree_predict_staged): ``(snodes, bool_cols, num_slots)``
        for the feature slots of one block layout. Split nodes refer to their feature as an index
        into the used bool columns, or (1 << 30) | index into the used numeric slots; leaves
        become self-loops (left = right = the leaf)."""
        nd = self.nodes
        n = len(nd)
        split = nd['feature'] >= 0
        fslot = np.full(n, -1, np.int64)
        fslot[split] = slots[nd['feature'][split]]
        kind = fslot >> 24
        bool_cols = np.unique(fslot[split & (kind == 0)] & 0xFFFFFF).astype(np.int32)
        num_slots = np.unique(fslot[split & (kind != 0)]).astype(np.int32)
        ref = np.zeros(n, np.int64)
        isb = split & (kind == 0)
        isn = split & (kind != 0)
        ref[isb] = np.searchsorted(bool_cols, fslot[isb] & 0xFFFFFF)
        ref[isn] = (1 << 30) | np.searchsorted(num_slots, fslot[isn])
        if not len(bool_cols):
            ref[~split] = 1 << 30  # leaves: any valid reference
        idx = np.arange(n)
        dt = np.dtype([('thr', '<f4'), ('ref', '<i4'), ('left', '<i4'), ('right', '<i4')]) \
            if self.f32 else \
            np.dtype([('thr', '<f8'), ('ref', '<i4'), ('left', '<i4'), ('right', '<i4'), ('pad', '<i4')])
        sn = np.zeros(n, dt)
        sn['thr'] = nd['thr'].astype(np.float32) if self.f32 else nd['thr']
        sn['ref'] = ref.astype(np.int32)
        sn['left'] = np.where(split, nd['left'], idx)
        sn['right'] = np.where(split, nd['right'], idx)
        return sn, bool_cols, num_slots

    def predict_blocks(self, blocks, feature_names: Optional[Sequence[str]] = None,
                       out: Optional[torch.Tensor] = None, staged: Optional[bool] = None) -> torch.Tensor:
        """P(class 1) of every row of the device feature blocks (``ops.FeatureBlocks``):
        float32 for xgboost models (as their ``predict_proba``), float64 for scikit-learn.
        ``staged`` (default: whenever the model's staged form fits LDS): the staged walk
        (sa_tree_predict_staged); False: the gather walk (sa_tree_predict)."""
        from .batch import stream_handle
        dev = blocks.bool_block.device
        d = self._device(dev)
        slots_np = self.feature_slots(blocks.plan, feature_names)
        n = blocks.n
        dt = torch.float32 if self.f32 else torch.float64
        if out is None:
            out = torch.empty(max(n, 1), dtype=dt, device=dev)
        bb, fb, ib = blocks.sa_blocks()
        if staged is not False and self.n_trees and d['depth'] is not None:
            key = ('staged', slots_np.tobytes())
            st = d.get(key)
            if st is None:
                sn, bc, ns = self.staged_layout(slots_np)
                lds = _native.lib().sa_tree_staged_lds_bytes(len(sn), len(bc), len(ns), int(self.f32))
                st = None if lds > 160 * 1024 else (
                    torch.from_numpy(sn.view(np.uint8).copy()).to(dev),
                    torch.from_numpy(bc).to(dev) if len(bc) else None, len(bc),
                    torch.from_numpy(ns).to(dev) if len(ns) else None, len(ns), len(sn))
                d[key] = st if st is not None else False
            if st:
                sn_t, bc_t, nbc, ns_t, nns, nnodes = st
                _native.check(_native.lib().sa_tree_predict_staged(
                    sn_t.data_ptr(), nnodes, d['roots'].data_ptr(), d['depth'].data_ptr(),
                    self.n_trees, bc_t.data_ptr() if bc_t is not None else None, nbc,
                    ns_t.data_ptr() if ns_t is not None else None, nns, ctypes.byref(bb),
                    ctypes.byref(fb), ctypes.byref(ib), n, float(self.base_margin), int(self.le),
                    int(self.f32), out.data_ptr(), stream_handle()))
                return out[:n]
            elif staged:
                raise ValueError('the staged form of this model does not fit LDS')
        slots = torch.from_numpy(slots_np).to(dev)
        _native.check(_native.lib().sa_tree_predict(
            d['nodes'].data_ptr(), len(self.nodes), d['roots'].data_ptr(),
            d['depth'].data_ptr() if (self.n_trees and d['depth'] is not None) else None,
            self.n_trees,
            slots.data_ptr(), len(slots), ctypes.byref(bb), ctypes.byref(fb), ctypes.byref(ib),
            n, float(self.base_margin), int(self.le), int(self.f32), out.data_ptr(),
            stream_handle()))
        return out[:n]


def xgb_classifier_iterations(model, raw: Optional[dict] = None) -> Optional[int]:
    """Boosting rounds ``XGBClassifier.predict_proba`` evaluates: ``best_iteration + 1`` after
    early stopping (xgboost 1.6 ``XGBModel._get_iteration_range``: the reference's default
    ``VAEP.fit`` passes ``early_stopping_rounds=10`` with an eval set, vaep/base.py:199-235),
    else every round (None).  Read from the estimator, or from the booster attributes the JSON
    model carries (``learner.attributes.best_iteration``)."""
    try:
        bi = model.best_iteration
    except Exception:  # xgboost raises AttributeError when early stopping did not run
        bi = None
    if bi is None and raw is not None:
        bi = raw.get('learner', {}).get('attributes', {}).get('best_iteration')
    if bi is None:
        return None
    return int(bi) + 1


def synthetic_xgboost_json(n_features: int, n_trees: int = 100, depth: int = 3, seed: int = 0,
                           feature_kinds: Optional[Sequence[str]] = None,
                           base_score: float = 0.5) -> dict:
    """An xgboost-1.6-shaped binary:logistic JSON model with random complete trees (the shape of
    the reference's default ``XGBClassifier(n_estimators=100, max_depth=3)``, vaep/base.py:
    226-231): used to benchmark and test the device path without xgboost installed. Splits on
    bool features use threshold 0.5 (the form xgboost learns for 0/1 columns)."""
    rng = np.random.default_rng(seed)
    trees = []
    for t in range(n_trees):
        n_int = 2 ** depth - 1
        m = 2 ** (depth + 1) - 1
        left = [-1] * m
        right = [-1] * m
        split_idx = [0] * m
        cond = [0.0] * m
        dleft = [0] * m
        for k in range(n_int):
            left[k], right[k] = 2 * k + 1, 2 * k + 2
            f = int(rng.integers(0, n_features))
            split_idx[k] = f
            kind = feature_kinds[f] if feature_kinds is not None else 'f'
            cond[k] = 0.5 if kind == 'b' else float(np.float32(rng.normal(0.0, 30.0)))
            dleft[k] = int(rng.integers(0, 2))
        for k in range(n_int, m):
            cond[k] = float(np.float32(rng.normal(0.0, 0.1)))
        trees.append({'left_children': left, 'right_children': right, 'split_indices': split_idx,
                      'split_conditions': cond, 'default_left': dleft, 'split_type': [0] * m,
                      'base_weights': cond, 'id': t})
    return {'learner': {
        'objective': {'name': 'binary:logistic'},
        'gradient_booster': {'name': 'gbtree', 'model': {'trees': trees,
                                                         'tree_info': [0] * n_trees}},
        'learner_model_param': {'base_score': repr(float(base_score)),
                                'num_feature': str(n_features), 'num_class': '0'},
        'feature_names': []}, 'version': [1, 6, 2]}


__all__ = ['TreeEnsemble', 'NODE_DTYPE', 'synthetic_xgboost_json', 'xgb_classifier_iterations']
