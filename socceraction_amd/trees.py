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

    def _split_outcomes(self, k: int):
        """(goes left on 0, goes left on 1) of split k as the producing library compares."""
        A = np.float32 if self.f32 else np.float64
        thr = A(self.nodes['thr'][k])
        if self.le:
            return bool(A(0) <= thr), bool(A(1) <= thr)
        return bool(A(0) < thr), bool(A(1) < thr)

    def conditions(self, slots: np.ndarray, bool_cols: set, num_keys: set) -> None:
        """Add the conditions of this model's splits (staged walk) to the two sets: bool block
        columns, and numeric (slot, threshold bytes, default_left) triples."""
        nd = self.nodes
        A = np.float32 if self.f32 else np.float64
        for k in np.nonzero(nd['feature'] >= 0)[0]:
            slot = int(slots[nd['feature'][k]])
            if slot >> 24 == 0:
                l0, l1 = self._split_outcomes(k)
                if l0 != l1:
                    bool_cols.add(slot & 0xFFFFFF)
            else:
                num_keys.add((slot, A(nd['thr'][k]).tobytes(), bool(int(nd['right'][k]) < 0)))

    def staged_nodes(self, slots: np.ndarray, bidx: dict, nidx: dict) -> dict:
        """This model's nodes for the staged condition walk, given the condition numbering
        (``bidx``: bool column -> condition, ``nidx``: numeric triple -> condition). Nodes are
        renumbered tree by tree so that a split's children are adjacent -- (child on a clear
        bit, child on a set bit) -- and stored as ``condition | first child << 16``; leaves are
        self-loops with condition 0 (never set); a bool split whose threshold sends 0 and 1 the
        same way is a condition-0 split whose first child is the one every row takes."""
        nd = self.nodes
        A = np.float32 if self.f32 else np.float64
        feat = nd['feature']
        cn = np.zeros(len(nd), np.uint32)
        leaf = np.zeros(len(nd), A)
        roots = np.empty(self.n_trees, np.int32)
        nxt = 0
        for t, r in enumerate(self.roots):
            roots[t] = nxt
            queue = [(int(r), nxt)]
            nxt += 1
            while queue:
                k, new = queue.pop(0)
                f = int(feat[k])
                if f < 0:
                    cn[new] = np.uint32(new) << np.uint32(16)
                    leaf[new] = A(nd['thr'][k])
                    continue
                left, right = int(nd['left'][k]), int(nd['right'][k]) & 0x7FFFFFFF
                slot = int(slots[f])
                if slot >> 24 == 0:
                    l0, l1 = self._split_outcomes(k)
                    cond = 0 if l0 == l1 else bidx[slot & 0xFFFFFF]
                    pair = (left, right) if l0 else (right, left)
                else:
                    cond = nidx[(slot, A(nd['thr'][k]).tobytes(), bool(int(nd['right'][k]) < 0))]
                    pair = (left, right)
                cn[new] = np.uint32(cond) | (np.uint32(nxt) << np.uint32(16))
                queue += [(pair[0], nxt), (pair[1], nxt + 1)]
                nxt += 2
        return {'nodes': cn[:nxt], 'leaf': leaf[:nxt], 'roots': roots}

    def staged_layout(self, slots: np.ndarray) -> dict:
        """The staged condition walk's model (sa_tree_predict_staged) of this model alone."""
        return staged_layout([self], [slots])

    def predict_blocks(self, blocks, feature_names: Optional[Sequence[str]] = None,
                       out: Optional[torch.Tensor] = None, staged: Optional[bool] = None,
                       method: Optional[str] = None) -> torch.Tensor:
        """P(class 1) of every row of the device feature blocks (``ops.FeatureBlocks``):
        float32 for xgboost models (as their ``predict_proba``), float64 for scikit-learn.
        ``method``: 'staged' (the staged condition walk, sa_tree_predict_staged; the default
        whenever the model fits LDS) or 'gather' (sa_tree_predict). ``staged`` True / False is
        the older spelling of the two."""
        from .batch import stream_handle
        if method is None and staged is not None:
            method = 'staged' if staged else 'gather'
        dev = blocks.device
        bits = getattr(blocks, 'bool_bits', None) if blocks.bool_block is None else None
        d = self._device(dev)
        slots_np = self.feature_slots(blocks.plan, feature_names)
        n = blocks.n
        dt = torch.float32 if self.f32 else torch.float64
        if out is None:
            out = torch.empty(max(n, 1), dtype=dt, device=dev)
        bb, fb, ib = blocks.sa_blocks()
        n32 = getattr(blocks, 'num32', False)
        if n32 and (not self.f32 or method == 'gather'):
            raise ValueError('float32 feature blocks feed the staged walk of xgboost learners only')
        if method != 'gather' and self.n_trees:
            key = ('staged', slots_np.tobytes())
            st = d.get(key)
            if st is None:
                lay = self.staged_layout(slots_np)
                lay.update(lay.pop('models')[0])
                n_cond = 1 + len(lay['bool_cols']) + len(lay['num_slots'])
                lds = _native.lib().sa_tree_staged_lds_bytes(len(lay['nodes']), n_cond, int(self.f32))
                fits = lds <= 160 * 1024 and n_cond <= 65536 and len(lay['nodes']) < 65536

                def t(v):
                    if not len(v):
                        return None
                    v = np.ascontiguousarray(v)
                    return torch.from_numpy(v.view(np.int32) if v.dtype == np.uint32 else v).to(dev)
                st = {k: t(v) for k, v in lay.items()} if fits else False
                if st:
                    st['n_num'] = len(lay['num_slots'])
                d[key] = st
            if st:
                def ptr(k):
                    return st[k].data_ptr() if st[k] is not None else None
                rec = _native.SaTreeModel(ptr('nodes'), ptr('leaf'), ptr('roots'), d['depth'].data_ptr(),
                                          st['nodes'].numel(), self.n_trees, float(self.base_margin),
                                          out.data_ptr())
                _native.check(_native.lib().sa_tree_predict_staged(
                    ctypes.byref(rec), ptr('bool_cols'),
                    0 if st['bool_cols'] is None else st['bool_cols'].numel(), ptr('num_cols'),
                    ptr('col_start'), 0 if st['num_cols'] is None else st['num_cols'].numel(),
                    ptr('num_thr'), ptr('num_dl'), st['n_num'], ctypes.byref(bb),
                    bits.data_ptr() if bits is not None else None,
                    bits.shape[1] * 8 if bits is not None else 0, ctypes.byref(fb),
                    ctypes.byref(ib), n, int(self.le), int(self.f32) | (2 if n32 else 0),
                    stream_handle()))
                return out[:n]
            elif method == 'staged' or n32:
                raise ValueError('the staged form of this model does not fit LDS')
        if bits is not None:  # the gather walk reads bool values from a bool block
            blocks._blk('b')
            bb, fb, ib = blocks.sa_blocks()
        slots = torch.from_numpy(slots_np).to(dev)
        _native.check(_native.lib().sa_tree_predict(
            d['nodes'].data_ptr(), len(self.nodes), d['roots'].data_ptr(),
            d['depth'].data_ptr() if (self.n_trees and d['depth'] is not None) else None,
            self.n_trees,
            slots.data_ptr(), len(slots), ctypes.byref(bb), ctypes.byref(fb), ctypes.byref(ib),
            n, float(self.base_margin), int(self.le), int(self.f32), out.data_ptr(),
            stream_handle()))
        return out[:n]


def _conditions_prep(plan, models: Sequence[TreeEnsemble], dev) -> dict:
    """Device tables of predict_pair_conditions for these learners on blocks of ``plan``, cached
    on the first learner (the entry holds the learners themselves, compared by identity)."""
    key = (tuple(plan.names), plan.n_bool, plan.n_f64, plan.n_i64, str(dev))
    cache = getattr(models[0], '_cond_cache', None)
    if cache is not None and cache['key'] == key and len(cache['models']) == len(models) and \
            all(a is b for a, b in zip(cache['models'], models)):
        return cache
    slots = [m.feature_slots(plan) for m in models]
    lay = staged_layout(models, slots)
    nb = plan.n_bool
    num_slots = lay['num_slots'].astype(np.int64)
    n_num = len(num_slots)
    kind, col = num_slots >> 24, num_slots & 0xFFFFFF
    fstart = np.searchsorted(np.where(kind == 1, col, 1 << 30), np.arange(plan.n_f64 + 1), 'left')
    istart = np.count_nonzero(kind == 1) + np.searchsorted(col[kind == 2], np.arange(plan.n_i64 + 1), 'left')
    t = lambda v, dt: torch.from_numpy(np.ascontiguousarray(v, dt)).to(dev)  # noqa: E731
    # the bitmap rows of the union's conditions: the used bool columns, then every numeric one
    rows_all = np.concatenate([lay['bool_cols'], nb + np.arange(n_num)]).astype(np.int32)
    walks = []
    for m, ml in zip(models, lay['models']):
        # each learner stages only the conditions ITS splits test (the union's other half is the
        # other learner's): its nodes renumbered to its own condition list
        cond = ml['nodes'] & 0xFFFF
        used = np.unique(cond[cond != 0])
        local = np.zeros(len(rows_all) + 1, np.uint32)
        local[used] = np.arange(1, len(used) + 1, dtype=np.uint32)
        nodes = (ml['nodes'] & np.uint32(0xFFFF0000)) | local[cond]
        rows_m = rows_all[used - 1].astype(np.int32)
        n_cond = 1 + len(rows_m)
        lds = _native.lib().sa_tree_staged_lds_bytes(len(nodes), n_cond, 1)
        if lds > 160 * 1024 or n_cond > 65536 or len(nodes) >= 65536:
            raise ValueError('the staged form of this model does not fit LDS')
        walks.append((t(nodes.view(np.int32), np.int32), t(ml['leaf'], np.float32),
                      t(ml['roots'], np.int32), m._device(dev)['depth'],
                      t(rows_m, np.int32) if len(rows_m) else None, len(rows_m)))
    cache = {'key': key, 'models': list(models), 'n_num': n_num, 'fstart': t(fstart, np.int32),
             'istart': t(istart, np.int32),
             'thr': t(lay['num_thr'] if n_num else np.zeros(1), np.float32),
             'dl': t(lay['num_dl'] if n_num else np.zeros(1), np.int32),
             'n_cond_union': len(rows_all), 'walks': walks}
    models[0]._cond_cache = cache
    return cache


def predict_pair_conditions(batch, plan, models: Sequence[TreeEnsemble], flip: bool = True):
    """``VAEP.rate``'s xgboost learners on ``batch`` through condition bitmaps: the union of
    their split conditions is evaluated inside the feature passes (``sa_vaep_features_conditions``:
    bool features and numeric split outcomes as bitmaps, the numeric values never written), then
    each learner's staged walk reads every condition as a bitmap (``sa_tree_predict_staged``,
    n_num = 0).  The same float32 probabilities as :meth:`TreeEnsemble.predict_blocks`, bit for
    bit.  Raises ValueError when a learner is not float32 (xgboost) or its walk does not fit LDS."""
    prep, bits, words = condition_bitmaps(batch, plan, models, flip)
    return [walk_conditions(prep, k, m, bits, words, batch.n, batch.device) for k, m in enumerate(models)]


def condition_bitmaps(batch, plan, models: Sequence[TreeEnsemble], flip: bool = True, bits=None):
    """predict_pair_conditions' first half: the feature passes writing the bool features and
    the union of the learners' numeric split outcomes as bitmaps (``sa_vaep_features_conditions``).
    Returns ``(prep, bits, words)``."""
    from .batch import stream_handle
    if not all(m.f32 and not m.le for m in models):
        raise ValueError('condition bitmaps are for xgboost (float32, `<`) learners')
    dev = batch.device
    prep = _conditions_prep(plan, models, dev)
    n, nb, n_num = batch.n, plan.n_bool, prep['n_num']
    words = max(2, -(-n // 128) * 2)  # int64 words per row: a whole number of 16-B runs
    if bits is None:
        bits = torch.empty((max(nb + n_num, 1), words), dtype=torch.int64, device=dev)
    s = batch.struct(flip=flip)
    _native.check(_native.lib().sa_vaep_features_conditions(
        ctypes.byref(s), ctypes.byref(plan.struct), bits.data_ptr(), words * 8, nb, plan.n_f64,
        plan.n_i64, prep['fstart'].data_ptr(), prep['istart'].data_ptr(), prep['thr'].data_ptr(),
        prep['dl'].data_ptr(), n_num, stream_handle()))
    return prep, bits, words


def walk_conditions(prep: dict, k: int, model: 'TreeEnsemble', bits: torch.Tensor, words: int,
                    n: int, dev, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Learner k's staged walk over the condition bitmaps ``bits`` (predict_pair_conditions'
    second half): it stages only its own conditions' bitmap rows."""
    from .batch import stream_handle
    z = _native.SaBlock()
    z.data, z.n_cols, z.tile_rows = None, 0, 16
    nodes, leaf, roots, depth, rows, n_rows = prep['walks'][k]
    out = torch.empty(max(n, 1), dtype=torch.float32, device=dev) if out is None else out
    rec = _native.SaTreeModel(nodes.data_ptr(), leaf.data_ptr(), roots.data_ptr(), depth.data_ptr(),
                              nodes.numel(), model.n_trees, float(model.base_margin), out.data_ptr())
    _native.check(_native.lib().sa_tree_predict_staged(
        ctypes.byref(rec), rows.data_ptr() if rows is not None else None, n_rows, None, None,
        0, None, None, 0, ctypes.byref(z), bits.data_ptr(), words * 8, ctypes.byref(z), ctypes.byref(z),
        n, 0, 1, stream_handle()))
    return out[:n]


def staged_layout(models: Sequence[TreeEnsemble], slots: Sequence[np.ndarray]) -> dict:
    """The staged condition walk's conditions for models evaluated on the same blocks -- 0 never
    set, then the used bool columns, then the distinct numeric (slot, threshold, default
    direction) triples in slot order -- and each model's renumbered nodes."""
    A = np.float32 if models[0].f32 else np.float64
    bset: set = set()
    nset: set = set()
    for te, sl in zip(models, slots):
        te.conditions(sl, bset, nset)
    bool_cols = np.array(sorted(bset), np.int32)
    bidx = {c: 1 + i for i, c in enumerate(bool_cols.tolist())}
    keys = sorted(nset)
    nidx = {key: 1 + len(bool_cols) + i for i, key in enumerate(keys)}
    num_slots = np.array([key[0] for key in keys], np.int32)
    num_cols, first = np.unique(num_slots, return_index=True)
    return {'bool_cols': bool_cols, 'num_slots': num_slots, 'num_cols': num_cols.astype(np.int32),
            'col_start': np.append(first, len(num_slots)).astype(np.int32),
            'num_thr': np.array([np.frombuffer(key[1], A)[0] for key in keys], A),
            'num_dl': np.array([int(key[2]) for key in keys], np.int32),
            'models': [te.staged_nodes(sl, bidx, nidx) for te, sl in zip(models, slots)]}


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


__all__ = ['TreeEnsemble', 'NODE_DTYPE', 'staged_layout', 'synthetic_xgboost_json',
           'xgb_classifier_iterations']
