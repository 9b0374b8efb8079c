"""CPU oracle (numpy restatement) of binary gradient-boosted tree prediction.

TEST INFRASTRUCTURE ONLY (see ``oracle/__init__.py``). The reference's VAEP learners
(vaep/base.py:199-282: xgboost by default, catboost, lightgbm) are not installed here. This
restates xgboost's documented prediction for a ``binary:logistic`` gbtree JSON model (the
reference pins xgboost 1.6.2, poetry.lock): every tree is walked from its root -- a node goes
to ``left_children`` when ``float32(x) < split_condition`` and to ``right_children``
otherwise, a missing (NaN) value follows ``default_left`` -- the leaf values
(``split_conditions`` of a leaf) are added in tree order onto the float32 base margin
``-log(1/base_score - 1)``, and ``predict_proba[:, 1] = 1 / (1 + exp(-margin))`` in float32.
"Parity unpinned" against xgboost itself (absent): the restatement is parsed independently of
the product's loader. The same walk with ``x <= threshold`` in float64 is pinned against
scikit-learn's ``HistGradientBoostingClassifier.predict_proba`` in ``tests/test_oracle.py``.
"""
from __future__ import annotations

import numpy as np


def _walk(X, left, right, feat, cond, dleft, lt: bool, dtype):
    n = X.shape[0]
    node = np.zeros(n, np.int64)
    while True:
        leaf = left[node] < 0
        if leaf.all():
            return cond[node].astype(dtype)
        k = node[~leaf]
        v = X[np.flatnonzero(~leaf), feat[k]].astype(dtype)
        thr = cond[k].astype(dtype)
        go_left = np.where(np.isnan(v), dleft[k], (v < thr) if lt else (v <= thr))
        node[~leaf] = np.where(go_left, left[k], right[k])


def predict_xgboost_json(model: dict, X: np.ndarray) -> np.ndarray:
    """P(class 1), float32, of an xgboost binary:logistic gbtree JSON model on rows X."""
    learner = model['learner']
    assert learner['objective']['name'] == 'binary:logistic'
    p = np.float32(float(learner['learner_model_param']['base_score']))
    margin = np.full(X.shape[0], np.float32(-np.log(np.float32(1.0) / p - np.float32(1.0))),
                     np.float32)
    for t in learner['gradient_booster']['model']['trees']:
        leaf = _walk(X, np.asarray(t['left_children']), np.asarray(t['right_children']),
                     np.asarray(t['split_indices']),
                     np.asarray(t['split_conditions'], np.float32),
                     np.asarray(t['default_left']).astype(bool), True, np.float32)
        margin = (margin + leaf).astype(np.float32)
    return (np.float32(1.0) / (np.float32(1.0) + np.exp(-margin))).astype(np.float32)


def predict_sklearn_nodes(clf, X: np.ndarray) -> np.ndarray:
    """The same walk over a HistGradientBoostingClassifier's nodes (x <= threshold, float64,
    expit) -- checked against the estimator's own predict_proba."""
    margin = np.full(X.shape[0], float(np.asarray(clf._baseline_prediction).reshape(-1)[0]))
    for it in clf._predictors:
        nd = it[0].nodes
        leaf = nd['is_leaf'].astype(bool)
        left = np.where(leaf, -1, nd['left'].astype(np.int64))
        cond = np.where(leaf, nd['value'], nd['num_threshold'])
        margin = margin + _walk(X, left, nd['right'].astype(np.int64), nd['feature_idx'], cond,
                                nd['missing_go_to_left'].astype(bool), False, np.float64)
    return 1.0 / (1.0 + np.exp(-margin))
