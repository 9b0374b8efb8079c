"""The VAEP framework on MI355X (drop-in for ``socceraction.vaep.base``).

``compute_features`` / ``compute_labels`` / ``rate`` keep the reference's per-game
signatures (vaep/base.py:97-137, 296-333) but run as one fused launch each: the game's
actions are flattened once into HBM columns and every known transformer in ``xfns`` is
computed by ``sa_vaep_features`` (windowed game states + left-to-right flip in-kernel).
The ``*_batch`` variants value many games per launch (one segment per game), which is
the throughput path the benchmark measures. ``fit`` / ``score`` delegate to the same
gradient-boosting learners as the reference (host-side, out of the kernel path).
"""
from __future__ import annotations

import math
from typing import Any, Dict, List, Optional, Tuple

import numpy as np
import pandas as pd
from sklearn.exceptions import NotFittedError
from sklearn.metrics import brier_score_loss, roc_auc_score

from .. import catalog, ops
from .. import spadl as spadlcfg
from ..batch import ActionBatch
from . import features as fs
from . import formula as vaep
from . import labels as lab

try:
    import xgboost
except ImportError:
    xgboost = None  # type: ignore
try:
    import catboost
except ImportError:
    catboost = None  # type: ignore
try:
    import lightgbm
except ImportError:
    lightgbm = None  # type: ignore

xfns_default = [
    fs.actiontype_onehot,
    fs.result_onehot,
    fs.actiontype_result_onehot,
    fs.bodypart_onehot,
    fs.time,
    fs.startlocation,
    fs.endlocation,
    fs.startpolar,
    fs.endpolar,
    fs.movement,
    fs.team,
    fs.time_delta,
    fs.space_delta,
    fs.goalscore,
]


class VAEP:
    """Valuing Actions by Estimating Probabilities (reference vaep/base.py:55-366).

    Parameters
    ----------
    xfns : list
        Feature transformers (default :data:`xfns_default`). Known transformers run in
        the fused HIP kernel; any other callable is evaluated on host game states.
    nb_prev_actions : int, default=3
        Number of previous actions in a game state (1..8 on this backend).
    """

    _spadlcfg = spadlcfg
    _fs = fs
    _lab = lab
    _vaep = vaep
    _atomic = False

    def __init__(self, xfns: Optional[List[Any]] = None, nb_prev_actions: int = 3) -> None:
        self.__models: Dict[str, Any] = {}
        self.xfns = xfns_default if xfns is None else xfns
        self.yfns = [self._lab.scores, self._lab.concedes]
        self.nb_prev_actions = nb_prev_actions

    # ---------------------------------------------------------------- features
    def _split_xfns(self) -> Tuple[List[str], List[Tuple[int, Any]]]:
        known, unknown = [], []
        for i, f in enumerate(self.xfns):
            x = self._fs.xfn_name(f, self._atomic)
            if x is None:
                unknown.append((i, f))
            else:
                known.append(x)
        return known, unknown

    def _host_gamestates(self, actions_with_names: pd.DataFrame, home_team_id):
        gs = self._fs.gamestates(actions_with_names.copy(), self.nb_prev_actions)
        return self._fs.play_left_to_right(gs, home_team_id)

    def _features_frame(self, ab: ActionBatch, actions: pd.DataFrame, homes, segments):
        known, unknown = self._split_xfns()
        parts: Dict[int, pd.DataFrame] = {}
        if known:
            fb = ops.features(ab, known, self.nb_prev_actions)
            kdf = fb.to_frame(index=pd.RangeIndex(ab.n))
        if unknown:  # user transformers: reference semantics on host game states
            named = self._spadlcfg.add_names(actions)
            for i, f in unknown:
                outs = []
                for (s, e), home in zip(segments, homes):
                    gs = self._host_gamestates(named.iloc[s:e].reset_index(drop=True), home)
                    outs.append(f(gs))
                parts[i] = pd.concat(outs, ignore_index=True) if outs else pd.DataFrame()
        if not unknown:
            return kdf
        frames, pos = [], 0
        for i, f in enumerate(self.xfns):
            if i in parts:
                frames.append(parts[i])
            else:
                ncols = len(catalog.xfn_columns(self._fs.xfn_name(f, self._atomic),
                                                self.nb_prev_actions, self._atomic))
                frames.append(kdf.iloc[:, pos:pos + ncols])
                pos += ncols
        return pd.concat(frames, axis=1)

    def compute_features(self, game: pd.Series, game_actions: pd.DataFrame) -> pd.DataFrame:
        """Feature representation of every game state of one game (vaep/base.py:97-116)."""
        home = game.home_team_id
        ab = ActionBatch.from_frame(game_actions, atomic=self._atomic, home_team_id=home)
        return self._features_frame(ab, game_actions, [home], [(0, len(game_actions))])

    def compute_features_batch(self, games: pd.DataFrame, actions: pd.DataFrame) -> pd.DataFrame:
        """Features of many games at once.

        ``actions`` holds the games' actions with each game's rows contiguous;
        ``games`` maps ``game_id -> home_team_id``. Equals ``pd.concat`` of the per-game
        :meth:`compute_features` outputs with ``ignore_index=True``.  With built-in
        transformers only, the pipelined path of :meth:`compute_batch` (features only); with a
        user transformer, one launch for the known ones and the host for the rest.
        """
        if len(actions) and not self._split_xfns()[1]:
            # every transformer a known one: the pipelined path (game-aligned chunks, copies out
            # overlapping the next chunk's encode; socceraction_amd.pipeline), the same frame
            from ..pipeline import value_frames
            return value_frames(self, games, actions, labels=False)[0]
        home_of = games.set_index('game_id')['home_team_id']
        ab = ActionBatch.from_frame(actions, atomic=self._atomic, home_team_id=home_of,
                                    segments='game')
        off = ab.cols['seg_off'].cpu().numpy()
        gids = actions['game_id'].to_numpy()[off[:-1]] if len(actions) else []
        homes = list(home_of.loc[gids]) if len(gids) else []  # one vectorised lookup
        return self._features_frame(ab, actions, homes, list(zip(off[:-1], off[1:])))

    # ---------------------------------------------------------------- labels
    def _labels_frame(self, actions: pd.DataFrame, segments: str) -> pd.DataFrame:
        known = {self._lab.scores: 'scores', self._lab.concedes: 'concedes',
                 self._lab.goal_from_shot: 'goal_from_shot'}
        if all(f in known for f in self.yfns):
            n = len(actions)
            out = {}
            if n:
                ab = ActionBatch.from_frame(actions, atomic=self._atomic, segments=segments)
                lb = ops.labels(ab)
                for f in self.yfns:
                    col = 'goal' if (self._atomic and known[f] == 'goal_from_shot') else known[f]
                    out[col] = getattr(lb, known[f])[:n].cpu().numpy().view(bool)
            else:
                out = {known[f]: np.zeros(0, bool) for f in self.yfns}
            return pd.DataFrame(out, index=pd.RangeIndex(n))
        named = self._spadlcfg.add_names(actions)
        if segments == 'single':
            return pd.concat([fn(named) for fn in self.yfns], axis=1)
        outs = []
        for _, g in named.groupby('game_id', sort=False):
            g = g.reset_index(drop=True)
            outs.append(pd.concat([fn(g) for fn in self.yfns], axis=1))
        return pd.concat(outs, ignore_index=True)

    def compute_labels(self, game: pd.Series, game_actions: pd.DataFrame) -> pd.DataFrame:
        """Labels of every game state of one game (vaep/base.py:118-137)."""
        return self._labels_frame(game_actions, 'single')

    def compute_labels_batch(self, games: pd.DataFrame, actions: pd.DataFrame) -> pd.DataFrame:
        """Labels of many games (contiguous per game) in one launch."""
        return self._labels_frame(actions, 'game')

    def compute_batch(self, games: pd.DataFrame, actions: pd.DataFrame,
                      p_scores=None, p_concedes=None, chunk_rows: int = 1 << 18):
        """``(compute_features_batch, compute_labels_batch, formula values)`` of the same
        games from ONE encode of the frame, pipelined over game-aligned chunks so the host
        encodes the next chunk while the DMA engine copies the last one out
        (:mod:`socceraction_amd.pipeline`).  ``p_scores`` / ``p_concedes``: one probability per
        action (e.g. a fitted model's), else the values are None.  Built-in transformers and
        label functions only."""
        from ..pipeline import value_frames
        return value_frames(self, games, actions, p_scores, p_concedes, chunk_rows)

    # ---------------------------------------------------------------- learning (host)
    def fit(self, X: pd.DataFrame, y: pd.DataFrame, learner: str = 'xgboost',
            val_size: float = 0.25, tree_params: Optional[Dict[str, Any]] = None,
            fit_params: Optional[Dict[str, Any]] = None) -> 'VAEP':
        """Fit one classifier per label (reference vaep/base.py:139-213)."""
        nb_states = len(X)
        idx = np.random.permutation(nb_states)
        train_idx = idx[:math.floor(nb_states * (1 - val_size))]
        val_idx = idx[(math.floor(nb_states * (1 - val_size)) + 1):]
        cols = self._fs.feature_column_names(self.xfns, self.nb_prev_actions)
        if not set(cols).issubset(set(X.columns)):
            missing_cols = ' and '.join(set(cols).difference(X.columns))
            raise ValueError(f'{missing_cols} are not available in the features dataframe')
        X_train, y_train = X.iloc[train_idx][cols], y.iloc[train_idx]
        X_val, y_val = X.iloc[val_idx][cols], y.iloc[val_idx]
        for col in list(y.columns):
            eval_set = [(X_val, y_val[col])] if val_size > 0 else None
            if learner == 'xgboost':
                self.__models[col] = self._fit_xgboost(X_train, y_train[col], eval_set,
                                                       tree_params, fit_params)
            elif learner == 'catboost':
                self.__models[col] = self._fit_catboost(X_train, y_train[col], eval_set,
                                                        tree_params, fit_params)
            elif learner == 'lightgbm':
                self.__models[col] = self._fit_lightgbm(X_train, y_train[col], eval_set,
                                                        tree_params, fit_params)
            else:
                raise ValueError(f'A {learner} learner is not supported')
        return self

    def _fit_xgboost(self, X, y, eval_set=None, tree_params=None, fit_params=None):
        if xgboost is None:
            raise ImportError('xgboost is not installed.')
        if tree_params is None:
            tree_params = dict(n_estimators=100, max_depth=3)
        if fit_params is None:
            fit_params = dict(eval_metric='auc', verbose=True)
        if eval_set is not None:
            fit_params = {**fit_params, **dict(early_stopping_rounds=10, eval_set=eval_set)}
        return xgboost.XGBClassifier(**tree_params).fit(X, y, **fit_params)

    def _fit_catboost(self, X, y, eval_set=None, tree_params=None, fit_params=None):
        if catboost is None:
            raise ImportError('catboost is not installed.')
        if tree_params is None:
            tree_params = dict(eval_metric='BrierScore', loss_function='Logloss', iterations=100)
        if fit_params is None:
            is_cat_feature = [c.dtype.name == 'category' for (_, c) in X.items()]
            fit_params = dict(cat_features=np.nonzero(is_cat_feature)[0].tolist(), verbose=True)
        if eval_set is not None:
            fit_params = {**fit_params, **dict(early_stopping_rounds=10, eval_set=eval_set)}
        return catboost.CatBoostClassifier(**tree_params).fit(X, y, **fit_params)

    def _fit_lightgbm(self, X, y, eval_set=None, tree_params=None, fit_params=None):
        if lightgbm is None:
            raise ImportError('lightgbm is not installed.')
        if tree_params is None:
            tree_params = dict(n_estimators=100, max_depth=3)
        if fit_params is None:
            fit_params = dict(eval_metric='auc', verbose=True)
        if eval_set is not None:
            fit_params = {**fit_params, **dict(early_stopping_rounds=10, eval_set=eval_set)}
        return lightgbm.LGBMClassifier(**tree_params).fit(X, y, **fit_params)

    def _estimate_probabilities(self, X: pd.DataFrame) -> pd.DataFrame:
        """predict_proba[:, 1] of each fitted model (reference vaep/base.py:284-294)."""
        cols = self._fs.feature_column_names(self.xfns, self.nb_prev_actions)
        if not set(cols).issubset(set(X.columns)):
            missing_cols = ' and '.join(set(cols).difference(X.columns))
            raise ValueError(f'{missing_cols} are not available in the features dataframe')
        Y_hat = pd.DataFrame()
        for col in self.__models:
            Y_hat[col] = [p[1] for p in self.__models[col].predict_proba(X[cols])]
        return Y_hat

    # ---------------------------------------------------------------- rating
    def _device_models(self):
        """The fitted learners as device tree ensembles (socceraction_amd.trees) when every
        one is a supported binary tree model and every transformer is a known one; else None
        (rate then runs the reference's host predict_proba)."""
        from ..trees import TreeEnsemble
        if not {'scores', 'concedes'} <= set(self.__models) or self._split_xfns()[1]:
            return None
        # the cache holds the model objects themselves (compared by identity), so a replaced
        # model can never be mistaken for the cached one through a reused id()
        key = tuple(self.__models.items())
        cached = getattr(self, '_trees_cache', None)
        if cached is not None and len(cached[0]) == len(key) and all(
                c0 == c1 and m0 is m1 for (c0, m0), (c1, m1) in zip(cached[0], key)):
            return cached[1]
        trees = {c: TreeEnsemble.from_model(m) for c, m in self.__models.items()}
        res = trees if all(t is not None for t in trees.values()) else None
        self._trees_cache = (key, res)
        return res

    def _rate_device(self, ab: ActionBatch, trees) -> pd.DataFrame:
        """features -> predict_proba -> formula without leaving HBM; only the three value
        columns are copied back. The probability dtype is the learner's (float32 for
        xgboost, float64 for scikit-learn), as in the reference's host path."""
        import torch
        known, _ = self._split_xfns()
        # the learners read the bool features as bitmaps (64 instead of 515 B/action written);
        # xgboost learners compare float32 values, so their numeric features are written and
        # staged in float32 (half the bytes, the same probabilities bit for bit); better still,
        # their split conditions are evaluated in the numeric pass and only bitmaps are written
        n32 = self.nb_prev_actions <= 3 and all(t.f32 for t in trees.values())
        ps = pc = None
        if n32 and not any(t.le for t in trees.values()):  # xgboost learners: their split conditions evaluated inside the feature passes
            from ..trees import predict_pair_conditions
            try:
                plan = ops.build_plan(known, self.nb_prev_actions, ab.atomic)
                ps, pc = predict_pair_conditions(ab, plan, [trees['scores'], trees['concedes']])
            except ValueError:
                ps = pc = None
        if ps is None and n32:  # float32 numeric blocks, the staged walk over them
            fb = ops.features(ab, known, self.nb_prev_actions, bool_bits=True, num32=True)
            try:
                ps = trees['scores'].predict_blocks(fb)
                pc = trees['concedes'].predict_blocks(fb)
            except ValueError:
                ps = pc = None
        if ps is None:  # a learner whose staged form does not fit LDS: the gather walk, float64 blocks
            fb = ops.features(ab, known, self.nb_prev_actions, bool_bits=True)
            ps = trees['scores'].predict_blocks(fb)
            pc = trees['concedes'].predict_blocks(fb)
        if ps.dtype != pc.dtype:  # pandas would upcast the mixed pair
            ps, pc = ps.to(torch.float64), pc.to(torch.float64)
        v = ops.formula(ab, ps, pc).cpu().numpy()[:, :ab.n]
        return pd.DataFrame({'offensive_value': v[0], 'defensive_value': v[1],
                             'vaep_value': v[2]})

    def rate(self, game: pd.Series, game_actions: pd.DataFrame,
             game_states: Optional[pd.DataFrame] = None) -> pd.DataFrame:
        """VAEP values of one game's actions (reference vaep/base.py:296-333). Supported
        tree learners (xgboost JSON-dumpable boosters, scikit-learn HistGradientBoosting)
        are evaluated on the device feature blocks when ``game_states`` is not given."""
        if not self.__models:
            raise NotFittedError()
        actions = self._spadlcfg.add_names(game_actions)
        if game_states is None:
            trees = self._device_models()
            if trees is not None:
                ab = ActionBatch.from_frame(game_actions, atomic=self._atomic,
                                            home_team_id=game.home_team_id)
                return self._rate_device(ab, trees)
            game_states = self.compute_features(game, game_actions)
        y_hat = self._estimate_probabilities(game_states)
        return self._vaep.value(actions, y_hat.scores, y_hat.concedes)

    def rate_batch(self, games: pd.DataFrame, actions: pd.DataFrame,
                   game_states: Optional[pd.DataFrame] = None) -> pd.DataFrame:
        """VAEP values of many games (contiguous per game): one feature launch, one host
        ``predict_proba`` per model, one formula launch with per-game segments."""
        if not self.__models:
            raise NotFittedError()
        if game_states is None:
            trees = self._device_models()
            if trees is not None:
                home_of = games.set_index('game_id')['home_team_id']
                ab = ActionBatch.from_frame(actions, atomic=self._atomic, home_team_id=home_of,
                                            segments='game')
                return self._rate_device(ab, trees)
            game_states = self.compute_features_batch(games, actions)
        y_hat = self._estimate_probabilities(game_states)
        n = len(actions)
        ps = np.asarray(y_hat.scores.to_numpy())
        pc = np.asarray(y_hat.concedes.to_numpy())
        dt = np.float32 if (ps.dtype == np.float32 and pc.dtype == np.float32) else np.float64
        import torch
        ab = ActionBatch.from_frame(actions, atomic=self._atomic, segments='game')
        out = ops.formula(ab, torch.from_numpy(np.ascontiguousarray(ps, dt)).to(ab.device),
                          torch.from_numpy(np.ascontiguousarray(pc, dt)).to(ab.device))
        v = out.cpu().numpy()[:, :n]
        return pd.DataFrame({'offensive_value': v[0], 'defensive_value': v[1], 'vaep_value': v[2]})

    def score(self, X: pd.DataFrame, y: pd.DataFrame) -> Dict[str, Dict[str, float]]:
        """Brier score and AUROC per label (reference vaep/base.py:335-366)."""
        if not self.__models:
            raise NotFittedError()
        y_hat = self._estimate_probabilities(X)
        scores: Dict[str, Dict[str, float]] = {}
        for col in self.__models:
            scores[col] = {}
            scores[col]['brier'] = brier_score_loss(y[col], y_hat[col])
            scores[col]['auroc'] = roc_auc_score(y[col], y_hat[col])
        return scores
