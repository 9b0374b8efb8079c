"""Seeded synthetic SPADL / Atomic-SPADL action sets (host-side, numpy, vectorised).

This is the generator behind the benchmark configurations of ``BASELINE.json``
(SURVEY.md §8(d) "Synthetic inputs"). It is *not* derived from reference code:
the reference ships no generator. Shapes follow the survey's spec:

* actions per game ``n_g = clip(round(N(1600, 120)), 1200, 2000)`` (atomic: ~4000);
* home team ``2g``, away ``2g+1``; possession switches with probability 0.2;
* two periods split at ``n_g // 2``; ``time_seconds`` is a cumulative Exp(3.4 s)
  that restarts per period (≈5 % of gaps exceed the formula's 10 s rule);
* a World-Cup-like type mix (pass .50, dribble .33, the rest over every id),
  shots biased towards goal, ~12 % of shots scored, ~1 % owngoals, cards on fouls,
  offsides on passes, plus ``bad_touch``+owngoal rows that must *not* count;
* ~0.1 % exact edge coordinates (0, 105, 68, goal centre, dx = 0) so that the
  ``arctan`` inf/NaN branches are exercised.

Everything is returned as a dict of flat numpy columns plus ``game_off`` (int64
``[n_games+1]``) and per-game ``home_team_id``; :func:`to_frame` turns it into a
reference-shaped pandas DataFrame.
"""
from __future__ import annotations

from typing import Dict

import numpy as np
import pandas as pd

FIELD_L = 105.0
FIELD_W = 68.0

_SPADL_TYPE_P = np.full(23, 0.0)
_SPADL_TYPE_P[0] = 0.50   # pass
_SPADL_TYPE_P[21] = 0.33  # dribble
_rest = [i for i in range(23) if i not in (0, 21)]
_SPADL_TYPE_P[_rest] = 0.17 / len(_rest)
# shots a bit more common than the flat remainder, so goals occur in every game
_SPADL_TYPE_P[11] += 0.012
_SPADL_TYPE_P /= _SPADL_TYPE_P.sum()

_ATOMIC_TYPE_P = np.full(33, 0.0)
_ATOMIC_TYPE_P[0] = 0.30   # pass
_ATOMIC_TYPE_P[21] = 0.20  # dribble
_ATOMIC_TYPE_P[23] = 0.27  # receival
_arest = [i for i in range(33) if i not in (0, 21, 23, 27, 28)]
_ATOMIC_TYPE_P[_arest] = 0.23 / len(_arest)
_ATOMIC_TYPE_P /= _ATOMIC_TYPE_P.sum()


def _game_sizes(rng: np.random.Generator, n_games: int, mean: float, sd: float,
                lo: int, hi: int) -> np.ndarray:
    n = np.clip(np.round(rng.normal(mean, sd, n_games)), lo, hi).astype(np.int64)
    return n


def _segment_ids(game_off: np.ndarray) -> np.ndarray:
    n = int(game_off[-1])
    seg = np.zeros(n, dtype=np.int64)
    if len(game_off) > 2:
        seg[game_off[1:-1]] = 1
    return np.cumsum(seg)


def _common(rng: np.random.Generator, sizes: np.ndarray, game_id0: int = 0) -> Dict[str, np.ndarray]:
    n_games = len(sizes)
    game_off = np.zeros(n_games + 1, dtype=np.int64)
    np.cumsum(sizes, out=game_off[1:])
    n = int(game_off[-1])
    g = _segment_ids(game_off)
    pos = np.arange(n, dtype=np.int64) - game_off[g]
    # possession: random start per game, switch w.p. 0.2 per action
    switch = rng.random(n) < 0.2
    switch[game_off[:-1]] = False
    start = rng.integers(0, 2, n_games)
    cs = np.cumsum(switch.astype(np.int64))
    cs -= cs[game_off[:-1]][g]
    side = (cs + start[g]) & 1
    gid = np.arange(game_id0, game_id0 + n_games, dtype=np.int64)
    team_id = 2 * gid[g] + side
    home_team_id = 2 * gid
    half = sizes // 2
    period_id = np.where(pos < half[g], 1, 2).astype(np.int64)
    # time: cumulative Exp(3.4) restarting per period
    gap = rng.exponential(3.4, n)
    pstart = (pos == 0) | (pos == half[g])
    gap[pstart] = 0.0
    seg2 = np.cumsum(pstart.astype(np.int64)) - 1
    csum = np.cumsum(gap)
    base = np.zeros(seg2[-1] + 1 if n else 0)
    if n:
        first_idx = np.flatnonzero(pstart)
        base = csum[first_idx]
        t = csum - base[seg2]
    else:
        t = csum
    return dict(game_off=game_off, game_id=gid[g], team_id=team_id,
                home_team_id=home_team_id, period_id=period_id,
                time_seconds=np.round(t, 3), seg=g, pos=pos)


def _edges(rng: np.random.Generator, x: np.ndarray, y: np.ndarray, frac: float = 0.001) -> None:
    n = len(x)
    m = rng.random(n) < frac
    idx = np.flatnonzero(m)
    choice = rng.integers(0, 5, len(idx))
    for c, vx, vy in ((0, 0.0, None), (1, FIELD_L, None), (2, None, FIELD_W),
                      (3, FIELD_L, FIELD_W / 2), (4, FIELD_L, 0.0)):
        sel = idx[choice == c]
        if vx is not None:
            x[sel] = vx
        if vy is not None:
            y[sel] = vy


def spadl_games(n_games: int, seed: int = 20250223, mean_actions: float = 1600.0,
                game_id0: int = 0) -> Dict[str, np.ndarray]:
    """Generate ``n_games`` synthetic SPADL games as flat columns."""
    rng = np.random.default_rng([seed, n_games, game_id0])
    sizes = _game_sizes(rng, n_games, mean_actions, 120.0 * mean_actions / 1600.0,
                        int(1200 * mean_actions / 1600), int(2000 * mean_actions / 1600))
    sizes = np.maximum(sizes, 1)
    d = _common(rng, sizes, game_id0)
    n = int(d['game_off'][-1])
    type_id = rng.choice(23, size=n, p=_SPADL_TYPE_P).astype(np.int64)
    result_id = (rng.random(n) < 0.8).astype(np.int64)  # success .8 / fail .2
    is_shot = (type_id == 11) | (type_id == 12) | (type_id == 13)
    u = rng.random(n)
    result_id[is_shot] = np.where(u[is_shot] < 0.12, 1,
                                  np.where(u[is_shot] < 0.13, 3, 0))
    pen = type_id == 12
    result_id[pen] = np.where(u[pen] < 0.75, 1, 0)
    bad = type_id == 19
    result_id[bad] = np.where(u[bad] < 0.05, 3, 0)   # bad_touch + owngoal (must not count)
    foul = type_id == 8
    result_id[foul] = np.where(u[foul] < 0.15, 4, np.where(u[foul] < 0.17, 5, 0))
    passes = type_id == 0
    off = passes & (rng.random(n) < 0.01)
    result_id[off] = 2
    bodypart_id = rng.choice(4, size=n, p=[0.85, 0.10, 0.04, 0.01]).astype(np.int64)
    sx = rng.uniform(0, FIELD_L, n)
    sy = rng.uniform(0, FIELD_W, n)
    nsh = int(is_shot.sum())
    sx[is_shot] = FIELD_L - np.abs(rng.normal(0, 12, nsh))
    sy[is_shot] = rng.normal(FIELD_W / 2, 8, nsh)
    ex = sx + rng.normal(5, 15, n)
    ey = sy + rng.normal(0, 12, n)
    ex[is_shot] = FIELD_L
    ey[is_shot] = FIELD_W / 2 + rng.normal(0, 2, nsh)
    sx = np.clip(sx, 0, FIELD_L)
    sy = np.clip(sy, 0, FIELD_W)
    ex = np.clip(ex, 0, FIELD_L)
    ey = np.clip(ey, 0, FIELD_W)
    _edges(rng, sx, sy)
    _edges(rng, ex, ey)
    still = rng.random(n) < 0.001  # dx = dy = 0
    ex[still] = sx[still]
    ey[still] = sy[still]
    d.update(type_id=type_id, result_id=result_id, bodypart_id=bodypart_id,
             start_x=np.round(sx, 4), start_y=np.round(sy, 4),
             end_x=np.round(ex, 4), end_y=np.round(ey, 4))
    return d


def atomic_games(n_games: int, seed: int = 20250223, mean_actions: float = 4000.0,
                 game_id0: int = 0) -> Dict[str, np.ndarray]:
    """Generate ``n_games`` synthetic Atomic-SPADL games as flat columns."""
    rng = np.random.default_rng([seed, n_games, game_id0, 1])
    sizes = _game_sizes(rng, n_games, mean_actions, 300.0 * mean_actions / 4000.0,
                        int(3000 * mean_actions / 4000), int(5000 * mean_actions / 4000))
    sizes = np.maximum(sizes, 1)
    d = _common(rng, sizes, game_id0)
    n = int(d['game_off'][-1])
    type_id = rng.choice(33, size=n, p=_ATOMIC_TYPE_P).astype(np.int64)
    # after some shots insert a goal (27) or owngoal (28) row (overwrite the next row)
    shots = np.flatnonzero(type_id[:-1] == 11)
    u = rng.random(len(shots))
    type_id[shots[u < 0.12] + 1] = 27
    type_id[shots[(u >= 0.12) & (u < 0.13)] + 1] = 28
    bodypart_id = rng.choice(4, size=n, p=[0.85, 0.10, 0.04, 0.01]).astype(np.int64)
    x = rng.uniform(0, FIELD_L, n)
    y = rng.uniform(0, FIELD_W, n)
    _edges(rng, x, y)
    dx = np.clip(x + rng.normal(5, 15, n), 0, FIELD_L) - x
    dy = np.clip(y + rng.normal(0, 12, n), 0, FIELD_W) - y
    z = rng.random(n)
    dx[z < 0.01] = 0.0
    dy[(z >= 0.005) & (z < 0.02)] = 0.0
    d.update(type_id=type_id, bodypart_id=bodypart_id, x=np.round(x, 4), y=np.round(y, 4),
             dx=np.round(dx, 4), dy=np.round(dy, 4))
    return d


def probabilities(n: int, seed: int = 7) -> Dict[str, np.ndarray]:
    """Classifier-like probabilities: Ps ~ Beta(0.5, 30), Pc ~ Beta(0.5, 60) (f64)."""
    rng = np.random.default_rng([seed, n])
    return dict(scores=rng.beta(0.5, 30, n), concedes=rng.beta(0.5, 60, n))


_SPADL_COLS = ['game_id', 'original_event_id', 'action_id', 'period_id', 'time_seconds',
               'team_id', 'player_id', 'start_x', 'start_y', 'end_x', 'end_y',
               'type_id', 'result_id', 'bodypart_id']
_ATOMIC_COLS = ['game_id', 'original_event_id', 'action_id', 'period_id', 'time_seconds',
                'team_id', 'player_id', 'x', 'y', 'dx', 'dy', 'type_id', 'bodypart_id']


def to_frame(d: Dict[str, np.ndarray], atomic: bool = False) -> pd.DataFrame:
    """Reference-shaped DataFrame (int64 ids, float64 coordinates, RangeIndex)."""
    n = len(d['type_id'])
    cols = {}
    for c in (_ATOMIC_COLS if atomic else _SPADL_COLS):
        if c == 'original_event_id':
            cols[c] = np.full(n, None, dtype=object)
        elif c == 'action_id':
            cols[c] = d['pos'].astype(np.int64)
        elif c == 'player_id':
            cols[c] = (d['team_id'] * 100 + d['pos'] % 11).astype(np.int64)
        else:
            cols[c] = d[c]
    return pd.DataFrame(cols)


def games_frame(d: Dict[str, np.ndarray]) -> pd.DataFrame:
    """One row per game: ``game_id``, ``home_team_id``, ``away_team_id``."""
    off = d['game_off']
    gid = d['game_id'][off[:-1]] if len(off) > 1 and off[-1] > 0 else np.zeros(0, np.int64)
    return pd.DataFrame({'game_id': gid, 'home_team_id': d['home_team_id'],
                         'away_team_id': d['home_team_id'] + 1})
