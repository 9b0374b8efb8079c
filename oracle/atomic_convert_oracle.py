"""CPU oracle (numpy restatement) of the reference's SPADL -> Atomic-SPADL conversion.

TEST INFRASTRUCTURE ONLY (see ``oracle/__init__.py``): imported by ``tests/`` as the checker,
never by the product. It restates ``socceraction/atomic/spadl/base.py:15-235`` pass by pass
-- each pass computes its extra rows from (row, next row) pairs, concatenates and stable-sorts
by (game_id, period_id, action_id), then resets action_id -- exactly the reference's shape,
deliberately NOT the single-pass group expansion the HIP kernel uses, so the two are
independent. Parity pinned against golden vectors produced by running the reference itself
(``tests/golden/make_golden_convert.py``) in ``tests/test_oracle.py``.

A frame is a dict of equal-length numpy columns: game_id, original_event_id (object, None =
missing), action_id (float64 during the passes), period_id, time_seconds, team_id, player_id,
start_x, start_y, end_x, end_y, type_id, result_id, bodypart_id.
"""
from __future__ import annotations

from typing import Dict

import numpy as np

# spadl/config.py:33-57 and atomic/spadl/config.py:25-36 (ids are list positions; the atomic
# list repeats 'interception', and `list.index` returns the FIRST position, 10)
PASS_IDS = (0, 1, 2, 4, 3, 5, 6, 18, 22)        # base.py:42-53 pass-like
INTERCEPTION_IDS = (10, 9, 16, 14, 15, 17)      # base.py:55-63 interception-like
SHOT_IDS = (11, 13, 12)                          # base.py:118-119
CORNER_GOALKICK = (5, 6, 22)                     # base.py:127-133
A_RECEIVAL, A_INTERCEPTION, A_OUT, A_OFFSIDE = 23, 10, 25, 26
A_GOAL, A_OWNGOAL, A_YELLOW, A_RED, A_CORNER, A_FREEKICK = 27, 28, 29, 30, 31, 32
T_THROW_IN, T_GOALKICK, T_DRIBBLE = 2, 22, 21
R_SUCCESS, R_OFFSIDE, R_OWNGOAL, R_YELLOW, R_RED = 1, 2, 3, 4, 5

COLS = ('game_id', 'original_event_id', 'action_id', 'period_id', 'time_seconds', 'team_id',
        'player_id', 'start_x', 'start_y', 'end_x', 'end_y', 'type_id', 'result_id',
        'bodypart_id')
OUT_COLS = ('game_id', 'original_event_id', 'action_id', 'period_id', 'time_seconds',
            'team_id', 'player_id', 'x', 'y', 'dx', 'dy', 'type_id', 'bodypart_id')


def _next(f: Dict[str, np.ndarray], fill=None) -> Dict[str, np.ndarray]:
    """``actions.shift(-1)``: row i+1, the last row missing (``valid`` False) or ``fill``."""
    n = len(f['type_id'])
    out = {}
    for c, v in f.items():
        nv = np.empty_like(v)
        nv[:n - 1] = v[1:]
        if n:
            nv[n - 1] = v[n - 1] if fill is None else fill  # placeholder where invalid
        out[c] = nv
    valid = np.ones(n, bool)
    if n:
        valid[-1] = fill is not None
    return out, valid


def _merge(f: Dict[str, np.ndarray], extra: Dict[str, np.ndarray]) -> Dict[str, np.ndarray]:
    """concat + stable sort by (game_id, period_id, action_id) + action_id = range (base.py:109-111)."""
    cat = {c: np.concatenate([f[c], extra[c]]) for c in f}
    order = np.lexsort((cat['action_id'], cat['period_id'], cat['game_id']))  # stable
    out = {c: v[order] for c, v in cat.items()}
    out['action_id'] = np.arange(len(order), dtype=np.float64)
    return out


def _extra_from_passes(f):
    """base.py:38-112."""
    nx, valid = _next(f)
    same_team = valid & (f['team_id'] == nx['team_id'])
    samegame = valid & (f['game_id'] == nx['game_id'])
    sameperiod = valid & (f['period_id'] == nx['period_id'])
    idx = (np.isin(f['type_id'], PASS_IDS) & samegame & sameperiod
           & ~(valid & np.isin(nx['type_id'], INTERCEPTION_IDS)))
    p = {c: v[idx] for c, v in f.items()}
    q = {c: v[idx] for c, v in nx.items()}
    st = same_team[idx]
    e = dict(p)
    e['action_id'] = p['action_id'] + 0.1
    e['time_seconds'] = (p['time_seconds'] + q['time_seconds']) / 2
    e['start_x'], e['start_y'] = p['end_x'], p['end_y']
    e['end_x'], e['end_y'] = p['end_x'], p['end_y']
    e['bodypart_id'] = np.zeros_like(p['bodypart_id'])
    e['result_id'] = np.full_like(p['result_id'], -1)
    offside = p['result_id'] == R_OFFSIDE
    out = ((q['type_id'] == T_GOALKICK) & ~st) | (q['type_id'] == T_THROW_IN)
    t = np.where(st, A_RECEIVAL, A_INTERCEPTION)
    t = np.where(out, A_OUT, t)
    t = np.where(offside, A_OFFSIDE, t)
    e['type_id'] = t.astype(p['type_id'].dtype)
    e['team_id'] = np.where(t == A_INTERCEPTION, q['team_id'], p['team_id'])
    e['player_id'] = np.where(out | offside, p['player_id'], q['player_id'])
    return _merge(f, e)


def _add_dribbles(f):
    """spadl/base.py:54-93 (``shift(-1, fill_value=0)``: the last row's next is all zeros)."""
    nx, _ = _next(f, fill=0)
    same_team = f['team_id'] == nx['team_id']
    dx = f['end_x'] - nx['start_x']
    dy = f['end_y'] - nx['start_y']
    d2 = dx ** 2 + dy ** 2
    far = d2 >= 3.0 ** 2
    near = d2 <= 60.0 ** 2
    dt = nx['time_seconds'] - f['time_seconds']
    idx = same_team & far & near & (dt < 10.0) & (f['period_id'] == nx['period_id'])
    p = {c: v[idx] for c, v in f.items()}
    q = {c: v[idx] for c, v in nx.items()}
    d = {}
    d['game_id'] = q['game_id']
    d['original_event_id'] = np.full(len(d['game_id']), None, dtype=object)  # not set: NaN
    d['period_id'] = q['period_id']
    d['action_id'] = p['action_id'] + 0.1
    d['time_seconds'] = (p['time_seconds'] + q['time_seconds']) / 2
    d['team_id'] = q['team_id']
    d['player_id'] = q['player_id']
    d['start_x'], d['start_y'] = p['end_x'], p['end_y']
    d['end_x'], d['end_y'] = q['start_x'], q['start_y']
    d['bodypart_id'] = np.zeros_like(p['bodypart_id'])
    d['type_id'] = np.full_like(p['type_id'], T_DRIBBLE)
    d['result_id'] = np.full_like(p['result_id'], R_SUCCESS)
    return _merge(f, d)


def _extra_from_shots(f):
    """base.py:115-165."""
    nx, valid = _next(f)
    samegame = valid & (f['game_id'] == nx['game_id'])
    sameperiod = valid & (f['period_id'] == nx['period_id'])
    shot = np.isin(f['type_id'], SHOT_IDS)
    goal = shot & (f['result_id'] == R_SUCCESS)
    owngoal = f['result_id'] == R_OWNGOAL
    nxt = valid & np.isin(nx['type_id'], CORNER_GOALKICK)
    out = shot & nxt & samegame & sameperiod
    idx = goal | owngoal | out
    p = {c: v[idx] for c, v in f.items()}
    e = dict(p)
    e['action_id'] = p['action_id'] + 0.1
    e['start_x'], e['start_y'] = p['end_x'], p['end_y']
    e['result_id'] = np.full_like(p['result_id'], -1)
    t = np.full(len(p['type_id']), -1)
    t = np.where(out[idx], A_OUT, t)
    t = np.where(goal[idx], A_GOAL, t)
    t = np.where(owngoal[idx], A_OWNGOAL, t)
    e['type_id'] = t.astype(p['type_id'].dtype)
    return _merge(f, e)


def _extra_from_fouls(f):
    """base.py:168-196."""
    yellow = f['result_id'] == R_YELLOW
    red = f['result_id'] == R_RED
    idx = yellow | red
    p = {c: v[idx] for c, v in f.items()}
    e = dict(p)
    e['action_id'] = p['action_id'] + 0.1
    e['start_x'], e['start_y'] = p['end_x'], p['end_y']
    e['result_id'] = np.full_like(p['result_id'], -1)
    t = np.where(red[idx], A_RED, np.where(yellow[idx], A_YELLOW, -1))
    e['type_id'] = t.astype(p['type_id'].dtype)
    return _merge(f, e)


def add_dribbles(cols: Dict[str, np.ndarray]) -> Dict[str, np.ndarray]:
    """spadl/base.py:54-93 on its own (the SPADL converters' last step): the SPADL columns of
    COLS in, the same columns out with action_id reset to int64 positions."""
    f = {c: np.asarray(cols[c]) for c in COLS}
    f['action_id'] = f['action_id'].astype(np.float64)
    f['original_event_id'] = f['original_event_id'].astype(object)
    if len(f['type_id']) == 0:
        return {c: (v.astype(np.int64) if c == 'action_id' else v) for c, v in f.items()}
    f = _add_dribbles(f)
    f['action_id'] = f['action_id'].astype(np.int64)
    return f


def convert_to_atomic(cols: Dict[str, np.ndarray]) -> Dict[str, np.ndarray]:
    """base.py:15-35: the four passes, _convert_columns (:199-220) and _simplify (:223-235)."""
    f = {c: np.asarray(cols[c]) for c in COLS}
    f['action_id'] = f['action_id'].astype(np.float64)
    f['original_event_id'] = f['original_event_id'].astype(object)
    for step in (_extra_from_passes, _add_dribbles, _extra_from_shots, _extra_from_fouls):
        f = step(f)
    out = {c: f[c] for c in ('game_id', 'original_event_id', 'period_id', 'time_seconds',
                             'team_id', 'player_id', 'bodypart_id')}
    out['action_id'] = f['action_id'].astype(np.int64)
    out['x'], out['y'] = f['start_x'], f['start_y']
    out['dx'] = f['end_x'] - f['start_x']
    out['dy'] = f['end_y'] - f['start_y']
    t = f['type_id'].copy()
    t[np.isin(t, (5, 6))] = A_CORNER      # corner_crossed, corner_short
    t[np.isin(t, (3, 4, 13))] = A_FREEKICK  # freekick_crossed, freekick_short, shot_freekick
    out['type_id'] = t
    return {c: out[c] for c in OUT_COLS}
