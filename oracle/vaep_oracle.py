"""CPU oracle (numpy restatement) of the reference's VAEP / Atomic-VAEP hot path.

TEST INFRASTRUCTURE ONLY. Imported solely by ``tests/``, ``__graft_entry__.smoke()``
and ``bench.py``'s ``cpu_baseline`` leg, always as the *checker* — never as the thing
measured or shipped. The product path (``socceraction_amd``) never imports it.

Parity pinned: every function below is checked against golden vectors produced by
running the reference itself (``tests/golden/make_golden.py`` imports
``/root/reference`` in the build container) in ``tests/test_oracle.py``.

Inputs are flat numpy columns (ids as integers, coordinates/times float64, raw team
ids) plus segment offsets; a segment is one game (batched API) or one whole frame
(the reference's module-level functions). Citations are file:line in the reference.
"""
from __future__ import annotations

from typing import Dict, List, Sequence, Tuple

import numpy as np

FIELD_L, FIELD_W = 105.0, 68.0  # spadl/config.py:21-22
SPADL_TYPES = ['pass', 'cross', 'throw_in', 'freekick_crossed', 'freekick_short',
               'corner_crossed', 'corner_short', 'take_on', 'foul', 'tackle', 'interception',
               'shot', 'shot_penalty', 'shot_freekick', 'keeper_save', 'keeper_claim',
               'keeper_punch', 'keeper_pick_up', 'clearance', 'bad_touch', 'non_action',
               'dribble', 'goalkick']  # spadl/config.py:33-57
RESULTS = ['fail', 'success', 'offside', 'owngoal', 'yellow_card', 'red_card']  # :25-32
BODYPARTS = ['foot', 'head', 'other', 'head/other']  # :24
ATOMIC_TYPES = SPADL_TYPES + ['receival', 'interception', 'out', 'offside', 'goal', 'owngoal',
                              'yellow_card', 'red_card', 'corner', 'freekick']  # atomic/spadl/config.py:25-36

SPADL_DEFAULT = ['actiontype_onehot', 'result_onehot', 'actiontype_result_onehot',
                 'bodypart_onehot', 'time', 'startlocation', 'endlocation', 'startpolar',
                 'endpolar', 'movement', 'team', 'time_delta', 'space_delta', 'goalscore']  # vaep/base.py:37-52
ATOMIC_DEFAULT = ['actiontype', 'actiontype_onehot', 'bodypart', 'bodypart_onehot', 'time',
                  'team', 'time_delta', 'location', 'polar', 'movement_polar', 'direction',
                  'goalscore']  # atomic/vaep/base.py:23-36


def segments_of(n: int, seg_off=None) -> np.ndarray:
    return np.array([0, n], dtype=np.int64) if seg_off is None else np.asarray(seg_off, np.int64)


def _seg_start_end(n: int, seg_off: np.ndarray) -> Tuple[np.ndarray, np.ndarray]:
    """Per-row segment start and (exclusive) end."""
    sizes = np.diff(seg_off)
    start = np.repeat(seg_off[:-1], sizes)
    end = np.repeat(seg_off[1:], sizes)
    return start, end


def window_rows(n: int, seg_off: np.ndarray, i: int) -> np.ndarray:
    """Row of game-state window i: max(j - i, segment start) (vaep/features.py:83-88)."""
    start, _ = _seg_start_end(n, seg_off)
    return np.maximum(np.arange(n) - i, start)


def _away(team: np.ndarray, seg_off: np.ndarray, home: Sequence) -> np.ndarray:
    """away(j) = team[j] != home of j's segment (vaep/features.py:109-110)."""
    sizes = np.diff(seg_off)
    h = np.repeat(np.asarray(home, dtype=object), sizes)
    return np.array([t != hh for t, hh in zip(team.tolist(), h.tolist())], dtype=bool)


def _polar(x, y):
    """startpolar/endpolar/polar (vaep/features.py:371-377)."""
    dx = np.abs(FIELD_L - x)
    dy = np.abs(FIELD_W / 2 - y)
    dist = np.sqrt(dx ** 2 + dy ** 2)
    with np.errstate(divide='ignore', invalid='ignore'):
        ang = np.nan_to_num(np.arctan(dy / dx))
    return dist, ang


def _goal_flags(cols: Dict[str, np.ndarray], atomic: bool):
    t = cols['type_id']
    if atomic:  # atomic/vaep/features.py:246-247, atomic/vaep/labels.py:27-28
        return t == 27, t == 28
    shot = (t == 11) | (t == 12) | (t == 13)  # str.contains('shot') (vaep/features.py:522)
    r = cols['result_id']
    return shot & (r == 1), shot & (r == 3)


def features(cols: Dict[str, np.ndarray], k: int, xfns: Sequence[str], atomic: bool = False,
             seg_off=None, home=None) -> List[Tuple[str, str, np.ndarray]]:
    """Feature columns ``(name, kind, values)`` in reference order (vaep/base.py:113-116).

    ``home`` = per-segment home team id (None: no flip). Windows and the flip follow
    vaep/features.py:62-116 / atomic/vaep/features.py:86-111.
    """
    n = len(cols['type_id'])
    so = segments_of(n, seg_off)
    rows = [window_rows(n, so, i) for i in range(k)]
    away = _away(cols['team_id'], so, home) if home is not None else np.zeros(n, bool)
    W = []
    for i in range(k):
        r = rows[i]
        w = {c: cols[c][r] for c in cols}
        if atomic:
            w['x'] = np.where(away, FIELD_L - w['x'], w['x'])
            w['y'] = np.where(away, FIELD_W - w['y'], w['y'])
            w['dx'] = np.where(away, -w['dx'], w['dx'])
            w['dy'] = np.where(away, -w['dy'], w['dy'])
        else:
            for c, ext in (('start_x', FIELD_L), ('end_x', FIELD_L), ('start_y', FIELD_W),
                           ('end_y', FIELD_W)):
                w[c] = np.where(away, ext - w[c], w[c])
        W.append(w)
    out: List[Tuple[str, str, np.ndarray]] = []
    types = ATOMIC_TYPES if atomic else SPADL_TYPES
    for x in xfns:
        for i in range(k):  # @simple transformers: a0 columns, then a1, ... (features.py:135-143)
            a = W[i]
            if x == 'actiontype':
                out.append((f'type_id_a{i}', 'i', a['type_id'].astype(np.int64)))
            elif x == 'actiontype_onehot':
                names = a['type_id']
                seen = {}
                for tid, tname in enumerate(types):  # duplicate name: later assignment wins
                    mask = np.isin(names, [q for q, nm in enumerate(types) if nm == tname])
                    seen[f'type_{tname}'] = mask
                for nm, v in seen.items():
                    out.append((f'{nm}_a{i}', 'b', v))
            elif x == 'result':
                out.append((f'result_id_a{i}', 'i', a['result_id'].astype(np.int64)))
            elif x == 'result_onehot':
                for rid, rn in enumerate(RESULTS):
                    out.append((f'result_{rn}_a{i}', 'b', a['result_id'] == rid))
            elif x == 'actiontype_result_onehot':
                for tid, tn in enumerate(SPADL_TYPES):
                    for rid, rn in enumerate(RESULTS):
                        out.append((f'type_{tn}_result_{rn}_a{i}', 'b',
                                    (a['type_id'] == tid) & (a['result_id'] == rid)))
            elif x == 'bodypart':
                out.append((f'bodypart_id_a{i}', 'i', a['bodypart_id'].astype(np.int64)))
            elif x == 'bodypart_onehot':
                for bid, bn in enumerate(BODYPARTS):
                    out.append((f'bodypart_{bn}_a{i}', 'b', a['bodypart_id'] == bid))
            elif x == 'time':  # features.py:312-314
                p = a['period_id'].astype(np.int64)
                out.append((f'period_id_a{i}', 'i', p))
                out.append((f'time_seconds_a{i}', 'f', a['time_seconds'].astype(np.float64)))
                out.append((f'time_seconds_overall_a{i}', 'f',
                            ((p - 1) * 45 * 60) + a['time_seconds']))
            elif x == 'startlocation':
                out += [(f'start_x_a{i}', 'f', a['start_x']), (f'start_y_a{i}', 'f', a['start_y'])]
            elif x == 'endlocation':
                out += [(f'end_x_a{i}', 'f', a['end_x']), (f'end_y_a{i}', 'f', a['end_y'])]
            elif x == 'startpolar':
                d, g = _polar(a['start_x'], a['start_y'])
                out += [(f'start_dist_to_goal_a{i}', 'f', d), (f'start_angle_to_goal_a{i}', 'f', g)]
            elif x == 'endpolar':
                d, g = _polar(a['end_x'], a['end_y'])
                out += [(f'end_dist_to_goal_a{i}', 'f', d), (f'end_angle_to_goal_a{i}', 'f', g)]
            elif x == 'movement':  # features.py:420-424
                dx = a['end_x'] - a['start_x']
                dy = a['end_y'] - a['start_y']
                out += [(f'dx_a{i}', 'f', dx), (f'dy_a{i}', 'f', dy),
                        (f'movement_a{i}', 'f', np.sqrt(dx ** 2 + dy ** 2))]
            elif x == 'location':
                out += [(f'x_a{i}', 'f', a['x']), (f'y_a{i}', 'f', a['y'])]
            elif x == 'polar':
                d, g = _polar(a['x'], a['y'])
                out += [(f'dist_to_goal_a{i}', 'f', d), (f'angle_to_goal_a{i}', 'f', g)]
            elif x == 'movement_polar':  # atomic/vaep/features.py:196-199
                md = np.sqrt(a['dx'] ** 2 + a['dy'] ** 2)
                with np.errstate(divide='ignore', invalid='ignore'):
                    ma = np.arctan2(a['dy'], a['dx'])
                ma = np.where(a['dy'] == 0, 0.0, ma)
                out += [(f'mov_d_a{i}', 'f', md), (f'mov_angle_a{i}', 'f', ma)]
            elif x == 'direction':  # atomic/vaep/features.py:219-224
                td = np.sqrt(a['dx'] ** 2 + a['dy'] ** 2)
                with np.errstate(divide='ignore', invalid='ignore'):
                    ox = np.where(td > 0, a['dx'] / td, a['dx'])
                    oy = np.where(td > 0, a['dy'] / td, a['dy'])
                out += [(f'dx_a{i}', 'f', ox), (f'dy_a{i}', 'f', oy)]
            else:
                break  # state / context features below
        a0 = W[0]
        if x == 'team':  # features.py:448-452
            for i in range(1, k):
                out.append((f'team_{i}', 'b', W[i]['team_id'] == a0['team_id']))
        elif x == 'time_delta':  # features.py:469-473
            for i in range(1, k):
                out.append((f'time_delta_{i}', 'f', a0['time_seconds'] - W[i]['time_seconds']))
        elif x == 'space_delta':  # features.py:491-499
            for i in range(1, k):
                dx = W[i]['end_x'] - a0['start_x']
                dy = W[i]['end_y'] - a0['start_y']
                out += [(f'dx_a0{i}', 'f', dx), (f'dy_a0{i}', 'f', dy),
                        (f'mov_a0{i}', 'f', np.sqrt(dx ** 2 + dy ** 2))]
        elif x == 'goalscore':
            out += goalscore(cols, atomic, so)
    return out


def goalscore(cols: Dict[str, np.ndarray], atomic: bool, seg_off: np.ndarray):
    """Segmented exclusive goal counts (vaep/features.py:520-539)."""
    n = len(cols['type_id'])
    goals, owngoals = _goal_flags(cols, atomic)
    team = cols['team_id']
    gt = np.zeros(n, np.int64)
    go = np.zeros(n, np.int64)
    for s, e in zip(seg_off[:-1], seg_off[1:]):
        if e <= s:
            continue
        sl = slice(s, e)
        isA = team[sl] == team[s]
        gA = ((goals[sl] & isA) | (owngoals[sl] & ~isA)).astype(np.int64)
        gB = ((goals[sl] & ~isA) | (owngoals[sl] & isA)).astype(np.int64)
        cA = np.cumsum(gA) - gA
        cB = np.cumsum(gB) - gB
        gt[sl] = cA * isA + cB * ~isA
        go[sl] = cB * isA + cA * ~isA
    return [('goalscore_team', 'i', gt), ('goalscore_opponent', 'i', go),
            ('goalscore_diff', 'i', gt - go)]


def labels(cols: Dict[str, np.ndarray], atomic: bool = False, nr_actions: int = 10,
           seg_off=None) -> Dict[str, np.ndarray]:
    """scores / concedes / goal_from_shot (vaep/labels.py:9-116, atomic/vaep/labels.py)."""
    n = len(cols['type_id'])
    so = segments_of(n, seg_off)
    goals, owngoals = _goal_flags(cols, atomic)
    team = cols['team_id']
    _, end = _seg_start_end(n, so)
    last = end - 1
    idx = np.arange(n)
    sc = goals.copy()
    co = owngoals.copy()
    for i in range(1, nr_actions):  # shift(-i), tail = last row (labels.py:38-48)
        c = np.minimum(idx + i, last)
        same = team[c] == team
        sc |= (goals[c] & same) | (owngoals[c] & ~same)
        co |= (goals[c] & ~same) | (owngoals[c] & same)
    if atomic:  # shot followed by goal; last row compares NaN -> False (labels.py:102-105)
        t = cols['type_id']
        nxt = np.minimum(idx + 1, last)
        gfs = (t == 11) & (t[nxt] == 27) & (idx < last)
    else:
        gfs = goals
    return {'scores': sc, 'concedes': co, 'goal_from_shot': gfs}


def formula(cols: Dict[str, np.ndarray], p_scores: np.ndarray, p_concedes: np.ndarray,
            atomic: bool = False, seg_off=None) -> Dict[str, np.ndarray]:
    """offensive / defensive / vaep value (vaep/formula.py:17-151; atomic formula.py).

    Arithmetic stays in the probability dtype, as in pandas.
    """
    n = len(cols['type_id'])
    so = segments_of(n, seg_off)
    start, _ = _seg_start_end(n, so)
    idx = np.arange(n)
    p = np.maximum(idx - 1, start)  # _prev (formula.py:8-11)
    ps, pc = np.asarray(p_scores), np.asarray(p_concedes)
    dt = ps.dtype
    team, t = cols['team_id'], cols['type_id']
    same = team[p] == team
    prev_s = ps[p] * same + pc[p] * (~same)
    prev_c = pc[p] * same + ps[p] * (~same)
    prev_s = prev_s.astype(dt)
    prev_c = prev_c.astype(dt)
    if atomic:
        prevgoal = np.isin(t[p], [27, 28])
    else:
        toolong = np.abs(cols['time_seconds'] - cols['time_seconds'][p]) > 10
        prev_s[toolong] = 0
        prev_c[toolong] = 0
        prevgoal = np.isin(t[p], [11, 12, 13]) & (cols['result_id'][p] == 1)
    prev_s[prevgoal] = 0
    prev_c[prevgoal] = 0
    if not atomic:
        prev_s[t == 12] = 0.792453
        prev_s[np.isin(t, [5, 6])] = 0.046500
    off = ps - prev_s
    de = -(pc - prev_c)
    return {'offensive_value': off, 'defensive_value': de, 'vaep_value': off + de}
