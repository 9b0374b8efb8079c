"""bench.py's parity check of the timed buffers (CPU): fed the oracle's own outputs laid out as
the device blocks it passes, and a single changed bool / int / float / count / surface value
makes it fail. The GPU side of the same check runs inside every bench.py line."""
import os
import sys
from types import SimpleNamespace

import numpy as np
import pytest

torch = pytest.importorskip('torch')

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from oracle import vaep_oracle as vo  # noqa: E402
from oracle import xt_oracle as xo  # noqa: E402
from socceraction_amd import catalog, ops, synthetic  # noqa: E402


def _blocks(d, atomic=False, Rb=1024, Rn=128):
    """The oracle's per-game features in the tiled device layout (CPU tensors)."""
    xfns = vo.ATOMIC_DEFAULT if atomic else vo.SPADL_DEFAULT
    plan = catalog.build_plan(xfns, 3, atomic)
    off = d['game_off']
    n = int(off[-1])
    full = {'b': np.zeros((plan.n_bool, n), np.uint8), 'f': np.zeros((plan.n_f64, n)),
            'i': np.zeros((plan.n_i64, n), np.int64)}
    names = bench.ATOMIC_COLS if atomic else bench.SPADL_COLS
    for g in range(len(off) - 1):
        s, e = int(off[g]), int(off[g + 1])
        ref = vo.features({c: d[c][s:e] for c in names}, 3, xfns, atomic=atomic,
                          home=[d['home_team_id'][g]])
        for (_, kind, col), (_, _, v) in zip(plan.order, ref):
            full[kind][col, s:e] = v

    def tile(a, R, dt):
        T = -(-n // R)
        pad = np.zeros((a.shape[0], T * R), a.dtype)
        pad[:, :n] = a
        return torch.from_numpy(pad.reshape(a.shape[0], T, R).transpose(1, 0, 2).copy()).to(dt)
    return ops.FeatureBlocks(plan, n, Rb, Rn, tile(full['b'], Rb, torch.uint8),
                             tile(full['f'], Rn, torch.float64), tile(full['i'], Rn, torch.int64))


def _labels_formula(d, p, atomic=False):
    off = d['game_off']
    n = int(off[-1])
    sc, co, val = np.zeros(n, np.uint8), np.zeros(n, np.uint8), np.zeros((3, n))
    names = bench.ATOMIC_COLS if atomic else bench.SPADL_COLS
    for g in range(len(off) - 1):
        s, e = int(off[g]), int(off[g + 1])
        cols = {c: d[c][s:e] for c in names}
        lab = vo.labels(cols, atomic=atomic)
        sc[s:e], co[s:e] = lab['scores'], lab['concedes']
        if p is not None:
            fo = vo.formula(cols, p['scores'][s:e], p['concedes'][s:e], atomic=atomic)
            val[:, s:e] = [fo[c] for c in ('offensive_value', 'defensive_value', 'vaep_value')]
    return torch.from_numpy(sc), torch.from_numpy(co), torch.from_numpy(val)


@pytest.mark.parametrize('atomic', [False, True])
def test_vaep_check_passes_and_catches_one_value(atomic):
    d = synthetic.atomic_games(3, mean_actions=300) if atomic else synthetic.spadl_games(3, mean_actions=700)
    p = None if atomic else synthetic.probabilities(int(d['game_off'][-1]))
    out = _blocks(d, atomic)
    sc, co, val = _labels_formula(d, p, atomic)
    par = bench.Parity()
    bench.check_vaep(par, d, out, sc, co, None if atomic else val, p, atomic=atomic)
    assert par.ok and par.games == 3 and par.values > 0, par.failures
    # one flipped bool in the last game, one changed goalscore, one float off by 1e-5 relative
    s = int(d['game_off'][2])
    out.bool_block.view(-1)[out.bool_block.numel() // 2] ^= 1
    par = bench.Parity()
    bench.check_vaep(par, d, out, sc, co, None, None, atomic=atomic)
    assert not par.ok
    out = _blocks(d, atomic)
    fcol = out.plan.order[[k for _, k, _ in out.plan.order].index('f')][2]
    R = out.Rn
    out.f64_block[(s + 5) // R, fcol, (s + 5) % R] *= 1 + 1e-5  # a non-zero time_seconds
    par = bench.Parity()
    bench.check_vaep(par, d, out, sc, co, None, None, atomic=atomic)
    assert not par.ok and any('game 2' in f for f in par.failures)
    out = _blocks(d, atomic)
    sc[s] ^= 1
    par = bench.Parity()
    bench.check_vaep(par, d, out, sc, co, None, None, atomic=atomic)
    assert not par.ok


def test_xt_check_passes_and_catches_one_count():
    d = synthetic.spadl_games(4, mean_actions=800)
    l, w = 16, 12
    cnt = bench.oracle_counts(d, l, w)
    fit = xo.solve(cnt, l, w)
    acc = SimpleNamespace(shot=torch.from_numpy(cnt['shot'].reshape(-1)),
                          goal=torch.from_numpy(cnt['goal'].reshape(-1)),
                          move=torch.from_numpy(cnt['move'].reshape(-1)),
                          trans=torch.from_numpy(cnt['trans'].reshape(-1).astype(np.int32)))
    xT = torch.from_numpy(fit['xT'].reshape(-1).copy())
    n_iter = len(fit['heatmaps']) - 1
    rate = torch.from_numpy(xo.rate({c: d[c] for c in ('start_x', 'start_y', 'end_x', 'end_y',
                                                         'type_id', 'result_id')}, fit['xT']))
    par = bench.Parity()
    ref = bench.check_xt(par, cnt, acc, xT, n_iter, l, w)
    bench.check_xt_rate(par, d, rate, ref)
    assert par.ok, par.failures
    par = bench.Parity()
    bench.check_xt(par, cnt, acc, xT, n_iter + 1, l, w)
    assert not par.ok
    xT2 = xT.clone()
    xT2[5] = np.nextafter(xT2[5].item(), 1.0)
    par = bench.Parity()
    bench.check_xt(par, cnt, acc, xT2, n_iter, l, w)
    assert par.failures == ['xT 16x12 surface']
    acc.trans[int(np.flatnonzero(cnt['trans'].reshape(-1))[0])] += 1
    par = bench.Parity()
    bench.check_xt(par, cnt, acc, xT, n_iter, l, w)
    assert 'xT 16x12 transition counts' in par.failures
    r2 = rate.clone()
    k = int(np.flatnonzero(~np.isnan(rate.numpy()))[0])
    r2[k] = float('nan')
    par = bench.Parity()
    bench.check_xt_rate(par, d, r2, ref)
    assert not par.ok


def test_sample_games_covers_first_and_last():
    g = bench.sample_games(10000)
    assert len(g) == 12 and g[0] == 0 and g[1] == 9999 and len(set(g)) == 12
    assert bench.sample_games(5) == [0, 1, 2, 3, 4]
