"""The debug build (-DSA_DEBUG=1, libsocceraction_amd_debug.so: device bounds checks in every
kernel) on the GPU: the golden parity tests pass through it with every call
followed by sa_debug_check(), and a corrupt segment table is reported instead of read past.

Each case runs in a child process, because the library is chosen when socceraction_amd loads
(SOCCERACTION_AMD_DEBUG=1)."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CORRUPT = r'''
import numpy as np, torch
from socceraction_amd import _native, batch as B, ops, synthetic
assert _native.lib().sa_debug_enabled() == 1
d = synthetic.spadl_games(3, seed=5)
ab = B.ActionBatch.from_columns(d)
ops.labels(ab)  # clean run: no report
# the segment table claims fewer rows than the batch holds: rows past the last offset would
# make the segment cursors walk past seg_off (the default build trusts the table)
ab.cols['seg_off'][-1] = ab.n - 7
try:
    ops.labels(ab)
except ValueError as e:
    assert 'device bounds check failed' in str(e), e
    print('caught:', e)
else:
    raise SystemExit('corrupt segment table not reported')
ab.cols['seg_off'][-1] = ab.n
ops.labels(ab)  # the record was cleared by the failing check
print('ok')
'''


def _run(args, timeout=600):
    # prepend: whatever PYTHONPATH the harness set (e.g. its library-mapping hook) stays
    path = [ROOT, os.path.join(ROOT, 'tests')] + [p for p in os.environ.get('PYTHONPATH', '').split(os.pathsep) if p]
    env = dict(os.environ, SOCCERACTION_AMD_DEBUG='1', PYTHONPATH=os.pathsep.join(path))
    p = subprocess.run([sys.executable] + args, cwd=ROOT, env=env, capture_output=True, text=True,
                       timeout=timeout)
    assert p.returncode == 0, (p.stdout[-3000:], p.stderr[-3000:])
    return p.stdout


def test_goldens_through_the_debug_build():
    out = _run(['-m', 'pytest', '-x', '-q', '-p', 'no:cacheprovider', 'tests/test_gpu_parity.py',
                '-k', 'goldens or small_segments or xt_rate_codes'])
    assert 'passed' in out


def test_debug_build_reports_a_corrupt_segment_table():
    out = _run(['-c', CORRUPT], timeout=300)
    assert out.strip().endswith('ok')


ABORT = r"""
import warnings
import numpy as np, torch
from socceraction_amd import _native, ops
assert _native.lib().sa_debug_enabled() == 1
rng = np.random.default_rng(11)
C = 1500
cnt = np.zeros((C, C), np.int32)
nz = rng.random((C, C)) < 0.2
cnt[nz] = rng.geometric(0.3, nz.sum())
move = cnt.sum(axis=1, dtype=np.int64) + rng.integers(1, 50, C)
gs, pm = rng.random(C) * 0.05, rng.random(C) * 0.95
dev = torch.device('cuda')
rows = torch.from_numpy(cnt).to(dev)
lib = _native.lib()
ell = torch.empty(int(lib.sa_xt_compact_bytes(C, C)) // 4, dtype=torch.int32, device=dev)
slen = torch.empty(C, dtype=torch.int32, device=dev)
from socceraction_amd.batch import stream_handle
_native.check(lib.sa_xt_compact_rows(rows.data_ptr(), C, C, ell.data_ptr(), slen.data_ptr(), stream_handle()))
t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
args = (ell, slen, rows, t(move), t(gs), t(pm), C, 1e-5, 1000)
he, ne, pe = ops.xt_solve_compact(*args, exact_order=True)
hr, nr, pr = ops.xt_solve_compact(*args)
assert pe == 'sequential' and pr == 'reordered' and nr == ne > 3, (pe, pr, nr, ne)
for k in (0, 3):  # the first barrier (50 ms bound) and a later one (1 s bound)
    _native.check(lib.sa_debug_xt_solve_abort(k))
    with warnings.catch_warnings(record=True) as wl:
        warnings.simplefilter('always')
        h, n, p = ops.xt_solve_compact(*args)
    assert p == 'timeout', p
    assert any('timed out' in str(w.message) for w in wl), [str(w.message) for w in wl]
    # the fallback redoes the solve in the reference's order: the same count, the same bits
    assert n == ne and torch.equal(h[:n + 1], he[:ne + 1]), (k, n, ne)
    print('abort at', k, 'ok')
_native.check(lib.sa_debug_xt_solve_abort(-1))
h, n, p = ops.xt_solve_compact(*args)
assert p == 'reordered' and n == nr and torch.equal(h[:n + 1], hr[:nr + 1])
print('ok')
"""


def test_reordered_solve_barrier_timeout_exit():
    """The persistent reordered solve's barrier-timeout exit, forced deterministically
    (sa_debug_xt_solve_abort: the last workgroup leaves at iteration k without arriving): at the
    first barrier and at a later one, the solve reports path 'timeout', ops warns, and the
    reference-order fallback gives the sequential solve's iteration count and heatmaps bit for
    bit; switched off, the reordered path runs again with its own bits."""
    out = _run(['-c', ABORT], timeout=300)
    assert out.strip().endswith('ok')


ABORT_FUSED = r"""
import warnings
import torch
from socceraction_amd import _native, ops, synthetic, batch as B
lib = _native.lib()
assert lib.sa_debug_enabled() == 1
ab = B.ActionBatch.from_columns(synthetic.spadl_games(60, game_id0=5))
ic = [ops.xt_interp_codes_buffer(ab.n, ab.device)]
acc = ops.xt_count_many([ab], 105, 68, interp_codes=ic, dense=False)
sol = ops.xt_solve(acc, transition=False, exact_order=True)
ref, _ = ops.xt_rate_interp_codes_many(ic, [ab.n], sol.mats[3].reshape(68, 105), 105, 68)
_native.check(lib.sa_debug_xt_solve_abort(2))
with warnings.catch_warnings(record=True) as wl:
    warnings.simplefilter('always')
    sol2, got, _ = ops.xt_fit_rate_interp_codes(acc, ic, [ab.n])
_native.check(lib.sa_debug_xt_solve_abort(-1))
assert sol2.path == 'timeout', sol2.path
assert any('timed out' in str(w.message) for w in wl)
assert sol2.n_iter == sol.n_iter > 3 and torch.equal(sol2.heatmaps, sol.heatmaps)
assert torch.equal(got[0].view(torch.int64), ref[0].view(torch.int64))
print('ok')
"""


def test_fused_fit_rate_after_a_barrier_timeout():
    """sa_xt_fit_rate_interp_codes when the reordered solve aborts (forced at iteration 2): the
    rate queued behind it ran over a half-written surface, the solve is redone in the
    reference's order and the rate again -- rates and heatmaps equal the exact-order solve's."""
    out = _run(['-c', ABORT_FUSED], timeout=300)
    assert out.strip().endswith('ok')
