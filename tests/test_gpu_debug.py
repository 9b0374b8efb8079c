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
