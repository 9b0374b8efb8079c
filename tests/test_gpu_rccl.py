"""The nccl (RCCL) branches of the multi-GPU xT exchange, executed for real with one rank on the
test GPU (tests/rccl_world1_check.py in its own process): every collective the N-GPU run issues,
with its real tensors and split lists, and results equal to the single-GPU fit."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_rccl_world1_xt_exchange_paths():
    env = dict(os.environ, MASTER_ADDR='127.0.0.1', MASTER_PORT='29517', RANK='0', WORLD_SIZE='1',
               LOCAL_RANK='0')
    p = subprocess.run([sys.executable, os.path.join(ROOT, 'tests', 'rccl_world1_check.py')],
                       env=env, capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-3000:]
    out = json.loads(p.stdout.strip().splitlines()[-1])
    assert out['allreduce_equal']
    assert out['bands_compact_equal'] and out['bands_rows_equal']
    assert out['rows_sharded_equal']
    assert 'all-to-all' in out['bands_compact_exchange']
