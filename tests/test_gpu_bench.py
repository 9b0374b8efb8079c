"""bench.py's multi-rank entry on the GPU box: ``bench.py --gpus 2`` (no torchrun around it)
launches two ranks itself and prints ONE line with n_gpus == 2.  The rehearsal shares the test
GPU between the ranks over gloo (SA_DIST_BACKEND=gloo); the driver's N = 1..8 runs use RCCL
with one rank per GPU."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_gpus_2_launches_two_ranks():
    env = dict(os.environ, SA_DIST_BACKEND='gloo')
    env.pop('WORLD_SIZE', None)
    p = subprocess.run([sys.executable, 'bench.py', '--gpus', '2', '--games', '20', '--steps', '2',
                        '--warmup', '1', '--no-side', '--no-cpu'], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=240)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith('{')]
    assert p.returncode == 0 and len(lines) == 1, p.stdout[-2000:] + p.stderr[-3000:]
    out = json.loads(lines[0])
    assert out['n_gpus'] == 2 and out['value'] > 0
    assert out['config']['actions_per_gpu'] > 0
    assert 0 < out['roofline']['step_frac'] < 1


@pytest.mark.parametrize('solve', ['sharded', 'sharded-rows', 'replicated'])
def test_bench_gpus_2_side_entries(solve):
    """The side entries under two ranks: cfg5's and cfg3's games split over the ranks; cfg5's
    fit band-sharded (the default for N > 1: all-to-all of the counted actions, each rank counting
    its own bands, then the compact rows all-gathered once, or each rank iterating its own rows)
    or replicated (all-reduce of the count table), its parity block
    (counts or surface, iterations, rates vs the oracle) ok either way."""
    env = dict(os.environ, SA_DIST_BACKEND='gloo')
    env.pop('WORLD_SIZE', None)
    p = subprocess.run([sys.executable, 'bench.py', '--gpus', '2', '--games', '20', '--steps', '2',
                        '--warmup', '1', '--no-cpu', '--cfg5-games', '45', '--atomic-games', '30',
                        '--e2e-games', '5', '--cfg5-solve', solve], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=240)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith('{')]
    assert p.returncode == 0 and len(lines) == 1, p.stdout[-2000:] + p.stderr[-3000:]
    out = json.loads(lines[0])
    assert out['n_gpus'] == 2
    x = out['xt105_cfg5']
    assert x['actions_total'] > x['actions_per_gpu'] > 0 and x['iterations'] > 0
    assert x['solve'].startswith('replicated' if solve == 'replicated' else 'band-sharded')
    if solve != 'replicated':
        assert ('row-sharded' in x['solve']) == (solve == 'sharded-rows')
    assert x['parity']['ok'] and x['parity']['values_checked'] > 0
    # per-phase HIP-event times of the exchange (DESIGN §6's projection is checked against them)
    ev = x['phase_events_ms']
    if solve == 'replicated':
        assert ev['count_all_reduce'] > 0 and ev['solve'] > 0 and 'compare_replicated' not in x
    else:
        want = ('bucket', 'key_all_to_all', 'band_count', 'vector_all_gather') + (
            ('compact_build', 'row_length_all_gather', 'compact_all_gather', 'solve')
            if solve == 'sharded' else ('row_sharded_solve',))
        assert all(ev[k] > 0 for k in want), ev
        # north_star's all-reduce-only scheme measured beside the band-sharded default
        rep = x['compare_replicated']
        assert rep['solve'].startswith('replicated') and rep['parity']['ok']
        assert rep['phase_events_ms']['count_all_reduce'] > 0 and rep['ms_fit_and_rate'] > 0
    a = out['atomic_cfg3']
    assert a['atomic_actions_total'] > a['atomic_actions_per_gpu'] > 0
    assert a['parity']['ok']


def test_bench_rccl_one_rank_every_entry():
    """bench.py's process-group path through REAL RCCL (backend nccl) with one rank on the test
    GPU (SA_BENCH_DIST=1 under torch.distributed.run): the step's all-reduce of the xT counts,
    the timing barriers and max-reductions, cfg5's sharded exchange and cfg3's split -- the code
    the driver's N-GPU runs execute -- end to end, every parity block ok, no side-entry error."""
    env = dict(os.environ, SA_BENCH_DIST='1')
    for k in ('WORLD_SIZE', 'RANK', 'LOCAL_RANK', 'SA_DIST_BACKEND'):
        env.pop(k, None)
    p = subprocess.run([sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', '--nproc-per-node', '1',
                        '--master-addr', '127.0.0.1', '--master-port', '29533', 'bench.py', '--gpus', '1',
                        '--games', '20', '--steps', '2', '--warmup', '1', '--no-cpu', '--cfg5-games', '45',
                        '--atomic-games', '30', '--e2e-games', '5'], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=280)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith('{')]
    assert p.returncode == 0 and len(lines) == 1, p.stdout[-2000:] + p.stderr[-3000:]
    out = json.loads(lines[0])
    assert out['n_gpus'] == 1 and out['value'] > 0 and out['parity']['ok']
    for name in ('xt105_cfg5', 'atomic_cfg3', 'convert_to_atomic', 'rate_on_device'):
        assert 'error' not in out[name], (name, out[name])
    assert out['xt105_cfg5']['parity']['ok'] and out['atomic_cfg3']['parity']['ok']


def test_device_events_order_streams_and_time():
    """socceraction_amd.events.DeviceEvent (sa_event_*, no system-scope fence): a side stream
    that waits on an event recorded after a producer kernel sees the producer's writes, and a
    timing pair measures a positive duration, like torch.cuda.Event."""
    import torch
    from socceraction_amd import events
    main, side = torch.cuda.current_stream(), torch.cuda.Stream()
    x = torch.zeros(1 << 24, dtype=torch.float32, device='cuda')
    for _ in range(5):
        a, b = events.DeviceEvent(True), events.DeviceEvent(True)
        a.record(main)
        x.add_(1.0)  # producer on the main stream
        b.record(main)
        done = events.DeviceEvent().record(main)
        done.wait(side)
        with torch.cuda.stream(side):
            y = x.sum()  # consumer on the side stream
        events.DeviceEvent().record(side).wait(main)
        b.synchronize()
        assert a.elapsed_time(b) > 0
    torch.cuda.synchronize()
    assert float(y.item()) == 5.0 * (1 << 24)
