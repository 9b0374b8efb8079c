"""Multi-rank rehearsal of the row-sharded xT fit (shard.xt_solve_sharded), launched from the
command line (never spawned from a process that already initialised the GPU):

    python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
        --master-port 29541 scripts/rehearse_xt_sharded.py [--games 400] [--grid 105x68]

Every rank counts its own games; the sharded solve (all-reduce of the count vectors,
reduce-scatter of the transition-count rows, per-iteration all-gather of x) must reproduce,
bit for bit, the single-GPU fit of all ranks' games together, which rank 0 recomputes.
SA_DIST_BACKEND=gloo rehearses several ranks on one GPU (collectives staged through host
memory); with nccl (RCCL over xGMI) each rank needs its own GPU. Prints one JSON line.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from socceraction_amd import batch as B  # noqa: E402
from socceraction_amd import ops, shard, synthetic  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--games', type=int, default=400, help='games per rank')
    ap.add_argument('--grid', default='105x68', help='l x w cells')
    ap.add_argument('--mode', default='auto', choices=('auto', 'bands', 'bands-rows', 'rows'),
                    help='bands: shard.xt_fit_bands_sharded (all-to-all of the counted actions, '
                         'the compact rows all-gathered once); bands-rows: the same count, '
                         'row-sharded iteration; '
                         'rows: xt_solve_sharded (reduce-scatter of the count table); auto: bands '
                         'where the band-owned count holds the grid')
    args = ap.parse_args()
    backend = os.environ.get('SA_DIST_BACKEND', 'nccl')
    lr = int(os.environ.get('LOCAL_RANK', '0'))
    torch.cuda.set_device(lr % torch.cuda.device_count())
    if backend == 'nccl':
        dist.init_process_group('nccl', device_id=torch.device('cuda', torch.cuda.current_device()))
    else:
        dist.init_process_group(backend)
    rank, world = dist.get_rank(), dist.get_world_size()
    dev = B.device()
    l, w = map(int, args.grid.split('x'))
    d = synthetic.spadl_games(args.games, game_id0=rank * args.games)
    ab = B.ActionBatch.from_columns(d, dev=dev)

    mode = args.mode
    if mode == 'auto':
        mode = 'bands' if ops.xt_band_shape(l, w) is not None else 'rows'

    stats = {}

    def fit():
        if mode in ('bands', 'bands-rows'):
            mats, heat, iters, err = shard.xt_fit_bands_sharded(
                [ab], l, w, solve='rows' if mode == 'bands-rows' else 'compact', stats=stats)
            assert int(err.item()) == 0
            return mats, heat, iters
        acc = ops.xt_zero_counts(l, w, dev, row_blocks=world)
        ops.xt_count(ab, l, w, acc)
        return shard.xt_solve_sharded(acc)
    fit()  # warm-up
    torch.cuda.synchronize()
    dist.barrier()
    t0 = time.perf_counter()
    mats, heat, iters = fit()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    out = {'rank': rank, 'world': world, 'backend': backend, 'grid': f'{l}x{w}', 'mode': mode,
           'actions_this_rank': ab.n, 'iterations': iters, 'ms_sharded_fit': round(dt * 1e3, 3),
           'exchange': stats}
    if rank == 0:
        cols = [synthetic.spadl_games(args.games, game_id0=r * args.games) for r in range(world)]
        acc = ops.xt_zero_counts(l, w, dev)
        for c in cols:
            ops.xt_count(B.ActionBatch.from_columns(c, dev=dev), l, w, acc)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        # the bands mode's replicated iteration is the single-GPU solve itself (reordered sums
        # under the error bound); the row-sharded iterations sum in the reference's order
        # (ranks sharing one GPU: a persistent solve that could not hold every CU falls back to
        # the reference's order; compare with the path the sharded fit took)
        sol = ops.xt_solve(acc, exact_order=mode in ('rows', 'bands-rows') or
                           stats.get('solve_path', 'reordered') != 'reordered')
        torch.cuda.synchronize()
        out['ms_single_solve'] = round((time.perf_counter() - t0) * 1e3, 3)
        out['single_iterations'] = sol.n_iter
        out['bit_identical_matrices'] = bool(torch.equal(sol.mats, mats))
        out['bit_identical_heatmaps'] = bool(sol.n_iter == iters and torch.equal(sol.heatmaps, heat))
        out['ok'] = out['bit_identical_matrices'] and out['bit_identical_heatmaps']
        print(json.dumps(out), flush=True)
    dist.barrier()
    dist.destroy_process_group()
    if rank == 0 and not out['ok']:
        sys.exit(1)


if __name__ == '__main__':
    main()
