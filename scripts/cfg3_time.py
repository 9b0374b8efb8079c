"""cfg3 (Atomic-VAEP features + labels of 10k synthetic atomic games) timed as bench.py's
atomic_extra does, N times in one process, optionally after the main line's allocations
(--after-step: the cfg2 batch and its feature blocks allocated first, as in the bench)."""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from socceraction_amd import batch as B, ops, synthetic  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--times', type=int, default=3)
    ap.add_argument('--after-step', action='store_true')
    ap.add_argument('--contiguous', default='require')
    ap.add_argument('--batch-contiguous', action='store_true')
    ap.add_argument('--reps', type=int, default=21)
    ap.add_argument('--warm-games', type=int, default=0,
                    help='one untimed cfg3 pass of this many games before the timed runs')
    ap.add_argument('--pre-mb', type=int, default=0,
                    help='a contiguous dummy range of this size held before the first run')
    args = ap.parse_args()
    dev = torch.device('cuda', 0)
    keep = []
    addrs = []  # device addresses of each run's batch buffer and blocks (layout vs speed)
    _alloc, _from = ops.alloc_feature_blocks, B.ActionBatch.from_columns

    def alloc(*a, **k):
        o = _alloc(*a, **k)
        addrs[-1].update(bool=hex(o.bool_block.data_ptr()), f64=hex(o.f64_block.data_ptr()),
                         i64=hex(o.i64_block.data_ptr()))
        return o

    def from_columns(*a, **k):
        o = _from(*a, **k)
        addrs.append({'batch': hex(o.buffer.data_ptr()), 'batch_mb': o.buffer.numel() >> 20})
        return o
    ops.alloc_feature_blocks, B.ActionBatch.from_columns = alloc, from_columns
    if args.pre_mb:
        keep.append(ops.DeviceBuffer(args.pre_mb << 20, contiguous=True))
    if args.after_step:
        ab = B.ActionBatch.from_columns(synthetic.spadl_games(10000))
        out = ops.alloc_feature_blocks(ops.build_plan(bench.SPADL_DEFAULT, 3, False), ab.n, dev, 1024, 128,
                                       contiguous=True)
        keep += [ab, out]
    res = []
    if args.warm_games:
        bench.atomic_extra(None, 0, 1, dev, args.warm_games, check=False, contiguous=args.contiguous)
        torch.cuda.empty_cache()
    for _ in range(args.times):
        r = bench.atomic_extra(None, 0, 1, dev, 10000, check=False, contiguous=args.contiguous,
                               batch_contiguous=args.batch_contiguous, reps=args.reps)
        series = [round(x, 3) for x in bench._LAST_TIMES]
        res.append((r['ms_per_step'], r['bool_block'], r['timing'], addrs[-1],
                    [float(np.median(series[i:i + 10])) for i in range(0, len(series), 10)]))
        torch.cuda.empty_cache()
    print(json.dumps({'after_step': args.after_step, 'contiguous': args.contiguous, 'pre_mb': args.pre_mb, 'warm_games': args.warm_games,
                      'batch_contiguous': args.batch_contiguous,
                      'runs': res}), flush=True)


if __name__ == '__main__':
    main()
