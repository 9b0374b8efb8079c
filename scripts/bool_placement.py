"""Tile-stride sweep: the feature kernels' time depends on how many (unwritten) padding columns
each record-batch tile carries, i.e. on the tile stride in memory.  For each padding the
blocks are allocated several times in ONE process (earlier allocations kept alive, so each
trial lands at a different address) and the kernel is timed with HIP events.

    python scripts/bool_placement.py bool --pads 0,1,5 [--trials 3]
    python scripts/bool_placement.py num --pads 0,1,5 [--ipads 0,2]

SOCCERACTION_AMD_LIB selects an A/B build of the library (scripts/ab_sweep.py convention).
"""
import argparse
import copy
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from socceraction_amd import batch as B  # noqa: E402
from socceraction_amd import catalog, ops, synthetic  # noqa: E402
from socceraction_amd._native import XFN  # noqa: E402

SPADL_DEFAULT = ['actiontype_onehot', 'result_onehot', 'actiontype_result_onehot',
                 'bodypart_onehot', 'time', 'startlocation', 'endlocation', 'startpolar',
                 'endpolar', 'movement', 'team', 'time_delta', 'space_delta', 'goalscore']


def timed(fn, reps=10):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('kind', choices=('bool', 'num'))
    ap.add_argument('--games', type=int, default=10000)
    ap.add_argument('--trials', type=int, default=3)
    ap.add_argument('--pads', default='0,1')
    ap.add_argument('--ipads', default='0')
    ap.add_argument('--keep', type=int, default=3, help='allocations kept alive at a time')
    args = ap.parse_args()
    dev = B.device()
    d = synthetic.spadl_games(args.games)
    ab = B.ActionBatch.from_columns(d, dev=dev)
    n = ab.n
    plan = catalog.build_plan(SPADL_DEFAULT, 3)
    q = copy.copy(plan)
    q.struct = copy.deepcopy(plan.struct)
    for x in range(len(q.struct.bool_col)):
        if args.kind == 'bool':
            q.struct.f64_col[x] = -1
            q.struct.i64_col[x] = -1
        else:
            q.struct.bool_col[x] = -1
            if x == XFN['goalscore']:
                q.struct.i64_col[x] = -1
    s = ab.struct()
    keep, res = [], {}
    nb = -(-n // 1024)
    nn = -(-n // 128)
    bytes_pa = 522 if args.kind == 'bool' else 448
    for pad in [int(p) for p in args.pads.split(',')]:
        for ipad in [int(p) for p in args.ipads.split(',')]:
            for t in range(args.trials):
                if args.kind == 'bool':
                    bb = torch.empty((nb, plan.n_bool + pad, 1024), dtype=torch.uint8, device=dev)
                    fb_ = torch.empty((1, 0, 128), dtype=torch.float64, device=dev)
                    ib_ = torch.empty((1, 0, 128), dtype=torch.int64, device=dev)
                    keep.append(bb)
                else:
                    bb = torch.empty((1, 0, 1024), dtype=torch.uint8, device=dev)
                    fb_ = torch.empty((nn, plan.n_f64 + pad, 128), dtype=torch.float64, device=dev)
                    ib_ = torch.empty((nn, plan.n_i64 + ipad, 128), dtype=torch.int64, device=dev)
                    keep.append((fb_, ib_))
                fb = ops.FeatureBlocks(q, n, 1024, 128, bb, fb_, ib_)
                ms = timed(lambda: ops.features_into(s, fb))
                key = f'pad{pad}' + (f'_ipad{ipad}' if args.kind == 'num' else '')
                res.setdefault(key, []).append(round(ms, 4))
                print(json.dumps({'kind': args.kind, 'pad': pad, 'ipad': ipad, 'trial': t,
                                  'ms': round(ms, 4),
                                  'TBps': round(bytes_pa * n / ms * 1e-9, 3)}), flush=True)
                if len(keep) > args.keep:
                    keep.pop(0)
    print(json.dumps(res))


if __name__ == '__main__':
    main()
