"""The xT 16 x 12 count pass from cell codes alone (cfg2: 10k games, ~16M actions), timed with HIP
events for the default library and variant builds (``python -m socceraction_amd.build -DNAME=V
--variant=tag``) on the same cell codes:

    python scripts/xt_count_time.py --variants b128,noflush
"""
import argparse
import ctypes
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from socceraction_amd import _native as N  # noqa: E402
from socceraction_amd import batch as B, ops, synthetic  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--games', type=int, default=10000)
    ap.add_argument('--reps', type=int, default=20)
    ap.add_argument('--variants', default='')
    ap.add_argument('--large', action='store_true', help='105 x 68 from coordinates (cfg5)')
    args = ap.parse_args()
    libs = {'default': N.lib()}
    for v in [x for x in args.variants.split(',') if x]:
        libs[v] = N.load_library(os.path.join(ROOT, 'socceraction_amd', '_lib',
                                              f'libsocceraction_amd_{v}.so'))
    ab = B.ActionBatch.from_columns(synthetic.spadl_games(args.games))
    if args.large:
        return large(ab, libs, args.reps)
    cells = ops.xt_cells(ab, 16, 12)
    ref = ops.xt_count_cells(cells, ab.n, 16, 12)
    stream = torch.cuda.current_stream().cuda_stream
    out = {'n': ab.n, 'ms': {}, 'equal': {}}
    for rnd in range(3):
        for name, lib in libs.items():
            acc = ops.xt_zero_counts(16, 12, ab.device)

            def run():
                N.check(lib.sa_xt_count_cells(cells.data_ptr(), ab.n, 16, 12, acc.shot.data_ptr(),
                                              acc.goal.data_ptr(), acc.move.data_ptr(),
                                              acc.trans.data_ptr(), acc.err.data_ptr(), 0, stream))
            run()
            torch.cuda.synchronize()
            out['equal'][name] = bool(torch.equal(acc.trans, ref.trans) and torch.equal(acc.move, ref.move))
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(args.reps):
                run()
            b.record()
            torch.cuda.synchronize()
            out['ms'].setdefault(name, []).append(round(a.elapsed_time(b) / args.reps, 4))
    print(json.dumps(out), flush=True)


def large(ab, libs, reps):
    """The 105 x 68 count pass from coordinates (sa_xt_count), per library."""
    import ctypes
    ref = ops.xt_count(ab, 105, 68)
    stream = torch.cuda.current_stream().cuda_stream
    s = ab.struct()
    out = {'n': ab.n, 'grid': '105x68', 'ms': {}, 'equal': {}}
    for rnd in range(3):
        for name, lib in libs.items():
            acc = ops.xt_zero_counts(105, 68, ab.device)

            def run():
                N.check(lib.sa_xt_count(ctypes.byref(s), 105, 68, acc.shot.data_ptr(), acc.goal.data_ptr(),
                                        acc.move.data_ptr(), acc.trans.data_ptr(), acc.err.data_ptr(), stream))
            run()
            torch.cuda.synchronize()
            out['equal'][name] = bool(torch.equal(acc.trans, ref.trans) and torch.equal(acc.move, ref.move)
                                      and torch.equal(acc.shot, ref.shot) and torch.equal(acc.goal, ref.goal))
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(reps):
                run()
            b.record()
            torch.cuda.synchronize()
            out['ms'].setdefault(name, []).append(round(a.elapsed_time(b) / reps, 4))
    print(json.dumps(out), flush=True)


if __name__ == '__main__':
    main()
