"""Standalone timing of the xT 16 x 12 fit pieces on cfg4's actions (10k synthetic games):
count pass (coordinates and cell codes), value iteration (sa_xt_solve) and rate, each on an
otherwise idle GPU, HIP events on the current stream.  Prints one JSON line.

    python scripts/xt_solve_time.py [--games 10000] [--reps 10]
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from socceraction_amd import batch as B  # noqa: E402
from socceraction_amd import ops, synthetic  # noqa: E402


def _ms(fn, reps):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return round(a.elapsed_time(b) / reps, 4)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--games', type=int, default=10000)
    ap.add_argument('--reps', type=int, default=10)
    ap.add_argument('--large', action='store_true', help='also time the 105 x 68 solve (cfg5)')
    args = ap.parse_args()
    ab = B.ActionBatch.from_columns(synthetic.spadl_games(args.games))
    cells = ops.xt_cells(ab, 16, 12)
    acc = ops.xt_count(ab, 16, 12)
    out = {'n': ab.n}
    out['count_coords_ms'] = _ms(lambda: ops.xt_count(ab, 16, 12), args.reps)
    out['count_cells_ms'] = _ms(lambda: ops.xt_count_cells(cells, ab.n, 16, 12), args.reps)
    out['count_cells_shared_ms'] = _ms(lambda: ops.xt_count_cells(cells, ab.n, 16, 12, shared=True),
                                       args.reps)
    out['cells_ms'] = _ms(lambda: ops.xt_cells(ab, 16, 12, out=cells), args.reps)
    sol = ops.xt_solve(acc)
    out['iterations'] = sol.n_iter
    out['solve_ms_incl_host_sync'] = _ms(lambda: ops.xt_solve(acc), args.reps)
    grid = sol.mats[3]
    out['rate_cells_ms'] = _ms(lambda: ops.xt_rate_cells(cells, ab.n, 16, 12, grid), args.reps)
    if args.large:
        big = ops.xt_count(ab, 105, 68)
        # sa_xt_count of one batch into a zeroed accumulator (band-owned: buckets + the table
        # read and written once; the atomics variant build: XC_VEC global atomics)
        out['count_105x68_ms'] = _ms(lambda: ops.xt_count(ab, 105, 68), args.reps)
        # the fit's form (bench cfg5): a fresh accumulator, the table written without a read
        out['count_many_105x68_ms'] = _ms(lambda: ops.xt_count_many([ab], 105, 68), args.reps)
        # random int32 atomics of the same number and spread into a 105x68 transition table
        # (torch index_add_: one global atomic per element), the old pass's ceiling
        C = 105 * 68
        tbl = torch.zeros(C * C, dtype=torch.int32, device=ab.device)
        idx = torch.randint(0, C * C, (int(big.trans.sum().item()),), device=ab.device)
        one = torch.ones(idx.numel(), dtype=torch.int32, device=ab.device)
        out['random_int32_atomics'] = idx.numel()
        out['random_int32_atomics_ms'] = _ms(lambda: tbl.index_add_(0, idx, one), args.reps)
        sol = ops.xt_solve(big)
        out['iterations_105x68'] = sol.n_iter
        out['solve_105x68_ms_incl_host_sync'] = _ms(lambda: ops.xt_solve(big), args.reps)
        out['solve_105x68_no_transition_ms'] = _ms(lambda: ops.xt_solve(big, transition=False),
                                                   args.reps)
    print(json.dumps(out), flush=True)


if __name__ == '__main__':
    main()
