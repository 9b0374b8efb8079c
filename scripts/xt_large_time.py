"""cfg5's pieces on one GPU, each timed alone (HIP events / wall clock, medians of --reps calls):
the band-owned count of ``--batches`` device batches of 10k synthetic games (per-batch bucket
pass and the once-per-fit table pass), the large-grid solve (compact rows + value iteration,
host syncs included) and the interpolated rate from the bucket pass's operands.  For rocprofv3
kernel traces of the 105 x 68 fit.  Prints one JSON line.

    python scripts/xt_large_time.py [--batches 2] [--reps 10] [--l 105 --w 68]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from socceraction_amd import batch as B  # noqa: E402
from socceraction_amd import ops, synthetic  # noqa: E402


def _ms(fn, reps):
    fn()
    torch.cuda.synchronize()
    t = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        t.append((time.perf_counter() - t0) * 1e3)
    return round(float(np.median(t)), 4)


def _ev(fn, reps):
    """Median ms of ``reps`` calls, a HIP event pair around each (after one warm-up call)."""
    fn()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for a, b in ev:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    return round(float(np.median([a.elapsed_time(b) for a, b in ev])), 4)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--batches', type=int, default=2)
    ap.add_argument('--games', type=int, default=10000)
    ap.add_argument('--reps', type=int, default=10)
    ap.add_argument('--l', type=int, default=105)
    ap.add_argument('--w', type=int, default=68)
    args = ap.parse_args()
    l, w = args.l, args.w
    bs = [B.ActionBatch.from_columns(synthetic.spadl_games(args.games, game_id0=k * args.games))
          for k in range(args.batches)]
    dev = bs[0].device
    ic = [ops.xt_interp_codes_buffer(b.n, dev) for b in bs]
    out = {'n': sum(b.n for b in bs), 'batches': len(bs), 'grid': f'{l}x{w}',
           'band_shape': ops.xt_band_shape(l, w)}
    acc = ops.xt_count_many(bs, l, w, interp_codes=ic)
    err = acc.err
    parts = [ops.xt_bucket(b, l, w, err, interp_codes=c) for b, c in zip(bs, ic)]
    out['bucket_ms_per_batch'] = _ms(lambda: ops.xt_bucket(bs[0], l, w, err, interp_codes=ic[0]), args.reps)
    out['bucket_noicodes_ms_per_batch'] = _ms(lambda: ops.xt_bucket(bs[0], l, w, err), args.reps)
    out['table_ms'] = _ms(lambda: ops.xt_count_buckets(parts, l, w, acc, overwrite=True), args.reps)
    out['count_many_ms'] = _ms(lambda: ops.xt_count_many(bs, l, w, interp_codes=ic), args.reps)
    sol = ops.xt_solve(acc, transition=False)
    ex = ops.xt_solve(acc, transition=False, exact_order=True)
    out['iterations'] = sol.n_iter
    out['iterations_exact_order'] = ex.n_iter
    out['solve_path'] = sol.path
    h, r = sol.heatmaps.cpu().numpy(), ex.heatmaps.cpu().numpy()
    d = np.abs(h - r)
    out['heatmaps_max_rel_diff'] = float(np.max(np.where(d == 0, 0.0, d / np.maximum(np.abs(r), 1e-300))))
    out['solve_ms'] = _ms(lambda: ops.xt_solve(acc, transition=False), args.reps)
    out['solve_exact_order_ms'] = _ms(lambda: ops.xt_solve(acc, transition=False, exact_order=True), args.reps)
    # one value iteration alone (sa_xt_iterate_compact on the fitted counts, x = the surface)
    # and the compact form's build, HIP events
    from socceraction_amd import _native
    from socceraction_amd.batch import stream_handle
    lib, C = _native.lib(), l * w
    p = lambda t: t.data_ptr()  # noqa: E731
    ell = torch.empty(int(lib.sa_xt_compact_bytes(C, C)) // 4, dtype=torch.int32, device=dev)
    rl = torch.empty(C, dtype=torch.int32, device=dev)
    build = lambda: _native.check(lib.sa_xt_compact_rows(p(acc.trans), C, C, p(ell), p(rl),  # noqa: E731
                                                          stream_handle()))
    out['compact_build_ms'] = _ev(build, args.reps)
    gp = torch.empty((2, C), dtype=torch.float64, device=dev)
    mats = torch.empty((4, C), dtype=torch.float64, device=dev)
    _native.check(lib.sa_xt_probabilities(p(acc.shot), p(acc.goal), p(acc.move), C, p(mats), p(gp[0]),
                                          p(gp[1]), stream_handle()))
    xo = torch.empty(C, dtype=torch.float64, device=dev)
    fl = torch.zeros(1, dtype=torch.int32, device=dev)
    x = sol.mats[3].contiguous()
    it = lambda: _native.check(lib.sa_xt_iterate_compact(  # noqa: E731
        p(ell), p(rl), p(acc.trans), p(acc.move), p(gp[0]), p(gp[1]), C, 0, C, p(x), 1e-5, p(xo), None,
        p(fl), stream_handle()))
    out['iteration_ms'] = _ev(it, 3 * args.reps)
    # the whole reordered iteration from the prebuilt compact form (one launch + its host sync)
    t = lambda: ops.xt_solve_compact(ell, rl, acc.trans, acc.move, gp[0], gp[1], C)  # noqa: E731
    out['solve_compact_reordered_ms'] = _ms(t, args.reps)
    out['solve_compact_reordered_path'] = t()[2]
    out['solve_compact_exact_ms'] = _ms(lambda: ops.xt_solve_compact(ell, rl, acc.trans, acc.move, gp[0], gp[1], C,
                                                                     exact_order=True), args.reps)
    out['row_len_max'] = int(rl.max().item())
    out['row_len_mean'] = round(float(rl.float().mean().item()), 1)
    xT = sol.mats[3].reshape(w, l)
    axes = ops.xt_interp_axes(l, w, dev)
    out['rate_codes_ms_per_batch'] = _ms(lambda: ops.xt_rate_interp_codes(ic[0], bs[0].n, xT, l, w, axes=axes),
                                         args.reps)
    out['rate_coords_ms_per_batch'] = _ms(lambda: ops.xt_rate_interp(bs[0], xT, l, w, axes=axes), args.reps)
    print(json.dumps(out), flush=True)


if __name__ == '__main__':
    main()
