"""Where one compact value iteration of the 105 x 68 fit spends its time: HIP-event medians of
sa_xt_iterate_compact over every row (the solve's launch), over the slice of 32 rows holding the
longest row alone (one workgroup: the launch's critical path without contention), over the
slice with the shortest rows alone (the fixed per-workgroup cost), and over the first k slices
for a few k.  Counts of ``--batches`` batches of 10k synthetic games.  Prints one JSON line.

    python scripts/xt_iter_probe.py [--batches 7]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from socceraction_amd import _native, ops, synthetic  # noqa: E402
from socceraction_amd import batch as B  # noqa: E402
from socceraction_amd.batch import stream_handle  # noqa: E402


def _ev(fn, reps):
    fn()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for a, b in ev:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    return round(float(np.median([a.elapsed_time(b) for a, b in ev])) * 1e3, 2)  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--batches', type=int, default=7)
    ap.add_argument('--reps', type=int, default=30)
    args = ap.parse_args()
    l, w = 105, 68
    bs = [B.ActionBatch.from_columns(synthetic.spadl_games(10000, game_id0=k * 10000))
          for k in range(args.batches)]
    dev = bs[0].device
    acc = ops.xt_count_many(bs, l, w)
    probe = os.environ.get('SOCCERACTION_AMD_LIB', '').split('_lib')[-1].startswith('/libsocceraction_amd_xtime')  # SA_XE_PROBE=16 build
    lib, C = _native.lib(), l * w
    p = lambda t: t.data_ptr()  # noqa: E731
    ell = torch.empty(int(lib.sa_xt_compact_bytes(C, C)) // 4, dtype=torch.int32, device=dev)
    pe = ell.numel() // C
    rl = torch.empty(C, dtype=torch.int32, device=dev)
    _native.check(lib.sa_xt_compact_rows(p(acc.trans), C, C, p(ell), p(rl), stream_handle()))
    gp = torch.empty((2, C), dtype=torch.float64, device=dev)
    mats = torch.empty((4, C), dtype=torch.float64, device=dev)
    _native.check(lib.sa_xt_probabilities(p(acc.shot), p(acc.goal), p(acc.move), C, p(mats), p(gp[0]),
                                          p(gp[1]), stream_handle()))
    xo = torch.empty(C, dtype=torch.float64, device=dev)
    fl = torch.zeros(1, dtype=torch.int32, device=dev)
    # the surface when the library is the product one, else (the probe build's values are
    # wrong, its solve would not converge) a random x in [0, 0.1)
    x = (torch.rand(C, dtype=torch.float64, device=dev) * 0.1 if probe
         else ops.xt_solve(acc, transition=False).mats[3].contiguous())
    lens = rl.cpu().numpy()
    ns = (C + 31) // 32
    slice_max = np.array([lens[32 * s:32 * s + 32].max() for s in range(ns)])

    def run(r0, nrows):
        return lambda: _native.check(lib.sa_xt_iterate_compact(
            p(ell) + 4 * r0 * pe, p(rl) + 4 * r0, p(acc.trans) + 4 * r0 * C, p(acc.move), p(gp[0]), p(gp[1]),
            C, r0, nrows, p(x), 1e-5, p(xo) + 8 * r0, None, p(fl), stream_handle()))

    out = {'row_len_max': int(lens.max()), 'slices': ns,
           'slice_max_len_pctl': {q: int(np.percentile(slice_max, q)) for q in (10, 50, 90, 100)}}
    out['all_us'] = _ev(run(0, C), args.reps)
    smax, smin = int(slice_max.argmax()), int(slice_max.argmin())
    out['longest_slice'] = {'slice': smax, 'len': int(slice_max[smax]), 'us': _ev(run(32 * smax, 32), args.reps)}
    out['shortest_slice'] = {'slice': smin, 'len': int(slice_max[smin]), 'us': _ev(run(32 * smin, 32), args.reps)}
    mid = int(np.argsort(slice_max)[ns // 2])
    out['median_slice'] = {'slice': mid, 'len': int(slice_max[mid]), 'us': _ev(run(32 * mid, 32), args.reps)}
    out['first_k_slices_us'] = {k: _ev(run(0, min(C, 32 * k)), args.reps) for k in (8, 32, 64, 128)}
    if probe:
        ph = {}
        for name, sl in (('longest', smax), ('shortest', smin), ('median', mid)):
            run(32 * sl, 32)()
            torch.cuda.synchronize()
            v = xo[32 * sl:32 * sl + 44].cpu().numpy()  # chunks, then 100 MHz ticks from entry
            ph[name] = {'chunks': int(v[0]), 'setup_us': v[1] / 100, 'chain_done_us': v[2] / 100,
                        'clk_product_wave0_work_barrier': [int(v[40]), int(v[41])],
                        'clk_chain_work_barrier': [int(v[42]), int(v[43])]}
        out['phases_one_workgroup'] = ph
    print(json.dumps(out), flush=True)


if __name__ == '__main__':
    main()
