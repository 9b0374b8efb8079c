"""cfg5's fit + rate (bench.py xt105_extra, one GPU) in isolation, for a rocprofv3 kernel trace
of its timeline: 7 device batches of 10k synthetic games (~1.1e8 actions), band-owned count,
reordered solve, interpolated rate from the count pass's operands; `--calls` calls, each
bracketed by synchronisations (the trace's gaps between them mark the calls).

    rocprofv3 --kernel-trace --output-format csv -d out -o run -- python3 scripts/cfg5_trace.py
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--batches', type=int, default=7)
    ap.add_argument('--calls', type=int, default=5)
    args = ap.parse_args()
    l, w = 105, 68
    bs = [B.ActionBatch.from_columns(synthetic.spadl_games(10000, game_id0=k * 10000))
          for k in range(args.batches)]
    dev = bs[0].device
    ic = [ops.xt_interp_codes_buffer(b.n, dev) for b in bs]
    ro = [torch.empty(max(b.n, 16), dtype=torch.float64, device=dev) for b in bs]
    axes = ops.xt_interp_axes(l, w, dev)

    def once():
        acc = ops.xt_count_many(bs, l, w, interp_codes=ic, dense=False)
        sol = ops.xt_solve(acc, transition=False)
        xT = sol.mats[3].reshape(w, l)
        ops.xt_rate_interp_codes_many(ic, [b.n for b in bs], xT, l, w, 1050, 680, axes=axes,
                                      outs=ro)
        return sol
    once()
    torch.cuda.synchronize()
    t = []
    for _ in range(args.calls):
        time.sleep(0.002)  # a visible gap between calls in the trace
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        sol = once()
        torch.cuda.synchronize()
        t.append((time.perf_counter() - t0) * 1e3)
    print(json.dumps({'n': sum(b.n for b in bs), 'iterations': sol.n_iter, 'path': sol.path,
                      'ms': [round(x, 3) for x in t], 'median_ms': round(float(np.median(t)), 3)}), flush=True)


if __name__ == '__main__':
    main()
