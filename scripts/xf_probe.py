"""Phase times of the reordered large-grid solve (a probe build, -DSA_XF_PROBE=1: workgroup 0's
wall-clock ticks per phase printed to stderr by the library) on a cfg5-shaped 105 x 68 fit.

    SOCCERACTION_AMD_LIB=socceraction_amd/_lib/libsocceraction_amd_xfprobe.so \
        python scripts/xf_probe.py [--batches 7]
"""
import argparse
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from socceraction_amd import batch as B  # noqa: E402
from socceraction_amd import ops, synthetic  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--batches', type=int, default=7)
    ap.add_argument('--reps', type=int, default=5)
    args = ap.parse_args()
    bs = [B.ActionBatch.from_columns(synthetic.spadl_games(10000, game_id0=k * 10000))
          for k in range(args.batches)]
    acc = ops.xt_count_many(bs, 105, 68)
    for _ in range(args.reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        sol = ops.xt_solve(acc, transition=False)
        print(f'solve {sol.path} {sol.n_iter} iterations {(time.perf_counter() - t0) * 1e3:.3f} ms',
              file=sys.stderr, flush=True)


if __name__ == '__main__':
    main()
