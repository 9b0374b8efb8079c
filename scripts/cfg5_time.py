"""cfg5 (xT 105x68 fit + interpolated rate of 62,500 synthetic games) timed as bench.py's
xt105_cfg5 entry does, in the library chosen with SOCCERACTION_AMD_LIB (A/B of builds across
processes), plus a checksum of the counts of a full batch and a 2,500-game tail batch (equal
across builds: the counts are integers)."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from socceraction_amd import _native as N, batch as B, ops, synthetic  # noqa: E402


def main():
    dev = torch.device('cuda', 0)
    d = synthetic.spadl_games(10000)
    ab = B.ActionBatch.from_columns(d, dev=dev)
    tail = B.ActionBatch.from_columns(synthetic.spadl_games(2500, game_id0=99_000_000), dev=dev)
    acc = ops.xt_count_many([ab, tail], 105, 68)
    h = torch.arange(1, acc.trans.numel() + 1, device=dev, dtype=torch.float64)
    csum = [int(acc.shot.sum()), int(acc.goal.sum()), int(acc.move.sum()),
            float((acc.trans.reshape(-1).to(torch.float64) * h).sum())]
    r = bench.xt105_extra(ab, None, dev, False, 62500, d=d, check=False)
    print(json.dumps({'lib': os.path.basename(N.LIB_PATH), 'ms': r['ms_fit_and_rate'],
                      'phases': {k: v for k, v in r['phases_ms'].items() if k != 'note'},
                      'counts_checksum': csum}), flush=True)


if __name__ == '__main__':
    main()
