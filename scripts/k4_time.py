"""K4 (the band count's table pass, sa_xt_count_from_buckets_ex) over cfg5's 7 bucketed batches,
with and without the compact-row emission, HIP events."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from socceraction_amd import batch as B, ops, synthetic  # noqa: E402


def main():
    bs = [B.ActionBatch.from_columns(synthetic.spadl_games(10000, game_id0=k * 10000)) for k in range(7)]
    acc = ops.xt_zero_counts(105, 68, bs[0].device)
    parts = [ops.xt_bucket(b, 105, 68, acc.err) for b in bs]
    res = {}
    for rnd in range(3):
        for compact in (False, True):
            ops.xt_count_buckets(parts, 105, 68, acc, overwrite=True, compact=compact)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                ops.xt_count_buckets(parts, 105, 68, acc, overwrite=True, compact=compact)
            e1.record()
            torch.cuda.synchronize()
            res.setdefault('compact' if compact else 'dense_only', []).append(round(e0.elapsed_time(e1) / 10, 4))
    # the build pass over the dense table (sa_xt_compact_rows), what the solve runs without them
    from socceraction_amd import _native as N
    C = 105 * 68
    pe = int(N.lib().sa_xt_compact_bytes(C, 1)) // 4
    ell = torch.empty(C * pe, dtype=torch.int32, device=acc.trans.device)
    rl = torch.empty(C, dtype=torch.int32, device=acc.trans.device)
    st = torch.cuda.current_stream().cuda_stream
    for rnd in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            N.check(N.lib().sa_xt_compact_rows(acc.trans.data_ptr(), C, C, ell.data_ptr(), rl.data_ptr(), st))
        e1.record()
        torch.cuda.synchronize()
        res.setdefault('compact_rows_from_dense', []).append(round(e0.elapsed_time(e1) / 10, 4))
    print(json.dumps(res), flush=True)


if __name__ == '__main__':
    main()
