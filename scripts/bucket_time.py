"""Time the per-batch bucket pass of the band-owned count (K1 + K2 + K3, ``ops.xt_bucket``) on
one 10k-game batch with HIP events -- for A/B of library builds chosen with
SOCCERACTION_AMD_LIB (probe builds may write wrong keys; only the time is read)."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from socceraction_amd import batch as B, ops, synthetic  # noqa: E402


def main():
    b = B.ActionBatch.from_columns(synthetic.spadl_games(10000))
    ic = ops.xt_interp_codes_buffer(b.n, b.device)
    err = torch.zeros(1, dtype=torch.int32, device=b.device)
    for _ in range(3):
        ops.xt_bucket(b, 105, 68, err, interp_codes=ic)
    torch.cuda.synchronize()
    out = []
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            ops.xt_bucket(b, 105, 68, err, interp_codes=ic)
        e1.record()
        torch.cuda.synchronize()
        out.append(round(e0.elapsed_time(e1) / 10, 4))
    print(json.dumps({'lib': os.environ.get('SOCCERACTION_AMD_LIB', 'default'), 'n': b.n,
                      'bucket_ms': out}), flush=True)


if __name__ == '__main__':
    main()
