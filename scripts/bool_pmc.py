"""The bool feature kernel alone, block form and bitmap form (cfg2, 3 launches each), for
rocprofv3 counter passes:

    rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU ... -- python3 scripts/bool_pmc.py
"""
import copy
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from socceraction_amd import batch as B, catalog, ops, synthetic  # noqa: E402

SPADL_DEFAULT = ['actiontype_onehot', 'result_onehot', 'actiontype_result_onehot',
                 'bodypart_onehot', 'time', 'startlocation', 'endlocation', 'startpolar',
                 'endpolar', 'movement', 'team', 'time_delta', 'space_delta', 'goalscore']


def main():
    ab = B.ActionBatch.from_columns(synthetic.spadl_games(10000))
    plan = catalog.build_plan(SPADL_DEFAULT, 3)
    q = copy.copy(plan)  # bool families only
    q.struct = copy.deepcopy(plan.struct)
    for x in range(len(q.struct.bool_col)):
        q.struct.f64_col[x] = -1
        q.struct.i64_col[x] = -1
    blk = ops.alloc_feature_blocks(q, ab.n, ab.device, 1024, 128)
    bits = ops.features(ab, SPADL_DEFAULT, 3, num_tile=128, bool_bits=True)
    bits.plan = q
    for _ in range(3):
        ops.features_into(ab.struct(), blk)
    for _ in range(3):
        ops.features(ab, SPADL_DEFAULT, 3, out=bits)
    torch.cuda.synchronize()
    if '--time' in sys.argv:  # HIP-event ms per launch of each form (bool families only)
        res = {}
        for name, fn in (('block', lambda: ops.features_into(ab.struct(), blk)),
                         ('bitmaps', lambda: ops.features(ab, SPADL_DEFAULT, 3, out=bits))):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(10):
                fn()
            b.record()
            torch.cuda.synchronize()
            res[name] = round(a.elapsed_time(b) / 10, 4)
        print(res)
    print('done', ab.n)


if __name__ == '__main__':
    main()
