"""The f64 / i64 feature kernel alone (cfg2, 3 launches, with and without the xT cell codes)
for rocprofv3 counter passes."""
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
    q = copy.copy(plan)  # f64 / i64 families only, goalscore excluded
    q.struct = copy.deepcopy(plan.struct)
    gsx = _gs_index()
    for x in range(len(q.struct.bool_col)):
        q.struct.bool_col[x] = -1
        if x == gsx:
            q.struct.i64_col[x] = -1
    blk = ops.alloc_feature_blocks(q, ab.n, ab.device, 1024, 128)
    cells = ops.xt_cells_buffer(ab.n, ab.device)
    s = ab.struct()
    for _ in range(3):
        ops.features_into(s, blk)
    for _ in range(3):
        ops.features_into(s, blk, xt_cells=(16, 12, cells))
    torch.cuda.synchronize()
    print('done', ab.n)


def _gs_index():
    from socceraction_amd import _native
    return _native.XFN_NAMES.index('goalscore')


if __name__ == '__main__':
    main()
