"""A/B of the bool-block kernels on the SAME allocations: several bool blocks are kept alive
(each lands at a different physical placement) and every variant (SA_BOOL_KERNEL, read by the
library at each launch) is timed on each of them with HIP events; every variant's block must
equal the column-group kernel's byte for byte.  ``torch_fill`` times ``fill_`` of the same
block (the allocation's store ceiling for a one-store-per-thread pattern).

    python scripts/bool_kernel_ab.py --allocs 5 --variants colgroup,staged:4:4,staged:16:1
"""
import argparse
import copy
import ctypes
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from socceraction_amd import batch as B  # noqa: E402
from socceraction_amd import catalog, synthetic  # noqa: E402
from socceraction_amd import _native as N  # noqa: E402

SPADL_DEFAULT = ['actiontype_onehot', 'result_onehot', 'actiontype_result_onehot',
                 'bodypart_onehot', 'time', 'startlocation', 'endlocation', 'startpolar',
                 'endpolar', 'movement', 'team', 'time_delta', 'space_delta', 'goalscore']


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--games', type=int, default=10000)
    ap.add_argument('--allocs', type=int, default=5)
    ap.add_argument('--reps', type=int, default=10)
    ap.add_argument('--variants', default='colgroup,staged:4:4')
    args = ap.parse_args()
    dev = B.device()
    d = synthetic.spadl_games(args.games)
    ab = B.ActionBatch.from_columns(d, dev=dev)
    n = ab.n
    plan = catalog.build_plan(SPADL_DEFAULT, 3)
    q = copy.copy(plan)
    q.struct = copy.deepcopy(plan.struct)
    for x in range(len(q.struct.bool_col)):
        q.struct.f64_col[x] = -1
        q.struct.i64_col[x] = -1
    s = ab.struct()
    nb = -(-n // 1024)
    variants = args.variants.split(',')
    stream = torch.cuda.current_stream().cuda_stream
    blocks = []
    out = {'n': n, 'variants': variants, 'ms': {v: [] for v in variants}, 'equal': {}}
    for a in range(args.allocs):
        bb = torch.empty((nb, plan.n_bool, 1024), dtype=torch.uint8, device=dev)
        blocks.append(bb)
        bd = N.SaBlock()
        bd.data, bd.n_cols, bd.tile_rows = bb.data_ptr(), plan.n_bool, 1024
        ref = None
        for v in variants:
            # "lib:NAME@KERNEL" = variant build NAME with SA_BOOL_KERNEL=KERNEL
            lv, _, kv = v.partition('@')
            os.environ['SA_BOOL_KERNEL'] = kv if lv.startswith('lib:') and kv else v
            bb.zero_()

            lib = N.lib()
            if lv.startswith('lib:'):  # a variant build loaded next to the default library
                lib = N.load_library(os.path.join(ROOT, 'socceraction_amd', '_lib',
                                                  f'libsocceraction_amd_{lv[4:]}.so'))

            def run():
                if v == 'torch_fill':  # store ceiling of this allocation: torch's fill kernel
                    bb.fill_(1)
                    return
                N.check(lib.sa_vaep_features(ctypes.byref(s), ctypes.byref(q.struct),
                                                 ctypes.byref(bd), None, None, stream))
            run()
            torch.cuda.synchronize()
            if v == 'torch_fill':
                pass
            elif ref is None:
                ref = bb.clone()
            else:
                out['equal'].setdefault(v, True)
                out['equal'][v] &= bool(torch.equal(ref, bb))
            run()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.reps):
                run()
            e1.record()
            torch.cuda.synchronize()
            out['ms'][v].append(round(e0.elapsed_time(e1) / args.reps, 4))
        del ref
        print(json.dumps({'alloc': a, **{v: out['ms'][v][-1] for v in variants}}), flush=True)
    os.environ.pop('SA_BOOL_KERNEL', None)
    out['tbs'] = {v: [round(522 * n / (m * 1e-3) / 1e12, 3) for m in out['ms'][v]]
                  for v in variants}
    print(json.dumps(out))


if __name__ == '__main__':
    main()
