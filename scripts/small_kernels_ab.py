"""A/B of the goalscore and labels launch variants on the cfg2 batch, in one process (the
library reads SA_GS_KERNEL / SA_LABELS_SEARCH at each launch); outputs must be equal.

    python scripts/small_kernels_ab.py [--games 10000] [--reps 20]
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from socceraction_amd import batch as B  # noqa: E402
from socceraction_amd import catalog, ops, synthetic  # noqa: E402

SPADL_DEFAULT = ['actiontype_onehot', 'result_onehot', 'actiontype_result_onehot',
                 'bodypart_onehot', 'time', 'startlocation', 'endlocation', 'startpolar',
                 'endpolar', 'movement', 'team', 'time_delta', 'space_delta', 'goalscore']


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return round(a.elapsed_time(b) / reps, 4)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--games', type=int, default=10000)
    ap.add_argument('--reps', type=int, default=20)
    ap.add_argument('--atomic', action='store_true')
    args = ap.parse_args()
    dev = B.device()
    gen = synthetic.atomic_games if args.atomic else synthetic.spadl_games
    ab = B.ActionBatch.from_columns(gen(args.games), atomic=args.atomic, dev=dev)
    n = ab.n
    plan = catalog.build_plan(SPADL_DEFAULT if not args.atomic else
                              ['actiontype', 'goalscore'], 3, atomic=args.atomic)
    out = ops.alloc_feature_blocks(plan, n, dev, bool_tile=1024, num_tile=128)
    ld = (n + 15) // 16 * 16
    lab_buf = torch.zeros((3, ld), dtype=torch.uint8, device=dev)
    lab = ops.LabelBlocks(n, lab_buf[0], lab_buf[1], lab_buf[2])
    res = {'n': n, 'games': args.games, 'atomic': args.atomic}
    gs_ref = None
    for v in ('wave2', 'wave16'):
        os.environ['SA_GS_KERNEL'] = v
        out.i64_block.zero_()
        res[f'goalscore_{v}_ms'] = timed(lambda: ops.goalscore_into(ab, out), args.reps)
        got = out.i64_block.clone()
        if gs_ref is None:
            gs_ref = got
        else:
            res['goalscore_equal'] = bool(torch.equal(gs_ref, got))
    lab_ref = None
    for v in ('lane', 'wave'):
        os.environ['SA_LABELS_SEARCH'] = v
        lab_buf.zero_()
        res[f'labels_{v}_ms'] = timed(lambda: ops.labels(ab, 10, lab), args.reps)
        got = lab_buf.clone()
        if lab_ref is None:
            lab_ref = got
        else:
            res['labels_equal'] = bool(torch.equal(lab_ref, got))
    from socceraction_amd import synthetic as syn_
    pr = syn_.probabilities(n)
    ps = torch.from_numpy(pr['scores']).to(dev)
    pc = torch.from_numpy(pr['concedes']).to(dev)
    val = torch.zeros((3, ld), dtype=torch.float64, device=dev)
    f_ref = None
    for v in ('lane', 'wave'):
        os.environ['SA_FORMULA_SEARCH'] = v
        val.zero_()
        res[f'formula_{v}_ms'] = timed(lambda: ops.formula(ab, ps, pc, val), args.reps)
        got = val.clone()
        if f_ref is None:
            f_ref = got
        else:
            res['formula_equal'] = bool(torch.equal(f_ref, got))
    for k in ('SA_GS_KERNEL', 'SA_LABELS_SEARCH', 'SA_FORMULA_SEARCH'):
        os.environ.pop(k, None)
    print(json.dumps(res), flush=True)


if __name__ == '__main__':
    main()
