"""A/B of bool-block kernel builds on the SAME allocations: the default library and variant
builds (``python -m socceraction_amd.build -DNAME=V --variant=tag``) are loaded into one process,
several bool output blocks are kept alive (each lands at its own physical placement) and every
library's ``sa_vaep_features`` (bool-only plan, cfg2) is timed on each with HIP events; outputs
must be byte-identical.

    python scripts/bool_ab.py --allocs 4 --variants strided
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

from socceraction_amd import _native as N  # noqa: E402
from socceraction_amd import batch as B  # noqa: E402
from socceraction_amd import catalog, synthetic  # noqa: E402

SPADL_DEFAULT = ['actiontype_onehot', 'result_onehot', 'actiontype_result_onehot',
                 'bodypart_onehot', 'time', 'startlocation', 'endlocation', 'startpolar',
                 'endpolar', 'movement', 'team', 'time_delta', 'space_delta', 'goalscore']


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--games', type=int, default=10000)
    ap.add_argument('--allocs', type=int, default=4)
    ap.add_argument('--reps', type=int, default=10)
    ap.add_argument('--variants', default='')
    args = ap.parse_args()
    libs = {'default': N.lib()}
    for v in [x for x in args.variants.split(',') if x]:
        libs[v] = N.load_library(os.path.join(ROOT, 'socceraction_amd', '_lib',
                                              f'libsocceraction_amd_{v}.so'))
    dev = B.device()
    ab = B.ActionBatch.from_columns(synthetic.spadl_games(args.games), dev=dev)
    n = ab.n
    plan = catalog.build_plan(SPADL_DEFAULT, 3)
    q = copy.copy(plan)
    q.struct = copy.deepcopy(plan.struct)
    for x in range(len(q.struct.bool_col)):
        q.struct.f64_col[x] = -1
        q.struct.i64_col[x] = -1
    s = ab.struct()
    nt = -(-n // 1024)
    stream = torch.cuda.current_stream().cuda_stream
    keep = []
    out = {'n': n, 'bytes_per_action': 522, 'ms': {v: [] for v in libs}, 'equal': {}}
    for a in range(args.allocs):
        bb = torch.empty((nt, plan.n_bool, 1024), dtype=torch.uint8, device=dev)
        keep.append(bb)
        blk = N.SaBlock()
        blk.data, blk.n_cols, blk.tile_rows = bb.data_ptr(), plan.n_bool, 1024
        ref = None
        for v, lib in libs.items():
            def run():
                N.check(lib.sa_vaep_features(ctypes.byref(s), ctypes.byref(q.struct),
                                             ctypes.byref(blk), None, None, stream))
            bb.zero_()
            run()
            torch.cuda.synchronize()
            if ref is None:
                ref = bb.clone()
            else:
                out['equal'].setdefault(v, True)
                out['equal'][v] &= bool(torch.equal(ref, bb))
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.reps):
                run()
            e1.record()
            torch.cuda.synchronize()
            out['ms'][v].append(round(e0.elapsed_time(e1) / args.reps, 4))
        del ref
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        bb.fill_(1)
        e0.record()
        for _ in range(args.reps):
            bb.fill_(1)
        e1.record()
        torch.cuda.synchronize()
        out['ms'].setdefault('torch_fill', []).append(round(e0.elapsed_time(e1) / args.reps, 4))
        print(json.dumps({'alloc': a, 'va': hex(bb.data_ptr()),
                          **{v: out['ms'][v][-1] for v in out['ms']}}), flush=True)
    print(json.dumps(out), flush=True)


if __name__ == '__main__':
    main()
