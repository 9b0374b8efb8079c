"""A/B of library builds for the f64/i64 feature kernel on the SAME allocations: the default
library and variant builds (``python -m socceraction_amd.build -DNAME=V --variant=tag``) are
loaded into one process, several f64/i64 output blocks are kept alive, and every library's
``sa_vaep_features`` (num-only plan) is timed on each allocation with HIP events.

    python scripts/num_kernel_ab.py --allocs 4 --variants minw5,minw6,noatan
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
from socceraction_amd._native import XFN  # noqa: E402

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
        q.struct.bool_col[x] = -1
        if x == XFN['goalscore']:
            q.struct.i64_col[x] = -1
    s = ab.struct()
    nt = -(-n // 128)
    stream = torch.cuda.current_stream().cuda_stream
    keep = []
    out = {'n': n, 'ms': {v: [] for v in libs}, 'equal': {}}
    for a in range(args.allocs):
        fb = torch.empty((nt, plan.n_f64, 128), dtype=torch.float64, device=dev)
        ib = torch.empty((nt, plan.n_i64, 128), dtype=torch.int64, device=dev)
        keep += [fb, ib]
        bf, bi = N.SaBlock(), N.SaBlock()
        bf.data, bf.n_cols, bf.tile_rows = fb.data_ptr(), plan.n_f64, 128
        bi.data, bi.n_cols, bi.tile_rows = ib.data_ptr(), plan.n_i64, 128
        ref = None
        for v, lib in libs.items():
            def run():
                N.check(lib.sa_vaep_features(ctypes.byref(s), ctypes.byref(q.struct), None,
                                             ctypes.byref(bf), ctypes.byref(bi), stream))
            fb.zero_()
            run()
            torch.cuda.synchronize()
            if ref is None:
                ref = (fb.clone(), ib.clone())
            elif not v.startswith('no'):  # probe builds compute wrong values on purpose
                out['equal'].setdefault(v, True)
                out['equal'][v] &= bool(torch.equal(ref[0], fb) and torch.equal(ref[1], ib))
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.reps):
                run()
            e1.record()
            torch.cuda.synchronize()
            out['ms'][v].append(round(e0.elapsed_time(e1) / args.reps, 4))
        del ref
        print(json.dumps({'alloc': a, **{v: out['ms'][v][-1] for v in libs}}), flush=True)
    print(json.dumps(out))


if __name__ == '__main__':
    main()
