"""A/B of the feature kernels across library builds on the SAME blocks: the default library and
variant builds (``python -m socceraction_amd.build -DNAME=V --variant=tag``) time
``sa_vaep_features`` (numeric families only, and the whole plan) on one batch with HIP events,
round-robin; outputs must be byte-identical.

    python scripts/feature_lib_ab.py --atomic --games 10000 --variants w4
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
from socceraction_amd import batch as B, catalog, ops, synthetic  # noqa: E402

SPADL_DEFAULT = ['actiontype_onehot', 'result_onehot', 'actiontype_result_onehot',
                 'bodypart_onehot', 'time', 'startlocation', 'endlocation', 'startpolar',
                 'endpolar', 'movement', 'team', 'time_delta', 'space_delta', 'goalscore']
ATOMIC_DEFAULT = ['actiontype', 'actiontype_onehot', 'bodypart', 'bodypart_onehot', 'time',
                  'team', 'time_delta', 'location', 'polar', 'movement_polar', 'direction',
                  'goalscore']


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--games', type=int, default=10000)
    ap.add_argument('--atomic', action='store_true')
    ap.add_argument('--reps', type=int, default=10)
    ap.add_argument('--variants', default='')
    args = ap.parse_args()
    libs = {'default': N.lib()}
    for v in [x for x in args.variants.split(',') if x]:
        libs[v] = N.load_library(os.path.join(ROOT, 'socceraction_amd', '_lib',
                                              f'libsocceraction_amd_{v}.so'))
    gen = synthetic.atomic_games if args.atomic else synthetic.spadl_games
    ab = B.ActionBatch.from_columns(gen(args.games), atomic=args.atomic)
    plan = catalog.build_plan(ATOMIC_DEFAULT if args.atomic else SPADL_DEFAULT, 3, args.atomic)
    num = copy.copy(plan)
    num.struct = copy.deepcopy(plan.struct)
    for x in range(len(num.struct.bool_col)):
        num.struct.bool_col[x] = -1
    bonly = copy.copy(plan)  # the bool pass alone
    bonly.struct = copy.deepcopy(plan.struct)
    for x in range(len(bonly.struct.bool_col)):
        bonly.struct.f64_col[x] = -1
        bonly.struct.i64_col[x] = -1
    out = ops.alloc_feature_blocks(plan, ab.n, ab.device, 1024, 128)
    s = ab.struct()
    stream = torch.cuda.current_stream().cuda_stream
    bb, fb, ib = out.sa_blocks()
    res = {'n': ab.n, 'atomic': args.atomic, 'ms': {}, 'equal': {}}
    ref = None
    # the bench step's numeric pass (sa_vaep_step_f64: + xT cell codes, labels, f64 formula)
    ld = (ab.n + 15) // 16 * 16
    lab = torch.empty((3, ld), dtype=torch.uint8, device=ab.device)
    val = torch.empty((3, ld), dtype=torch.float64, device=ab.device)
    ps = torch.rand(ab.n, dtype=torch.float64, device=ab.device)
    pc = torch.rand(ab.n, dtype=torch.float64, device=ab.device)
    cells = ops.xt_cells_buffer(ab.n, ab.device)
    tags = (('num', num), ('bool', bonly), ('all', plan)) + ((('step', num), ('step_nocells', num), ('step_labels', num),
                                             ('num_cells', num)) if not args.atomic else ())
    for rnd in range(3):
        for name, lib in libs.items():
            for tag, p in tags:
                def run():
                    if tag.startswith('step'):  # step: cells + labels + formula; the parts dropped
                        nc, lo = tag == 'step_nocells', tag == 'step_labels'
                        N.check(lib.sa_vaep_step_f64(
                            ctypes.byref(s), ctypes.byref(p.struct), ctypes.byref(bb), ctypes.byref(fb),
                            ctypes.byref(ib), 0 if nc else 16, 0 if nc else 12, None if nc else cells.data_ptr(),
                            10, lab[0].data_ptr(), lab[1].data_ptr(), None, ld,
                            None if lo else ps.data_ptr(), None if lo else pc.data_ptr(),
                            None if lo else val[0].data_ptr(), None if lo else val[1].data_ptr(),
                            None if lo else val[2].data_ptr(), stream))
                        return
                    if tag == 'num_cells':
                        N.check(lib.sa_vaep_features_xt(ctypes.byref(s), ctypes.byref(p.struct), ctypes.byref(bb),
                                                        ctypes.byref(fb), ctypes.byref(ib), 16, 12,
                                                        cells.data_ptr(), stream))
                        return
                    N.check(lib.sa_vaep_features(ctypes.byref(s), ctypes.byref(p.struct), ctypes.byref(bb),
                                                 ctypes.byref(fb), ctypes.byref(ib), stream))
                run()
                torch.cuda.synchronize()
                if tag == 'step':  # the step form's outputs, compared across the builds too
                    got = [t.clone() for t in (out.f64_block, out.i64_block, lab, val, cells)]
                    sref = res.setdefault('_sref', {})
                    if 'v' not in sref:
                        sref['v'] = got
                    res['equal'][name + ':step'] = all(torch.equal(a, b) for a, b in zip(got, sref['v']))
                    del got
                if tag == 'all':
                    got = [t.clone() for t in (out.bool_block, out.f64_block, out.i64_block)]
                    if ref is None:
                        ref = got
                    res['equal'][name] = all(torch.equal(a, b) for a, b in zip(got, ref))
                    del got
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                for _ in range(args.reps):
                    run()
                b.record()
                torch.cuda.synchronize()
                res['ms'].setdefault(f'{name}:{tag}', []).append(round(a.elapsed_time(b) / args.reps, 4))
    # the bench step's two VAEP launches back to back (numeric step pass, then the bool pass),
    # each timed by its own events: what one pass costs right after the other
    if not args.atomic:
        for rnd in range(3):
            for name, lib in libs.items():
                def step():
                    N.check(lib.sa_vaep_step_f64(
                        ctypes.byref(s), ctypes.byref(num.struct), ctypes.byref(bb), ctypes.byref(fb),
                        ctypes.byref(ib), 16, 12, cells.data_ptr(), 10, lab[0].data_ptr(), lab[1].data_ptr(), None,
                        ld, ps.data_ptr(), pc.data_ptr(), val[0].data_ptr(), val[1].data_ptr(), val[2].data_ptr(),
                        stream))

                def boolp():
                    N.check(lib.sa_vaep_features(ctypes.byref(s), ctypes.byref(bonly.struct), ctypes.byref(bb),
                                                 ctypes.byref(fb), ctypes.byref(ib), stream))
                step()
                boolp()
                ev = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(args.reps)]
                for e in ev:
                    e[0].record()
                    step()
                    e[1].record()
                    boolp()
                    e[2].record()
                torch.cuda.synchronize()
                for part, (x, y) in (('pair_step', (0, 1)), ('pair_bool', (1, 2)), ('pair_total', (0, 2))):
                    res['ms'].setdefault(f'{name}:{part}', []).append(
                        round(sum(e[x].elapsed_time(e[y]) for e in ev) / args.reps, 4))
    res.pop('_sref', None)
    print(json.dumps(res), flush=True)


if __name__ == '__main__':
    main()
