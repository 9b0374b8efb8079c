"""A/B of the interpolated rate from count-pass operands (sa_xt_rate_interp_codes_many) across
library builds on the SAME operands: the default library and variant builds
(``python -m socceraction_amd.build -DNAME=V --variant=tag``), HIP events, round-robin; the
outputs must be bit-identical.

    python scripts/rate_lib_ab.py --variants xripack
"""
import argparse
import ctypes
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from socceraction_amd import _native as N  # noqa: E402
from socceraction_amd import batch as B, ops, synthetic  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--batches', type=int, default=7)
    ap.add_argument('--reps', type=int, default=10)
    ap.add_argument('--variants', default='')
    args = ap.parse_args()
    libs = {'default': N.lib()}
    for v in [x for x in args.variants.split(',') if x]:
        libs[v] = N.load_library(os.path.join(ROOT, 'socceraction_amd', '_lib',
                                              f'libsocceraction_amd_{v}.so'))
    l, w, L, W = 105, 68, 1050, 680
    bs = [B.ActionBatch.from_columns(synthetic.spadl_games(10000, game_id0=k * 10000))
          for k in range(args.batches)]
    dev = bs[0].device
    ic = [ops.xt_interp_codes_buffer(b.n, dev) for b in bs]
    acc = ops.xt_count_many(bs, l, w, interp_codes=ic)
    xT = ops.xt_solve(acc, transition=False).mats[3].reshape(w, l).contiguous()
    axes = ops.xt_interp_axes(l, w, dev, L, W)
    outs = [torch.empty(max(b.n, 16), dtype=torch.float64, device=dev) for b in bs]
    err = torch.zeros(1, dtype=torch.int32, device=dev)
    k = len(bs)
    cp = (ctypes.c_void_p * k)(*[c.data_ptr() for c in ic])
    op = (ctypes.c_void_p * k)(*[o.data_ptr() for o in outs])
    nn = (ctypes.c_int64 * k)(*[b.n for b in bs])
    o = l + w
    stream = torch.cuda.current_stream().cuda_stream
    n_total = sum(b.n for b in bs)
    res = {'n': n_total, 'batches': k, 'ms': {}, 'equal': {}}
    ref = None
    for rnd in range(3):
        for name, lib in libs.items():
            def run():
                N.check(lib.sa_xt_rate_interp_codes_many(
                    k, cp, nn, xT.data_ptr(), axes[:l].data_ptr(), axes[l:o].data_ptr(), l, w,
                    axes[o:o + L].data_ptr(), L, axes[o + L:].data_ptr(), W, op, err.data_ptr(), stream))
            run()
            torch.cuda.synchronize()
            got = torch.cat([t[:b.n] for t, b in zip(outs, bs)])
            if ref is None:
                ref = got.clone()
            res['equal'][name] = bool(torch.equal(torch.isnan(got), torch.isnan(ref)) and
                                      torch.equal(torch.nan_to_num(got), torch.nan_to_num(ref)))
            del got
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(args.reps):
                run()
            b.record()
            torch.cuda.synchronize()
            ms = a.elapsed_time(b) / args.reps
            res['ms'].setdefault(name, []).append(round(ms, 4))
            res.setdefault('GBs', {})[name] = round(16 * n_total / ms * 1e-6, 1)
    print(json.dumps(res), flush=True)


if __name__ == '__main__':
    main()
