"""cfg5's rate(use_interpolation=True) on one batch: the 1050 x 680 grid + gather (sa_xt_interp_grid
+ sa_xt_rate) against per-action node values (sa_xt_rate_interp).  Outputs are compared bit for
bit before timing; HIP events, rounds interleaved.

    python scripts/xt_rate_interp_time.py [--games 10000] [--reps 10]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from socceraction_amd import batch as B, ops, synthetic  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument('--games', type=int, default=10000)
    ap.add_argument('--reps', type=int, default=10)
    ap.add_argument('--variants', default='', help='library variant tags (socceraction_amd.build --variant)')
    args = ap.parse_args()
    dev = B.device()
    ab = B.ActionBatch.from_columns(synthetic.spadl_games(args.games), dev=dev)
    xT = torch.rand((68, 105), dtype=torch.float64, device=dev) * 0.3
    axes = ops.xt_interp_axes(105, 68, dev)
    out = torch.empty(ab.n + 16, dtype=torch.float64, device=dev)
    grid = ops.xt_interp_grid(xT, 105, 68)
    forms = {'grid_gather': lambda: ops.xt_rate(ab, ops.xt_interp_grid(xT, 105, 68), 1050, 680),
             'gather_only': lambda: ops.xt_rate(ab, grid, 1050, 680),
             'per_action': lambda: ops.xt_rate_interp(ab, xT, 105, 68, axes=axes, out=out)}
    import ctypes
    from socceraction_amd import _native as N
    s_act = ab.struct()
    err = torch.zeros(1, dtype=torch.int32, device=dev)
    for v in [x for x in args.variants.split(',') if x]:  # the same call through a variant build
        lib = N.load_library(os.path.join(ROOT, 'socceraction_amd', '_lib', f'libsocceraction_amd_{v}.so'))

        def run(lib=lib):
            o = 105 + 68
            N.check(lib.sa_xt_rate_interp(ctypes.byref(s_act), xT.data_ptr(), axes[:105].data_ptr(),
                                          axes[105:o].data_ptr(), 105, 68, axes[o:o + 1050].data_ptr(), 1050,
                                          axes[o + 1050:].data_ptr(), 680, out.data_ptr(), err.data_ptr(),
                                          torch.cuda.current_stream().cuda_stream))
        forms['per_action_' + v] = run
    a, _ = forms['grid_gather']()
    b, _ = forms['per_action']()
    x, y = a.cpu().numpy(), b.cpu().numpy()
    equal = bool((np.isnan(x) == np.isnan(y)).all() and (x[~np.isnan(x)] == y[~np.isnan(x)]).all())
    for k in [k for k in forms if k.startswith('per_action_')]:
        forms[k]()
        y = out[:ab.n].cpu().numpy()
        equal &= bool((np.isnan(x) == np.isnan(y)).all() and (x[~np.isnan(x)] == y[~np.isnan(x)]).all())
    ms = {k: [] for k in forms}
    for _ in range(4):
        for k, fn in forms.items():
            fn()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.reps):
                fn()
            e1.record()
            torch.cuda.synchronize()
            ms[k].append(round(e0.elapsed_time(e1) / args.reps, 4))
    print(json.dumps({'actions': ab.n, 'equal': equal, 'ms': ms,
                      'GBs_42B': {k: round(42 * ab.n / min(v) * 1e-6, 1) for k, v in ms.items()}}))
    if not equal:
        raise SystemExit(3)


if __name__ == '__main__':
    main()
