"""Time the tree walks on cfg2's feature blocks: gather walk (sa_tree_predict) vs staged walk
(sa_tree_predict_staged), HIP events; optional variant libraries for probes.

    python scripts/tree_probe.py [--games 10000] [--libs default,ts_nowalk,ts_nostage]
"""
import argparse
import ctypes
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from socceraction_amd import _native, batch as B, catalog, ops, synthetic, trees  # noqa: E402

SPADL_DEFAULT = ['actiontype_onehot', 'result_onehot', 'actiontype_result_onehot',
                 'bodypart_onehot', 'time', 'startlocation', 'endlocation', 'startpolar',
                 'endpolar', 'movement', 'team', 'time_delta', 'space_delta', 'goalscore']


def _ms(fn, reps=5):
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
    ap.add_argument('--libs', default='default')
    args = ap.parse_args()
    ab = B.ActionBatch.from_columns(synthetic.spadl_games(args.games))
    fb = ops.features(ab, SPADL_DEFAULT, 3, bool_tile=1024, num_tile=128)
    fbits = ops.features(ab, SPADL_DEFAULT, 3, num_tile=128, bool_bits=True)
    out_feat = {'features_block_ms': _ms(lambda: ops.features(ab, SPADL_DEFAULT, 3, out=fb)),
                'features_bitmaps_ms': _ms(lambda: ops.features(ab, SPADL_DEFAULT, 3, out=fbits))}
    kinds = [k for _, k, _ in fb.plan.order]
    te = trees.TreeEnsemble.from_xgboost_json(trees.synthetic_xgboost_json(
        len(kinds), n_trees=100, depth=3, seed=1, feature_kinds=kinds))
    out = {'n': ab.n, **out_feat}
    lay = te.staged_layout(te.feature_slots(fb.plan))
    out['model'] = {'nodes': len(lay['models'][0]['nodes']), 'bool_conditions': len(lay['bool_cols']),
                    'numeric_conditions': len(lay['num_slots']),
                    'numeric_columns': len(set(lay['num_slots'].tolist()))}
    for name in args.libs.split(','):
        if name != 'default':  # every later call goes to the variant library
            _native._lib = _native.load_library(os.path.join(
                ROOT, 'socceraction_amd', '_lib', f'libsocceraction_amd_{name}.so'))
        te._dev = None
        res = {'staged': _ms(lambda: te.predict_blocks(fb, method='staged')),
               'staged_from_bitmaps': _ms(lambda: te.predict_blocks(fbits, method='staged'))}
        if name == 'default':
            res['gather'] = _ms(lambda: te.predict_blocks(fb, method='gather'))
        out[name] = res
        print(json.dumps(out), flush=True)


if __name__ == '__main__':
    main()
