"""VAEP.rate's two xgboost-shaped learners (100 trees, depth 3) on cfg2 through condition bitmaps
(trees.predict_pair_conditions) vs the float32-block path, HIP events; for rocprofv3 traces.
Both paths' probabilities are compared (torch.equal) before any timing; exit 3 on a mismatch.

    python scripts/cond_probe.py
"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from socceraction_amd import batch as B, catalog, ops, synthetic, trees  # noqa: E402

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
    ab = B.ActionBatch.from_columns(synthetic.spadl_games(int(sys.argv[1]) if len(sys.argv) > 1 else 10000))
    plan = catalog.build_plan(SPADL_DEFAULT, 3)
    kinds = [k for _, k, _ in plan.order]
    models = [trees.TreeEnsemble.from_xgboost_json(trees.synthetic_xgboost_json(
        len(kinds), n_trees=100, depth=3, seed=s, feature_kinds=kinds)) for s in (1, 2)]
    f32 = ops.features(ab, SPADL_DEFAULT, 3, num_tile=128, bool_bits=True, num32=True)

    def blocks():
        ops.features(ab, SPADL_DEFAULT, 3, out=f32)
        return [m.predict_blocks(f32) for m in models]
    # parity before timing: both paths give the same probabilities bit for bit
    cond = trees.predict_pair_conditions(ab, plan, models)
    ref = blocks()
    equal = all(torch.equal(a, b) for a, b in zip(cond, ref))
    prep, bits, words = trees.condition_bitmaps(ab, plan, models)
    out = torch.empty(ab.n, dtype=torch.float32, device=ab.device)
    res = {'n': ab.n, 'equal': equal,
           'conditions_ms': _ms(lambda: trees.predict_pair_conditions(ab, plan, models)),
           'conditions_features_ms': _ms(lambda: trees.condition_bitmaps(ab, plan, models, bits=bits)),
           'conditions_walk_ms': [_ms(lambda k=k: trees.walk_conditions(prep, k, models[k], bits, words, ab.n,
                                                                        ab.device, out=out)) for k in range(2)],
           'conditions': {'union': prep['n_cond_union'], 'per_model': [w[5] for w in prep['walks']],
                          'nodes': [w[0].numel() for w in prep['walks']]},
           'f32_blocks_ms': _ms(blocks)}
    print(json.dumps(res), flush=True)
    if not equal:
        raise SystemExit(3)


if __name__ == '__main__':
    main()
