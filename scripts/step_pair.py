"""The bench step's two VAEP launches back to back -- the numeric step pass (sa_vaep_step_f64:
f64 / i64 blocks, goalscore, xT cell codes, labels, f64 formula) then the bool pass -- on cfg2's
10k synthetic games, ``--reps`` times after a warm-up, for rocprofv3 counter passes (one kernel
name per pass kind, every launch the step's size).  ``--atomic``: cfg3's atomic numeric pass,
bool pass and labels launch instead (10k atomic games).

    rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES -- python3 scripts/step_pair.py
"""
import argparse
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
ATOMIC_DEFAULT = ['actiontype', 'actiontype_onehot', 'bodypart', 'bodypart_onehot', 'time',
                  'team', 'time_delta', 'location', 'polar', 'movement_polar', 'direction',
                  'goalscore']


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--games', type=int, default=10000)
    ap.add_argument('--reps', type=int, default=5)
    ap.add_argument('--atomic', action='store_true')
    args = ap.parse_args()
    gen = synthetic.atomic_games if args.atomic else synthetic.spadl_games
    ab = B.ActionBatch.from_columns(gen(args.games), atomic=args.atomic)
    plan = catalog.build_plan(ATOMIC_DEFAULT if args.atomic else SPADL_DEFAULT, 3, args.atomic)
    out = ops.alloc_feature_blocks(plan, ab.n, ab.device, 1024, 128, contiguous=True)
    s = ab.struct()
    lab = ops.labels(ab)
    if args.atomic:
        def step():
            ops.step_into(s, out, None, None, 10, lab, None)
    else:
        num = copy.copy(plan)
        num.struct = copy.deepcopy(plan.struct)
        bonly = copy.copy(plan)
        bonly.struct = copy.deepcopy(plan.struct)
        for x in range(len(plan.struct.bool_col)):
            num.struct.bool_col[x] = -1
            bonly.struct.f64_col[x] = -1
            bonly.struct.i64_col[x] = -1
        ld = (ab.n + 15) // 16 * 16
        val = torch.empty((3, ld), dtype=torch.float64, device=ab.device)
        p = synthetic.probabilities(ab.n)
        ps = torch.from_numpy(p['scores']).to(ab.device)
        pc = torch.from_numpy(p['concedes']).to(ab.device)
        cells = ops.xt_cells_buffer(ab.n, ab.device)
        numo = copy.copy(out)
        numo.plan = num
        boolo = copy.copy(out)
        boolo.plan = bonly

        def step():
            ops.step_into(s, numo, ps, pc, 10, lab, val, xt_cells=(16, 12, cells))
            ops.features_into(s, boolo)
    for _ in range(2):
        step()
    torch.cuda.synchronize()
    for _ in range(args.reps):
        step()
    torch.cuda.synchronize()
    print('done', ab.n, flush=True)


if __name__ == '__main__':
    main()
