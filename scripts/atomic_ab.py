"""In-process A/B of cfg3's Atomic-VAEP step forms on the same allocations (bench.py atomic_cfg3):

  fused     sa_vaep_step_f64 labels-only (labels computed in the numeric pass)
  separate  sa_vaep_features + sa_vaep_labels (two launches plus the bool pass)
  features  sa_vaep_features alone (no labels)

Every form's outputs are compared (torch.equal) before any timing.  Rounds are interleaved so
box drift hits every form alike; per-kernel times come from rocprofv3 when run under it.

    python scripts/atomic_ab.py [--games 10000] [--reps 10] [--rounds 4]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from socceraction_amd import batch as B, ops, synthetic  # noqa: E402

ATOMIC_DEFAULT = ['actiontype', 'actiontype_onehot', 'bodypart', 'bodypart_onehot', 'time',
                  'team', 'time_delta', 'location', 'polar', 'movement_polar', 'direction',
                  'goalscore']


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument('--games', type=int, default=10000)
    ap.add_argument('--reps', type=int, default=10)
    ap.add_argument('--rounds', type=int, default=4)
    args = ap.parse_args()
    dev = B.device()
    d = synthetic.atomic_games(args.games)
    ab = B.ActionBatch.from_columns(d, atomic=True, dev=dev)
    out = ops.features(ab, ATOMIC_DEFAULT, 3, bool_tile=1024, num_tile=128)
    lab = ops.labels(ab)
    s = ab.struct()
    forms = {
        'fused': lambda: ops.step_into(s, out, None, None, 10, lab, None),
        'separate': lambda: (ops.features_into(s, out), ops.labels(ab, 10, lab)),
        'features': lambda: ops.features_into(s, out),
    }
    # parity first: every labelled form leaves the same blocks and labels
    snap = {}
    for k in ('fused', 'separate'):
        for t in (out.bool_block, out.f64_block, out.i64_block, lab.scores, lab.concedes):
            t.fill_(0x5A if t.dtype == torch.uint8 else 7)
        forms[k]()
        torch.cuda.synchronize()
        snap[k] = [t.clone() for t in (out.bool_block, out.f64_block, out.i64_block,
                                       lab.scores[:ab.n], lab.concedes[:ab.n])]
    same = all(torch.equal(a, b) for a, b in zip(snap['fused'], snap['separate']))
    del snap
    times = {k: [] for k in forms}
    for fn in forms.values():
        fn()
    torch.cuda.synchronize()
    for _ in range(args.rounds):
        for k, fn in forms.items():
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(args.reps):
                fn()
            b.record()
            torch.cuda.synchronize()
            times[k].append(round(a.elapsed_time(b) / args.reps, 4))
    bpa = 47 + out.plan.n_bool + 8 * (out.plan.n_f64 + out.plan.n_i64) + 2
    print(json.dumps({'atomic_actions': ab.n, 'outputs_equal': same, 'ms': times,
                      'frac_of_8TBs': {k: round(bpa * ab.n / min(v) * 1e-6 / 8000, 4)
                                       for k, v in times.items() if k != 'features'}}), flush=True)
    if not same:
        raise SystemExit(3)


if __name__ == '__main__':
    main()
