"""Drop-in API timings (pandas in -> pandas out), the way a notebook calls the reference:
per-game ``VAEP.compute_features`` / ``compute_labels`` / ``formula.value`` loops and the batched
``*_batch`` calls, with a breakdown of where the time goes (H2D, kernels, D2H, DataFrame
assembly). Prints one JSON line.

    python scripts/bench_dropin.py [--games 64]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import pandas as pd
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from socceraction_amd import synthetic  # noqa: E402
import socceraction_amd.vaep as vaep  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--games', type=int, default=64)
    args = ap.parse_args()
    d = synthetic.spadl_games(args.games)
    actions = synthetic.to_frame(d)
    games = synthetic.games_frame(d)
    n = len(actions)
    p = synthetic.probabilities(n)
    model = vaep.VAEP()
    per_game = [(g, actions[actions.game_id == g.game_id].reset_index(drop=True))
                for g in games.itertuples()]
    # warm-up
    model.compute_features(per_game[0][0], per_game[0][1])
    model.compute_labels(per_game[0][0], per_game[0][1])
    torch.cuda.synchronize()

    t = time.perf_counter()
    for g, a in per_game:
        model.compute_features(g, a)
    tf = time.perf_counter() - t
    t = time.perf_counter()
    for g, a in per_game:
        model.compute_labels(g, a)
    tl = time.perf_counter() - t
    off = 0
    t = time.perf_counter()
    for g, a in per_game:
        m = len(a)
        vaep.formula.value(a, pd.Series(p['scores'][off:off + m]), pd.Series(p['concedes'][off:off + m]))
        off += m
    tv = time.perf_counter() - t
    t = time.perf_counter()
    X = model.compute_features_batch(games, actions)
    tb = time.perf_counter() - t
    t = time.perf_counter()
    model.compute_labels_batch(games, actions)
    tlb = time.perf_counter() - t
    print(json.dumps({
        'workload': f'drop-in pandas API, {args.games} synthetic games ({n} actions)',
        'per_game_loop_actions_per_s': {'compute_features': round(n / tf, 1),
                                        'compute_labels': round(n / tl, 1),
                                        'formula_value': round(n / tv, 1),
                                        'all_three': round(n / (tf + tl + tv), 1)},
        'per_game_ms': {'compute_features': round(tf / args.games * 1e3, 3),
                        'compute_labels': round(tl / args.games * 1e3, 3),
                        'formula_value': round(tv / args.games * 1e3, 3)},
        'batched_actions_per_s': {'compute_features_batch': round(n / tb, 1),
                                  'compute_labels_batch': round(n / tlb, 1)},
        'feature_columns': X.shape[1],
        'reference_cpu_actions_per_s_1proc': 7856.0}), flush=True)


if __name__ == '__main__':
    main()
