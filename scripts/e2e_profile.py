"""Where the pandas-in / pandas-out drop-in path spends its time (bench.py's end_to_end entry,
1000 games): cProfile of compute_features_batch + compute_labels_batch, top functions."""
import cProfile
import io
import os
import pstats
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from socceraction_amd import synthetic, vaep  # noqa: E402


def main():
    d = synthetic.spadl_games(1000)
    actions = synthetic.to_frame(d)
    games = synthetic.games_frame(d)
    model = vaep.VAEP()
    for _ in range(2):
        model.compute_features_batch(games, actions)
        model.compute_labels_batch(games, actions)
    t = time.perf_counter()
    X = model.compute_features_batch(games, actions)
    t1 = time.perf_counter()
    Y = model.compute_labels_batch(games, actions)
    t2 = time.perf_counter()
    print(f'features {t1 - t:.4f} s labels {t2 - t1:.4f} s rows {len(X)}', flush=True)
    pr = cProfile.Profile()
    pr.enable()
    X = model.compute_features_batch(games, actions)
    pr.disable()
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats('cumulative').print_stats(35)
    print(s.getvalue())


if __name__ == '__main__':
    main()
