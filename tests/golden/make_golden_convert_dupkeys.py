"""Golden vectors for SPADL -> Atomic-SPADL conversion of frames whose (game_id, period_id,
action_id) keys repeat, produced by running the *reference* (build container only):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_convert_dupkeys.py

Same shims and storage as ``make_golden_convert.py``.  With repeated keys the reference's
stable sort after its concat (atomic/spadl/base.py:109-110) puts the rows _extra_from_passes
inserts after ALL the rows sharing their parent's key, not directly after the parent; the
drop-in takes its general path there (first pass on its own, placed by the stable lexsort).
Cases: every second action sharing its predecessor's id; runs of up to four equal ids; one id
for a whole game; duplicates with rows swapped inside a game.
"""
from __future__ import annotations

import numpy as np

from make_golden_convert import case, synthetic_frame


def main() -> None:
    rng = np.random.default_rng(4242)
    df = synthetic_frame(3, 71, rng)
    df['action_id'] = (df.groupby('game_id').cumcount() // 2).astype(np.int64)
    case('dupkeys_pairs', df)
    df = synthetic_frame(2, 72, rng)
    runs = rng.integers(1, 5, size=len(df))
    df['action_id'] = (np.cumsum(runs) // 4).astype(np.int64)
    case('dupkeys_runs', df)
    df = synthetic_frame(2, 73, rng)
    df['action_id'] = np.zeros(len(df), np.int64)
    case('dupkeys_constant', df)
    df = synthetic_frame(2, 74, rng)
    df['action_id'] = (df.groupby('game_id').cumcount() // 3).astype(np.int64)
    idx = np.arange(len(df))
    for j in rng.choice(len(df) - 1, 12, replace=False):
        idx[j], idx[j + 1] = idx[j + 1], idx[j]
    case('dupkeys_swapped', df.iloc[idx])


if __name__ == '__main__':
    main()
