"""Per run of scripts/cfg3_counters.sh's passes: each step kernel's median duration and counters
in run 1 vs runs 2-3 of the same process (a process's dispatches of one kernel split into its
three runs in order).  Prints one table per pass.

    python scripts/cfg3_counters_summary.py TAG
"""
import glob
import os
import sys

import numpy as np
import pandas as pd

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def short(k):
    return k.replace('void ', '').replace('sa::', '').split('(')[0][:58]


def main(tag):
    for path in sorted(glob.glob(os.path.join(ROOT, 'gpurun_out', f'{tag}_*', 'run_*.csv'))):
        if not (path.endswith('kernel_trace.csv') or path.endswith('counter_collection.csv')):
            continue
        t = pd.read_csv(path)
        t = t[t.Kernel_Name.str.contains('atomic|colgroup|num_features|labels', regex=True)]
        if t.empty:
            continue
        t['K'] = t.Kernel_Name.map(short)
        t['dur_us'] = (t.End_Timestamp - t.Start_Timestamp) / 1e3
        print(f'== {os.path.relpath(path, ROOT)}')
        rows = []
        for k, g in t.groupby('K'):
            if 'Counter_Name' in g:
                for c, gc in g.groupby('Counter_Name'):
                    gc = gc.sort_values('Dispatch_Id')
                    parts = np.array_split(gc, 3)
                    rows.append(dict(kernel=k, what=c, **{f'run{i + 1}': float(p.Counter_Value.median())
                                                         for i, p in enumerate(parts)},
                                     **{f'us{i + 1}': float(p.dur_us.median()) for i, p in enumerate(parts)}))
            else:
                g = g.sort_values('Correlation_Id' if 'Correlation_Id' in g else 'Start_Timestamp')
                parts = np.array_split(g, 3)
                rows.append(dict(kernel=k, what='duration_us',
                                 **{f'run{i + 1}': float(p.dur_us.median()) for i, p in enumerate(parts)}))
        pd.set_option('display.width', 250)
        print(pd.DataFrame(rows).to_string(index=False, float_format=lambda v: f'{v:.4g}'))


if __name__ == '__main__':
    main(sys.argv[1])
