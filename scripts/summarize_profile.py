"""Copy rocprofv3 results of one profiling round into profiles/ and derive HBM traffic.

    python scripts/summarize_profile.py r01 [N_ACTIONS]

Reads gpurun_out/prof_<tag>_{trace,fetch,write}/ (see scripts/profile_round.sh) and writes
  profiles/<tag>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary of the step alone
  profiles/<tag>_side_kernel_stats.csv   the same with bench.py's side entries
  profiles/<tag>_pmc.csv            per-kernel mean FETCH_SIZE / WRITE_SIZE (KiB) + HBM bytes
  profiles/pmc_dominant_kernel.json HBM bytes per action of the dominant kernel (read by bench.py,
                                    which quotes them only while the loaded library's build id
                                    equals the profiled one, gpurun_out/prof_<tag>_build_id.txt)
HBM bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024: on gfx950 FETCH_SIZE reports half the
bytes of wide streaming reads (MI355X_MICROARCH.md, HBM section); WRITE_SIZE is exact for
16-byte-per-lane streaming stores.
"""
import json
import os
import shutil
import sys

import pandas as pd

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main(tag: str, n_actions: int, dominant=None) -> None:
    out = os.path.join(ROOT, 'profiles')
    src = os.path.join(ROOT, 'gpurun_out')
    shutil.copy(os.path.join(src, f'prof_{tag}_trace', 'run_kernel_stats.csv'),
                os.path.join(out, f'{tag}_kernel_stats.csv'))
    side = os.path.join(src, f'prof_{tag}_side', 'run_kernel_stats.csv')
    if os.path.exists(side):
        shutil.copy(side, os.path.join(out, f'{tag}_side_kernel_stats.csv'))
    rows = {}
    for kind in ('fetch', 'write'):
        p = os.path.join(src, f'prof_{tag}_{kind}', 'run_counter_collection.csv')
        t = pd.read_csv(p)
        for (k, c), v in t.groupby(['Kernel_Name', 'Counter_Name']).Counter_Value.mean().items():
            rows.setdefault(k, {})[c] = v
    df = pd.DataFrame.from_dict(rows, orient='index')
    df['hbm_bytes'] = (2 * df['FETCH_SIZE'] + df['WRITE_SIZE']) * 1024
    df['hbm_bytes_per_action'] = df['hbm_bytes'] / n_actions
    df.index.name = 'kernel'
    df.to_csv(os.path.join(out, f'{tag}_pmc.csv'))
    if dominant is None:  # the step kernel with the longest total duration in the trace
        st = pd.read_csv(os.path.join(out, f'{tag}_kernel_stats.csv'))
        st = st[st.Name.str.contains('bool_colgroup_kernel|num_features_kernel')]
        dominant = st.sort_values('TotalDurationNs').Name.iloc[-1]
    feat = [k for k in df.index if dominant in k][0]
    bid = os.path.join(src, f'prof_{tag}_build_id.txt')
    build_id = open(bid).read().strip() if os.path.exists(bid) else None
    rec = {'tag': tag, 'build_id': build_id, 'kernel': feat, 'n_actions': n_actions,
           'fetch_kib': float(df.loc[feat, 'FETCH_SIZE']),
           'write_kib': float(df.loc[feat, 'WRITE_SIZE']),
           'hbm_bytes_per_launch_per_action': float(df.loc[feat, 'hbm_bytes_per_action']),
           # every step kernel's PMC bytes, so bench.py can quote whichever its HIP events
           # find dominant
           'per_kernel': {k: float(df.loc[k, 'hbm_bytes_per_action']) for k in df.index
                          if 'bool_colgroup_kernel' in k or 'num_features_kernel' in k}}
    with open(os.path.join(out, 'pmc_dominant_kernel.json'), 'w') as f:
        json.dump(rec, f, indent=1)
    print(df.to_string())


if __name__ == '__main__':
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 15992198,
         sys.argv[3] if len(sys.argv) > 3 else None)
