"""Per-kernel medians of rocprofv3 counter passes (scripts/pmc_passes.sh) with derived ratios.

    python scripts/pmc_table.py DIR1/run_counter_collection.csv DIR2/... [--match REGEX]

Derived (MI355X_MICROARCH.md "rocprofv3 PMC slots"): SQ_WAVE_CYCLES / SQ_ACTIVE_INST_* /
SQ_WAIT_* count quad-cycles, so they compare with each other directly:
  valu    SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES   share of a wave's resident time issuing VALU
  any     SQ_ACTIVE_INST_ANY / SQ_WAVE_CYCLES    issuing anything
  wait    SQ_WAIT_ANY / SQ_WAVE_CYCLES           parked on s_waitcnt / barrier
  stall   SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES      issue stalls (pipe busy, dependencies)
  lds     SQ_ACTIVE_INST_LDS / SQ_WAVE_CYCLES
  clk     GRBM_GUI_ACTIVE / 8 / duration (MHz; the effective DVFS clock)
  hbm     (2 FETCH_SIZE + WRITE_SIZE) KiB per dispatch (FETCH_SIZE x2: the gfx950 correction)
"""
import re
import sys

import pandas as pd


def main():
    args = [a for a in sys.argv[1:] if not a.startswith('--match')]
    m = [a.split('=', 1)[1] for a in sys.argv[1:] if a.startswith('--match=')]
    frames = []
    for p in args:
        try:
            frames.append(pd.read_csv(p))
        except (OSError, ValueError):
            pass
    t = pd.concat(frames)
    t['Kernel'] = t.Kernel_Name.str.replace(r'\(.*$', '', regex=True).str.replace('void ', '').str.replace('sa::', '')
    if m:
        t = t[t.Kernel.str.contains(m[0])]
    t['dur_ns'] = t.End_Timestamp - t.Start_Timestamp
    med = t.groupby(['Kernel', 'Counter_Name']).Counter_Value.median().unstack()
    dur = t.groupby('Kernel').dur_ns.median()
    calls = t.groupby(['Kernel', 'Counter_Name']).size().unstack().max(axis=1)
    g = lambda k, c: med.loc[k, c] if c in med.columns else float('nan')  # noqa: E731
    rows = []
    for k in med.index:
        wc = g(k, 'SQ_WAVE_CYCLES')
        r = dict(kernel=k[:60], calls=int(calls[k]), dur_us=round(dur[k] / 1e3, 1))
        for name, c in (('valu', 'SQ_ACTIVE_INST_VALU'), ('any', 'SQ_ACTIVE_INST_ANY'),
                        ('wait', 'SQ_WAIT_ANY'), ('stall', 'SQ_WAIT_INST_ANY'),
                        ('lds', 'SQ_ACTIVE_INST_LDS')):
            r[name] = round(g(k, c) / wc, 3) if wc == wc and wc else float('nan')
        r['clk'] = round(g(k, 'GRBM_GUI_ACTIVE') / 8 / dur[k] * 1e3, 0)
        r['waves'] = g(k, 'SQ_WAVES')
        r['valu_insts/wave'] = round(g(k, 'SQ_INSTS_VALU') / g(k, 'SQ_WAVES'), 0) if 'SQ_WAVES' in med.columns else float('nan')
        r['hbm_MB'] = round((2 * g(k, 'FETCH_SIZE') + g(k, 'WRITE_SIZE')) * 1024 / 1e6, 1)
        r['GB/s'] = round(r['hbm_MB'] * 1e6 / dur[k], 0)
        rows.append(r)
    out = pd.DataFrame(rows).sort_values('dur_us', ascending=False)
    pd.set_option('display.width', 250)
    pd.set_option('display.max_columns', 30)
    print(out.to_string(index=False))


if __name__ == '__main__':
    main()
