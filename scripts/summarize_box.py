"""One row per kernel of scripts/step_pair.py's launches from the counter passes of
scripts/profile_box.sh on one box: median duration (kernel trace), effective shader clock
(GRBM_GUI_ACTIVE cycles / duration), wave-cycle occupancy, VALU activity and HBM bytes.

    python scripts/summarize_box.py <tag> <out.csv> [--atomic]

Columns:
  dur_us_median      median kernel duration of the trace pass (HIP kernel trace)
  eff_clock_mhz      GRBM_GUI_ACTIVE / 8 / duration: the effective (DVFS) clock while the kernel
                     ran (rocprofv3 sums GRBM_GUI_ACTIVE over the 8 XCDs; MI355X_MICROARCH.md)
  sq_busy_ratio      SQ_BUSY_CYCLES / GRBM_GUI_ACTIVE, raw (summed over different block counts)
  valu_active_frac   SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES (both in quad-cycles): share of a
                     wave's resident cycles it was issuing VALU work
  wait_frac          SQ_WAIT_ANY / SQ_WAVE_CYCLES (waves waiting on memory or dependencies)
  insts_valu_per_wave, waves
  hbm_mb             (2 * FETCH_SIZE + WRITE_SIZE) KiB -> MB (FETCH_SIZE's gfx950 x2 correction,
                     MI355X_MICROARCH.md HBM section)
  hbm_gbs            hbm_mb / duration
"""
import os
import sys

import pandas as pd

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _counters(d):
    p = os.path.join(ROOT, 'gpurun_out', d, 'run_counter_collection.csv')
    if not os.path.exists(p):
        return {}
    t = pd.read_csv(p)
    return {(k, c): v for (k, c), v in t.groupby(['Kernel_Name', 'Counter_Name']).Counter_Value.median().items()}


def main(tag, out, atomic=False):
    a = 'a' if atomic else ''
    tr = pd.read_csv(os.path.join(ROOT, 'gpurun_out', f'{tag}_prof_{a}trace', 'run_kernel_trace.csv'))
    tr['dur_us'] = (tr.End_Timestamp - tr.Start_Timestamp) / 1e3
    dur = tr.groupby('Kernel_Name').dur_us.median()
    c = {}
    for kind in ('clk', 'inst', 'fetch', 'write'):
        c.update(_counters(f'{tag}_prof_{a}{kind}'))
    rows = []
    for k, d in dur.items():
        g = lambda n: c.get((k, n), float('nan'))  # noqa: E731
        gui, wc = g('GRBM_GUI_ACTIVE'), g('SQ_WAVE_CYCLES')
        hbm = (2 * g('FETCH_SIZE') + g('WRITE_SIZE')) * 1024 / 1e6
        rows.append(dict(kernel=k.split('(')[0], dur_us_median=round(d, 1),
                         eff_clock_mhz=round(gui / 8 / d, 0),
                         sq_busy_ratio=round(g('SQ_BUSY_CYCLES') / gui, 3),
                         valu_active_frac=round(g('SQ_ACTIVE_INST_VALU') / wc, 3),
                         wait_frac=round(g('SQ_WAIT_ANY') / wc, 3),
                         insts_valu_per_wave=round(g('SQ_INSTS_VALU') / g('SQ_WAVES'), 0),
                         waves=g('SQ_WAVES'), hbm_mb=round(hbm, 1), hbm_gbs=round(hbm / d * 1e3, 0)))
    df = pd.DataFrame(rows).sort_values('dur_us_median', ascending=False)
    df.insert(0, 'tag', tag)
    df.to_csv(out, index=False)
    print(df.to_string(index=False))


if __name__ == '__main__':
    main(sys.argv[1], sys.argv[2], '--atomic' in sys.argv[3:])
