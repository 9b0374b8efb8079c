"""Per-kernel average durations (us) of several rocprofv3 `--stats` CSVs side by side.

    python scripts/stats_table.py DIR1/run_kernel_stats.csv DIR2/run_kernel_stats.csv ...
"""
import csv
import os
import re
import sys


def short(name: str) -> str:
    name = re.sub(r'^void ', '', name)
    name = re.sub(r'\(.*$', '', name)
    return name.replace('sa::', '')[:70]


def main():
    cols, rows = [], {}
    for path in sys.argv[1:]:
        tag = os.path.basename(os.path.dirname(path))
        cols.append(tag)
        with open(path) as fh:
            for rec in csv.DictReader(fh):
                k = short(rec['Name'])
                rows.setdefault(k, {})[tag] = (float(rec['AverageNs']) / 1e3, int(rec['Calls']))
    print('kernel'.ljust(72) + ''.join(c[-14:].rjust(16) for c in cols))
    for k, v in sorted(rows.items(), key=lambda kv: -max(a for a, _ in kv[1].values())):
        print(k.ljust(72) + ''.join((f'{v[c][0]:9.1f} x{v[c][1]:<5d}' if c in v else ' ' * 16) for c in cols))


if __name__ == '__main__':
    main()
