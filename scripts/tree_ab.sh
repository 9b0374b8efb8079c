#!/usr/bin/env bash
# A/B of tree-kernel builds: kernel-trace average of tree_predict_kernel per variant.
set -u
export TMPDIR=/tmp
for v in "$@"; do
  if [ "$v" = default ]; then lib=""; else lib="SOCCERACTION_AMD_LIB=socceraction_amd/_lib/libsocceraction_amd_$v.so"; fi
  env $lib timeout -s KILL 100 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/tab_$v -o run -- python3 scripts/tree_prof_probe.py > gpurun_out/tab_$v.log 2>&1 || exit 1
  python3 -c "import pandas as pd; k=pd.read_csv('gpurun_out/tab_$v/run_kernel_stats.csv'); k=k[k.Name.str.contains('tree')]; print('$v', float(k.AverageNs.iloc[0])/1e6, 'ms')"
done
