set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for c in require all require all; do
  timeout -k 10 300 python -u scripts/cfg3_time.py --times 3 --contiguous $c > gpurun_out/r05av_$c.json 2> gpurun_out/r05av_$c.err || exit $?
  cat gpurun_out/r05av_$c.json
done
python - <<'PY'
import pandas as pd
t = pd.read_csv('gpurun_out/r05au_prof/run_kernel_trace.csv') if False else None
PY
