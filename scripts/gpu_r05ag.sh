set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for e in 10 4 10 4; do
  timeout -k 10 300 python -u bench.py --no-side --no-cpu --event-every $e > gpurun_out/r05ag_e$e.json 2> gpurun_out/r05ag_e$e.err || exit $?
  python -c "import json; d=json.load(open('gpurun_out/r05ag_e$e.json')); print($e, d['ms_per_step'], d['roofline']['step_frac'], d['kernels']['num_step']['ms'], d['kernels']['bool_features']['ms'])"
done
