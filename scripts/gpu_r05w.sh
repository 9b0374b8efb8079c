set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for s in 20 60 20 60; do
  timeout -k 10 300 python -u bench.py --steps $s --no-side --no-cpu > gpurun_out/r05w_s$s.json 2> gpurun_out/r05w_s$s.err || exit $?
  python -c "import json; d=json.load(open('gpurun_out/r05w_s$s.json')); print($s, d['ms_per_step'], d['roofline']['step_frac'], d['kernels']['num_step']['ms'], d['kernels']['bool_features']['ms'])"
done
