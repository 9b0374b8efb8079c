set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for a in contig contig-all contig contig-all; do
  timeout -k 10 300 python -u bench.py --no-side --no-cpu --alloc-order $a > gpurun_out/r05am_$a.json 2> gpurun_out/r05am_$a.err || exit $?
  python -c "import json; d=json.load(open('gpurun_out/r05am_$a.json')); print('$a', d['ms_per_step'], d['roofline']['step_frac'], d['kernels']['num_step']['ms'], d['kernels']['bool_features']['ms'], d['config']['feature_layout'])"
done
