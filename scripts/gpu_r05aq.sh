set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/xt_count_time.py --variants nopair > gpurun_out/r05aq_count.json 2> gpurun_out/r05aq_count.err || exit $?
cat gpurun_out/r05aq_count.json
for v in base nopair base nopair base nopair; do
  if [ $v = base ]; then unset SOCCERACTION_AMD_LIB; else export SOCCERACTION_AMD_LIB=$PWD/socceraction_amd/_lib/libsocceraction_amd_$v.so; fi
  timeout -k 10 300 python -u bench.py --no-side --no-cpu > gpurun_out/r05aq_$v.json 2> gpurun_out/r05aq_$v.err || exit $?
  python -c "import json; d=json.load(open('gpurun_out/r05aq_$v.json')); print('$v', d['ms_per_step'], d['roofline']['step_frac'], d['kernels']['num_step']['ms'], d['kernels']['bool_features']['ms'], d['parity']['ok'])"
done
