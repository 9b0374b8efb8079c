set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_debug.py -k "xt or cell or step or debug" > gpurun_out/r05at_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r05at_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
for v in base c32; do
  if [ $v = base ]; then unset SOCCERACTION_AMD_LIB; else export SOCCERACTION_AMD_LIB=$PWD/socceraction_amd/_lib/libsocceraction_amd_$v.so; fi
  timeout -k 10 300 python -u scripts/xt_count_time.py > gpurun_out/r05at_count_$v.json 2> gpurun_out/r05at_count_$v.err || exit $?
  echo "$v $(tail -n 1 gpurun_out/r05at_count_$v.json)"
done
for v in base c32 base c32 base c32; do
  if [ $v = base ]; then unset SOCCERACTION_AMD_LIB; else export SOCCERACTION_AMD_LIB=$PWD/socceraction_amd/_lib/libsocceraction_amd_$v.so; fi
  timeout -k 10 300 python -u bench.py --no-side --no-cpu > gpurun_out/r05at_$v.json 2> gpurun_out/r05at_$v.err || exit $?
  python -c "import json; d=json.load(open('gpurun_out/r05at_$v.json')); print('$v', d['ms_per_step'], d['roofline']['step_frac'], d['kernels']['num_step']['ms'], d['kernels']['bool_features']['ms'], d['parity']['ok'])"
done
