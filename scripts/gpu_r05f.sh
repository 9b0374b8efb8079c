set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_xt_large.py "tests/test_gpu_parity.py::test_xt_large_grid_vs_oracle" > gpurun_out/r05f_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r05f_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
for v in xfprobe xfprobe_noreduce; do
  SOCCERACTION_AMD_LIB=socceraction_amd/_lib/libsocceraction_amd_$v.so timeout -k 10 200 python -u scripts/xf_probe.py --reps 2 > gpurun_out/r05f_$v.log 2>&1 || exit 1
  echo $v; grep -v amdgpu.ids gpurun_out/r05f_$v.log | tail -2
done
