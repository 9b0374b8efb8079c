set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_xt_large.py "tests/test_gpu_parity.py::test_xt_large_grid_vs_oracle" > gpurun_out/r05d_tests.log 2>&1
rc=$?
tail -4 gpurun_out/r05d_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
for v in xfprobe xfprobe_p1 xfprobe_p4; do
  SOCCERACTION_AMD_LIB=socceraction_amd/_lib/libsocceraction_amd_$v.so timeout -k 10 200 python -u scripts/xf_probe.py --reps 3 > gpurun_out/r05d_$v.log 2>&1 || exit 1
  grep -v amdgpu.ids gpurun_out/r05d_$v.log
done
