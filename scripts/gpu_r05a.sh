set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_xt_large.py "tests/test_gpu_parity.py::test_xt_large_grid_vs_oracle" > gpurun_out/r05a_tests.log 2>&1
rc=$?
tail -5 gpurun_out/r05a_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 240 python -u scripts/xt_large_time.py --batches 7 --reps 10 > gpurun_out/r05a_xt_large_time.json 2> gpurun_out/r05a_xt_large_time.err
rc=$?
cat gpurun_out/r05a_xt_large_time.json
exit $rc
