set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_xt_large.py tests/test_gpu_bench.py "tests/test_gpu_dropin.py::test_xt_row_sharded_solve_two_ranks" > gpurun_out/r05h_tests.log 2>&1
rc=$?
tail -15 gpurun_out/r05h_tests.log
exit $rc
