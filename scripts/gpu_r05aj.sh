set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_dropin.py tests/test_gpu_xt_large.py tests/test_gpu_parity.py > gpurun_out/r05aj_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r05aj_tests.log
exit $rc
