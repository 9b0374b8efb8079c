set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 350 --timeout-method thread tests/test_gpu_bench.py -k "rccl" > gpurun_out/r05al_tests.log 2>&1
rc=$?
tail -40 gpurun_out/r05al_tests.log
exit $rc
