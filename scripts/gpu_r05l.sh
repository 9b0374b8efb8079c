set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_xt_large.py > gpurun_out/r05l_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r05l_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u scripts/cfg5_trace.py > gpurun_out/r05l_plain.log 2>&1 || exit $?
cat gpurun_out/r05l_plain.log
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r05l_trace -o run -- python3 scripts/cfg5_trace.py > gpurun_out/r05l_trace.log 2>&1
