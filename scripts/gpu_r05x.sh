set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_xt_large.py tests/test_gpu_dropin.py -k "xt or compact or band or rate" > gpurun_out/r05x_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r05x_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
for i in 1 2; do timeout -k 10 200 python -u scripts/cfg5_trace.py > gpurun_out/r05x_t$i.log 2>&1 || exit $?; tail -n 1 gpurun_out/r05x_t$i.log; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r05x_trace -o run -- python3 scripts/cfg5_trace.py --calls 3 > gpurun_out/r05x_trace.log 2>&1
