set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_xt_large.py tests/test_gpu_dropin.py tests/test_gpu_debug.py tests/test_gpu_parity.py -k "xt or compact or band or rate or debug" > gpurun_out/r05ab_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r05ab_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 200 python -u scripts/bucket_time.py > gpurun_out/r05ab_bucket.log 2>&1 || exit $?
tail -n 1 gpurun_out/r05ab_bucket.log
for i in 1 2; do timeout -k 10 200 python -u scripts/cfg5_trace.py > gpurun_out/r05ab_t$i.log 2>&1 || exit $?; tail -n 1 gpurun_out/r05ab_t$i.log; done
