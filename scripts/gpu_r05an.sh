set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r05an_gpu_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r05an_gpu_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r05an_smoke.log 2>&1 || exit $?
tail -1 gpurun_out/r05an_smoke.log
