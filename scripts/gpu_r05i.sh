set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_trees.py > gpurun_out/r05i_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r05i_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 200 python -u scripts/cond_probe.py > gpurun_out/r05i_cond.json 2>gpurun_out/r05i_cond.err
rc=$?
cat gpurun_out/r05i_cond.json
exit $rc
