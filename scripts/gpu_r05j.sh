set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread "tests/test_gpu_parity.py::test_chunked_step_equals_step" > gpurun_out/r05j_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r05j_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 --ab "base:;c2m:chunk=2097152;c2mp:chunk=2097152/pf=1;c1mp:chunk=1048576/pf=1;c4mp:chunk=4194304/pf=1;c05mp:chunk=524288/pf=1" > gpurun_out/r05j_ab.json 2> gpurun_out/r05j_ab.err
rc=$?
cat gpurun_out/r05j_ab.json
exit $rc
