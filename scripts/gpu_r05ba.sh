set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
V=$GRAFT_REPO_ROOT/socceraction_amd/_lib/libsocceraction_amd_xkb0.so
timeout -k 10 200 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_xt_large.py > gpurun_out/r05ba_t.log 2>&1 || { tail -5 gpurun_out/r05ba_t.log; exit 1; }
tail -1 gpurun_out/r05ba_t.log
for i in 1 2 3; do
  timeout -k 10 200 python -u scripts/cfg5_time.py > gpurun_out/r05ba_new$i.json 2> gpurun_out/r05ba_new$i.err || exit $?
  cat gpurun_out/r05ba_new$i.json
  SOCCERACTION_AMD_LIB=$V timeout -k 10 200 python -u scripts/cfg5_time.py > gpurun_out/r05ba_old$i.json 2> gpurun_out/r05ba_old$i.err || exit $?
  cat gpurun_out/r05ba_old$i.json
done
