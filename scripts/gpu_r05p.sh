set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/rate_lib_ab.py --variants xripack,xripacku4 > gpurun_out/r05p_rate_ab.json 2> gpurun_out/r05p_rate_ab.err
rc=$?
cat gpurun_out/r05p_rate_ab.json
exit $rc
