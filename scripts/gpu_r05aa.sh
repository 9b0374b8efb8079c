set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 200 python -u scripts/k4_time.py > gpurun_out/r05aa_k4.log 2>&1 || exit $?
tail -n 1 gpurun_out/r05aa_k4.log
