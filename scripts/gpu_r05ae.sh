set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/e2e_profile.py > gpurun_out/r05ae_e2e.log 2>&1
rc=$?
head -80 gpurun_out/r05ae_e2e.log
exit $rc
