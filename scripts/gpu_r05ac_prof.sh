set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash scripts/profile_round.sh r05ac 10 > gpurun_out/r05ac_prof.log 2>&1
rc=$?
tail -3 gpurun_out/r05ac_prof.log
exit $rc
