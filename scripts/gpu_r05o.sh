set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u scripts/feature_lib_ab.py --variants stg1,stg2,stg4 --reps 10 > gpurun_out/r05o_stage_ab.json 2> gpurun_out/r05o_stage_ab.err
rc=$?
tail -c 3000 gpurun_out/r05o_stage_ab.json
exit $rc
