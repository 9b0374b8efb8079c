set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/cfg3_time.py --times 3 > gpurun_out/r05au_alone.json 2> gpurun_out/r05au_alone.err || exit $?
cat gpurun_out/r05au_alone.json
timeout -k 10 300 python -u scripts/cfg3_time.py --times 3 --after-step > gpurun_out/r05au_after.json 2> gpurun_out/r05au_after.err || exit $?
cat gpurun_out/r05au_after.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r05au_prof -o run -- python3 scripts/cfg3_time.py --times 2 > gpurun_out/r05au_prof.log 2>&1 || exit $?
tail -1 gpurun_out/r05au_prof.log
