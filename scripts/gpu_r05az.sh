set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
run() {  # tag, args...
  t=$1; shift
  timeout -k 10 300 python -u scripts/cfg3_time.py "$@" > gpurun_out/r05az_$t.json 2> gpurun_out/r05az_$t.err || exit $?
  cat gpurun_out/r05az_$t.json
}
run long1 --times 2 --reps 300
run warm1 --times 2 --warm-games 200
run plain --times 2
run warm2 --times 2 --warm-games 200
