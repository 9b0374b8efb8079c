set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
run() {  # tag, args...
  t=$1; shift
  timeout -k 10 300 python -u scripts/cfg3_time.py "$@" > gpurun_out/r05ay_$t.json 2> gpurun_out/r05ay_$t.err || exit $?
  cat gpurun_out/r05ay_$t.json
}
run bc1 --contiguous require --batch-contiguous --times 2
run req1 --contiguous require --times 2
run bc2 --contiguous require --batch-contiguous --times 2
run req2 --contiguous require --times 2
