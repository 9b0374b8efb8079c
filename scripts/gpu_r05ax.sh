set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
run() {  # tag, args...
  t=$1; shift
  timeout -k 10 300 python -u scripts/cfg3_time.py --times 3 "$@" > gpurun_out/r05ax_$t.json 2> gpurun_out/r05ax_$t.err || exit $?
  cat gpurun_out/r05ax_$t.json
}
run all1 --contiguous all
run req1 --contiguous require
run all2 --contiguous all
run req2 --contiguous require
