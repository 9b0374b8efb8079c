set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py --steps 20 --warmup 2 --ab "base:;noxt:xt=none/diag=1" > gpurun_out/r05ao_ab.json 2> gpurun_out/r05ao_ab.err
rc=$?
cat gpurun_out/r05ao_ab.json
exit $rc
