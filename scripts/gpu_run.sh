# One parameterised GPU runner (replaces the per-call gpu_r05*.sh scripts of round 5).
#   bash scripts/gpu_run.sh TAG STEP [STEP ...]
# Steps run in order, each under its own time limit; the first failing step ends the run (no
# retries).  Outputs land in gpurun_out/TAG_*.
#   tests[:A,B,..]    python -m pytest tests -m gpu (-k "A or B")    -> TAG_gpu_tests.log
#   smoke             __graft_entry__.smoke()                      -> TAG_smoke.log
#   bench[:ARGS]      python bench.py ARGS (commas = spaces)       -> TAG_bench.json / .err
#   prof              scripts/profile_round.sh TAG 10 (trace + PMC) -> gpurun_out/prof_TAG_*
#   py:SCRIPT[:ARGS]  python scripts/SCRIPT ARGS (commas = spaces) -> TAG_SCRIPT.log
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=$1
shift
for step in "$@"; do
  kind=${step%%:*}
  arg=""
  [ "$kind" != "$step" ] && arg=${step#*:}
  case $kind in
    tests)
      k=()
      [ -n "$arg" ] && k=(-k "${arg//,/ or }")  # commas: alternatives
      timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread "${k[@]}" \
        > gpurun_out/${tag}_gpu_tests.log 2>&1
      rc=$?
      tail -3 gpurun_out/${tag}_gpu_tests.log ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" \
        > gpurun_out/${tag}_smoke.log 2>&1
      rc=$?
      tail -1 gpurun_out/${tag}_smoke.log ;;
    bench)
      timeout -k 10 600 python -u bench.py ${arg//,/ } > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err
      rc=$?
      [ $rc -eq 0 ] && python -c "import json; d=json.load(open('gpurun_out/${tag}_bench.json')); x=d.get('xt105_cfg5', {}); print(d['ms_per_step'], d['roofline']['step_frac'], d['kernels']['num_step']['ms'], x.get('ms_fit_and_rate'), x.get('phases_ms'))" ;;
    prof)
      bash scripts/profile_round.sh ${tag} 10 > gpurun_out/${tag}_prof.log 2>&1
      rc=$?
      tail -1 gpurun_out/${tag}_prof.log ;;
    py)
      script=${arg%%:*}
      sargs=""
      [ "$script" != "$arg" ] && sargs=${arg#*:}
      timeout -k 10 600 python -u scripts/${script} ${sargs//,/ } > gpurun_out/${tag}_${script%.py}.log 2>&1
      rc=$?
      tail -5 gpurun_out/${tag}_${script%.py}.log ;;
    *)
      echo "unknown step $step"; exit 2 ;;
  esac
  if [ $rc -ne 0 ]; then
    echo "step $step failed: $rc"
    exit $rc
  fi
done
