# cfg3's bimodal placement: the same cfg3 runs (scripts/cfg3_time.py, 3 runs of the
# atomic step in one process) under a kernel trace and under counter passes -- address
# translation (UTCL1 hits / misses, UTCL2 busy), HBM bytes, the SQ wait mix -- so that a slow
# first run and the fast later runs of the same process can be compared dispatch by dispatch
# (scripts/cfg3_counters_summary.py).  Every pass is its own process: each may or may not land
# in the slow mode, and each reports its own runs.
#   bash scripts/cfg3_counters.sh TAG
set -e
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
tag=$1
run() {  # name, rocprofv3 options...
  local name=$1
  shift
  timeout -s KILL 200 rocprofv3 "$@" --output-format csv -d gpurun_out/${tag}_$name -o run \
    -- python3 scripts/cfg3_time.py --times 3 --reps 11 > gpurun_out/${tag}_$name.log 2>&1 || echo "pass $name failed"
  tail -1 gpurun_out/${tag}_$name.log | cut -c1-300
}
run trace --kernel-trace
run tlb --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum GRBM_UTCL2_BUSY GRBM_GUI_ACTIVE
run hbm --pmc FETCH_SIZE
run sq --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE
python3 scripts/cfg3_counters_summary.py $tag > gpurun_out/${tag}_summary.txt || true
cat gpurun_out/${tag}_summary.txt
