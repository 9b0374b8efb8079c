# rocprofv3 PMC passes (one counter group per run, each under its own kill timer) of one
# workload script: SQ issue / wait mix, clock, and HBM bytes.  Outputs gpurun_out/TAG_pmc_*.
#   bash scripts/pmc_passes.sh TAG SCRIPT [ARGS...]
set -e
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
tag=$1
script=$2
shift 2
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i + 1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/${tag}_pmc_$i -o run \
    -- python3 scripts/$script "$@" > gpurun_out/${tag}_pmc_$i.log 2>&1 || echo "pmc pass $i failed"
done
python3 scripts/pmc_table.py gpurun_out/${tag}_pmc_*/run_counter_collection.csv > gpurun_out/${tag}_pmc_table.txt || true
cat gpurun_out/${tag}_pmc_table.txt
