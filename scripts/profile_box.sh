#!/usr/bin/env bash
# Counter passes of the step's numeric and bool passes (scripts/step_pair.py) and of cfg3's atomic
# passes (--atomic) on whatever box this lands on: kernel trace, clock / wave cycles, instruction
# mix, FETCH_SIZE, WRITE_SIZE -- one rocprofv3 pass each (gfx950 counter slots).  Summarise with
#   python scripts/summarize_box.py TAG out.csv [--atomic]
# (effective clock = GRBM_GUI_ACTIVE / 8 / duration, VALU activity, HBM bytes per kernel).
set -euo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-box}
(rocm-smi --showclocks --showmemuse --showpower 2>&1 || true) > gpurun_out/${tag}_smi.txt
P="python3 scripts/step_pair.py --reps 5"
CLK="GRBM_GUI_ACTIVE GRBM_COUNT SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES"
INST="SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
for a in "" a; do
  flag=""; [ -n "$a" ] && flag="--atomic"
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_prof_${a}trace -o run -- $P $flag > gpurun_out/${tag}_${a}trace.log 2>&1
  timeout -s KILL 120 rocprofv3 --pmc $CLK --output-format csv -d gpurun_out/${tag}_prof_${a}clk -o run -- $P $flag > gpurun_out/${tag}_${a}clk.log 2>&1
  timeout -s KILL 120 rocprofv3 --pmc $INST --output-format csv -d gpurun_out/${tag}_prof_${a}inst -o run -- $P $flag > gpurun_out/${tag}_${a}inst.log 2>&1
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${tag}_prof_${a}fetch -o run -- $P $flag > gpurun_out/${tag}_${a}fetch.log 2>&1
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${tag}_prof_${a}write -o run -- $P $flag > gpurun_out/${tag}_${a}write.log 2>&1
done
echo box profile done
