#!/usr/bin/env bash
# rocprofv3 passes over the device tree inference (scripts/cond_probe.py: the condition-bitmap
# VAEP.rate path and the float32-block path on cfg2): kernel trace + stats, then separate PMC
# passes (FETCH_SIZE, WRITE_SIZE, SQ instruction / LDS counters). Outputs under gpurun_out/.
set -euo pipefail
export TMPDIR=/tmp
tag=${1:-r05_tree}
mkdir -p gpurun_out
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${tag}_trace -o run \
  -- python3 scripts/cond_probe.py > gpurun_out/prof_${tag}_trace.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof_${tag}_fetch -o run \
  -- python3 scripts/cond_probe.py > gpurun_out/prof_${tag}_fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof_${tag}_write -o run \
  -- python3 scripts/cond_probe.py > gpurun_out/prof_${tag}_write.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d gpurun_out/prof_${tag}_sq -o run \
  -- python3 scripts/cond_probe.py > gpurun_out/prof_${tag}_sq.log 2>&1 || echo "sq pass failed"
echo profile done
