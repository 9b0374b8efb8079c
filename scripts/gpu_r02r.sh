# round-2 GPU call R: counters of the bool feature kernel, block vs bitmap form
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r02r_trace -o run -- python3 scripts/bool_pmc.py > gpurun_out/r02r_trace.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY --output-format csv -d gpurun_out/prof_r02r_sq -o run -- python3 scripts/bool_pmc.py > gpurun_out/r02r_sq.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM_WR SQ_INSTS_SMEM --output-format csv -d gpurun_out/prof_r02r_sq2 -o run -- python3 scripts/bool_pmc.py > gpurun_out/r02r_sq2.log 2>&1
echo rc=$?
