# round-2 GPU call S: counters of the f64 / i64 feature kernel
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r02s_trace -o run -- python3 scripts/num_pmc.py > gpurun_out/r02s_trace.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY --output-format csv -d gpurun_out/prof_r02s_sq -o run -- python3 scripts/num_pmc.py > gpurun_out/r02s_sq.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 --output-format csv -d gpurun_out/prof_r02s_sq2 -o run -- python3 scripts/num_pmc.py > gpurun_out/r02s_sq2.log 2>&1
echo rc=$?
