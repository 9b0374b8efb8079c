# round-2 GPU call C: xT solve rework + LDS-free bool kernel: parity subset, standalone xT times,
# in-process A/B of the step variants, kernel trace
bash scripts/gpu_steps.sh \
 "tests:400:python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dropin.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider" \
 "xt_time:120:python scripts/xt_solve_time.py" \
 "ab:240:python bench.py --no-side --no-cpu --steps 20 --warmup 3 --ab 'cells:xt=cells;codes:xt=codes/fork=0;cells_bf:xt=cells/order=bool_features+num_features+goalscore+labels+formula/fork=2'" \
 "prof:150:rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o r02c -- python bench.py --steps 10 --warmup 3 --no-cpu --no-side"
