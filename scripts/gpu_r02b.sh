# round-2 GPU call B: GPU suite, bench, in-process A/B of the xT source, rocprof stats
bash scripts/gpu_steps.sh \
 "tests:600:python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread -p no:cacheprovider" \
 "bench:240:python bench.py --steps 20 --warmup 5" \
 "ab_xt:180:python bench.py --no-side --no-cpu --steps 20 --warmup 3 --ab 'cells:xt=cells;codes:xt=codes/fork=0;coords:xt=coords/fork=0'" \
 "prof:150:rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o r02b -- python bench.py --steps 10 --warmup 3 --no-cpu --e2e-games 0"
