# round-2 GPU call E: register-resident xT solve, batched staged tree walk
bash scripts/gpu_steps.sh \
 "tests:500:python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dropin.py tests/test_gpu_trees.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider" \
 "xt_time:120:python scripts/xt_solve_time.py" \
 "xt_time_small:120:SOCCERACTION_AMD_LIB=socceraction_amd/_lib/libsocceraction_amd_solve_small.so python scripts/xt_solve_time.py" \
 "prof:240:rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o r02e -- python bench.py --steps 10 --warmup 3 --no-cpu --e2e-games 0 --order num_features,bool_features,goalscore,labels_formula"
