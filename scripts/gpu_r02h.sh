# round-2 GPU call H: software-pipelined small-grid xT solve (prefetch depth variants)
bash scripts/gpu_steps.sh \
 "tests:300:python -u -m pytest tests/test_gpu_parity.py -k 'xt' -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider" \
 "xt_time:100:python scripts/xt_solve_time.py" \
 "xt_pf64:100:SOCCERACTION_AMD_LIB=socceraction_amd/_lib/libsocceraction_amd_pf64.so python scripts/xt_solve_time.py" \
 "xt_pf8:100:SOCCERACTION_AMD_LIB=socceraction_amd/_lib/libsocceraction_amd_pf8.so python scripts/xt_solve_time.py" \
 "ab:200:python bench.py --no-side --no-cpu --steps 20 --warmup 3 --ab 'sep:xt=cells;fused:xt=cells/order=num_features+bool_features+goalscore+labels_formula;fused_codes:xt=codes/fork=0/order=num_features+bool_features+goalscore+labels_formula'"
