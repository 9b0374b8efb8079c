# round-2 GPU call K: register-resident 16x12 solve (parts per row 2 / 1 / 4): xT parity per
# library, isolated timing, kernel trace, and the step with a normal / high-priority side stream
L=socceraction_amd/_lib
T="python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dropin.py -k xt -x -q --timeout 120 --timeout-method thread"
bash scripts/gpu_steps.sh \
 "xt_tests_xr2:300:$T" \
 "xt_tests_xr1:300:SOCCERACTION_AMD_LIB=$L/libsocceraction_amd_xr1.so $T" \
 "xt_tests_xr4:300:SOCCERACTION_AMD_LIB=$L/libsocceraction_amd_xr4.so $T" \
 "solve_xr2:120:python scripts/xt_solve_time.py" \
 "solve_xr1:120:SOCCERACTION_AMD_LIB=$L/libsocceraction_amd_xr1.so python scripts/xt_solve_time.py" \
 "solve_xr4:120:SOCCERACTION_AMD_LIB=$L/libsocceraction_amd_xr4.so python scripts/xt_solve_time.py" \
 "solve_trace:180:cd /tmp && rocprofv3 --kernel-trace --stats --output-format csv -d \$GRAFT_REPO_ROOT/gpurun_out/prof_r02k_solve -o run -- python3 \$GRAFT_REPO_ROOT/scripts/xt_solve_time.py" \
 "step_prio_xr2:300:python bench.py --no-side --no-cpu --steps 20 --warmup 3 --ab 'n:prio=normal;h:prio=high'" \
 "step_prio_xr1:300:SOCCERACTION_AMD_LIB=$L/libsocceraction_amd_xr1.so python bench.py --no-side --no-cpu --steps 20 --warmup 3 --ab 'n:prio=normal;h:prio=high'"
