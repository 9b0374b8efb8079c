# round-2 GPU call J: full GPU suite, smoke, default bench, rocprofv3 trace + PMC passes
bash scripts/gpu_steps.sh \
 "tests:900:python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread" \
 "smoke:180:python -c 'import __graft_entry__ as g; g.smoke()'" \
 "bench:420:python bench.py" \
 "profile:700:bash scripts/profile_round.sh r02 10"
