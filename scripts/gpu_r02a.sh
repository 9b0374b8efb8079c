# round-2 GPU call A: the GPU test suite + smoke()
bash scripts/gpu_steps.sh \
 "tests:900:python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread -p no:cacheprovider" \
 "smoke:200:python -c 'import __graft_entry__ as g; g.smoke()'"
