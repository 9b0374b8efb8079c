# round-2 GPU call G: staged tree walk v2
bash scripts/gpu_steps.sh \
 "tests:300:python -u -m pytest tests/test_gpu_trees.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider" \
 "tree_probe:200:python scripts/tree_probe.py --libs default,tg16,tg4"
