# round-2 GPU call L: wave-mask tree evaluation -- parity vs the gather walk, timing per build
bash scripts/gpu_steps.sh \
 "trees_tests:400:python -u -m pytest tests/test_gpu_trees.py -x -v --timeout 200 --timeout-method thread" \
 "tree_probe:300:python scripts/tree_probe.py --libs default" \
 "tree_trace:300:cd /tmp && rocprofv3 --kernel-trace --stats --output-format csv -d \$GRAFT_REPO_ROOT/gpurun_out/prof_r02l_trees -o run -- python3 \$GRAFT_REPO_ROOT/scripts/tree_probe.py"
