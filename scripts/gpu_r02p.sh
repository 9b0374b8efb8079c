# round-2 GPU call P: bitmap features + staged walk from bitmaps -- tests and kernel trace
bash scripts/gpu_steps.sh \
 "trees_tests:400:python -u -m pytest tests/test_gpu_trees.py tests/test_gpu_dropin.py -x -q --timeout 200 --timeout-method thread" \
 "tree_trace:300:cd /tmp && rocprofv3 --kernel-trace --stats --output-format csv -d \$GRAFT_REPO_ROOT/gpurun_out/prof_r02p_trees -o run -- python3 \$GRAFT_REPO_ROOT/scripts/tree_probe.py"
