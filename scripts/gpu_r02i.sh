# round-2 GPU call I: bool kernel column assignment A/B (same allocations)
bash scripts/gpu_steps.sh \
 "bool_ab:300:python scripts/bool_ab.py --allocs 5 --variants strided,strided16,strided64"
