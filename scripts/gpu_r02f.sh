# round-2 GPU call F: staged tree walk probes
bash scripts/gpu_steps.sh \
 "tree_probe:200:python scripts/tree_probe.py --libs default,ts_nowalk,ts_nostage"
