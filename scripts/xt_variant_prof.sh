# rocprofv3 kernel trace + stats of one workload per library variant (A/B of build knobs, e.g.
# `python -m socceraction_amd.build -DSA_XK_U=8 --variant=u8`), rounds interleaved, then the
# per-kernel averages side by side (scripts/stats_table.py).
#   VARIANTS="default u8" ROUNDS=2 bash scripts/xt_variant_prof.sh TAG SCRIPT [ARGS...]
set -e
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
tag=$1
script=$2
shift 2
for r in $(seq 1 ${ROUNDS:-1}); do
  for v in ${VARIANTS:-default}; do
    if [ $v = default ]; then unset SOCCERACTION_AMD_LIB; else export SOCCERACTION_AMD_LIB=$GRAFT_REPO_ROOT/socceraction_amd/_lib/libsocceraction_amd_$v.so; fi
    timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_${v}_${r} -o run \
      -- python3 scripts/$script "$@" > gpurun_out/${tag}_${v}_$r.log 2>&1
    tail -1 gpurun_out/${tag}_${v}_$r.log
  done
done
python3 scripts/stats_table.py gpurun_out/${tag}_*_*/run_kernel_stats.csv > gpurun_out/${tag}_table.txt
cat gpurun_out/${tag}_table.txt
