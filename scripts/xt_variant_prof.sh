set -e
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
for v in ${VARIANTS:-default}; do
  if [ $v = default ]; then unset SOCCERACTION_AMD_LIB; else export SOCCERACTION_AMD_LIB=$GRAFT_REPO_ROOT/socceraction_amd/_lib/libsocceraction_amd_$v.so; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/xtprof_$v -o run -- python3 scripts/bench_workloads.py xt105 > gpurun_out/xtprof_$v.log 2>&1
done
