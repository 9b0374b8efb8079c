set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for v in base xkp1 xkp2 xkp3 base; do
  if [ $v = base ]; then unset SOCCERACTION_AMD_LIB; else export SOCCERACTION_AMD_LIB=$PWD/socceraction_amd/_lib/libsocceraction_amd_$v.so; fi
  timeout -k 10 200 python -u scripts/bucket_time.py > gpurun_out/r05u_$v.log 2>&1 || exit $?
  echo "$v $(tail -n 1 gpurun_out/r05u_$v.log)"
done
unset SOCCERACTION_AMD_LIB
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r05u_prof -o run -- python3 scripts/bucket_time.py > gpurun_out/r05u_prof.log 2>&1
