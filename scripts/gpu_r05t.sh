set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for v in base xbr2 xbr3 xbr4 base xbr2 xbr3 xbr4; do
  if [ $v = base ]; then unset SOCCERACTION_AMD_LIB; else export SOCCERACTION_AMD_LIB=$PWD/socceraction_amd/_lib/libsocceraction_amd_$v.so; fi
  timeout -k 10 200 python -u scripts/cfg5_trace.py > gpurun_out/r05t_$v.log 2>&1 || exit $?
  echo "$v $(tail -n 1 gpurun_out/r05t_$v.log)"
done
