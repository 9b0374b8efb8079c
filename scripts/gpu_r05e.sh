cd $GRAFT_REPO_ROOT
for v in xfprobe xfprobe_bank xfprobe_noreduce xfprobe_both; do
  SOCCERACTION_AMD_LIB=socceraction_amd/_lib/libsocceraction_amd_$v.so timeout -k 10 200 python -u scripts/xf_probe.py --reps 2 > gpurun_out/r05e_$v.log 2>&1 || exit 1
  echo $v; grep -v amdgpu.ids gpurun_out/r05e_$v.log | grep xf_probe | tail -1
done
