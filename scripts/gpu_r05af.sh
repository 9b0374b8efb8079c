set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
(timeout -k 5 30 rocm-smi --showclocks --showpower --showtemp > gpurun_out/r05af_smi_before.log 2>&1 || true)
timeout -k 10 300 python -u bench.py --no-side --no-cpu --steps 50 > gpurun_out/r05af_bench.json 2> gpurun_out/r05af_bench.err || exit $?
(timeout -k 5 30 rocm-smi --showclocks --showpower --showtemp > gpurun_out/r05af_smi_after.log 2>&1 || true)
python -c "import json; d=json.load(open('gpurun_out/r05af_bench.json')); print(d['ms_per_step'], d['roofline']['step_frac'], d['kernels'])"
grep -i "sclk\|mclk\|fclk\|socclk\|Power\|Temp" gpurun_out/r05af_smi_after.log | head -20
