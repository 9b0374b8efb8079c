# Final validation at head on ONE box: -m gpu, smoke, the default bench line, then the rocprofv3
# trace + PMC passes of the same build (so roofline.traffic is quoted and the kernel averages
# compare with the line's HIP events on the same hardware).  Usage: bash scripts/gpu_final.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
tag=${1:-final}
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > gpurun_out/${tag}_gpu_tests.log 2>&1
rc=$?
tail -2 gpurun_out/${tag}_gpu_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${tag}_smoke.log 2>&1 || exit $?
tail -1 gpurun_out/${tag}_smoke.log
timeout -k 10 400 python -u bench.py > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err || exit $?
python -c "import json; d=json.load(open('gpurun_out/${tag}_bench.json')); print(d['ms_per_step'], d['roofline']['step_frac'], d['kernels']['num_step']['ms'], d['kernels']['bool_features']['ms'])"
bash scripts/profile_round.sh ${tag} 10 > gpurun_out/${tag}_prof.log 2>&1 || exit $?
tail -1 gpurun_out/${tag}_prof.log
