set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u - > gpurun_out/r05s_check.log 2>&1 <<'PY'
import sys; sys.path.insert(0, '.')
import torch
from socceraction_amd import batch as B, ops, synthetic
bs = [B.ActionBatch.from_columns(synthetic.spadl_games(10000, game_id0=k * 10000)) for k in range(7)]
a = ops.xt_count_many(bs, 105, 68, overlap=False)
b = ops.xt_count_many(bs, 105, 68, overlap=True)
torch.cuda.synchronize()
print('equal', all(torch.equal(x, y) for x, y in ((a.trans, b.trans), (a.shot, b.shot), (a.goal, b.goal), (a.move, b.move), (a.err, b.err))))
PY
rc=$?
cat gpurun_out/r05s_check.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u scripts/cfg5_trace.py > gpurun_out/r05s_base.log 2>&1 || exit $?
SA_XT_BUCKET_OVERLAP=1 timeout -k 10 300 python -u scripts/cfg5_trace.py > gpurun_out/r05s_ovl.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/cfg5_trace.py > gpurun_out/r05s_base2.log 2>&1 || exit $?
for f in base ovl base2; do tail -n 1 gpurun_out/r05s_$f.log; done
SA_XT_BUCKET_OVERLAP=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r05s_trace -o run -- python3 scripts/cfg5_trace.py --calls 3 > gpurun_out/r05s_trace.log 2>&1
