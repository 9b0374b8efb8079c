set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u scripts/feature_lib_ab.py --variants w4 --reps 10 > gpurun_out/r05ad_w4_ab.json 2> gpurun_out/r05ad_w4_ab.err
rc=$?
python -c "
import json; d=json.load(open('gpurun_out/r05ad_w4_ab.json'))
for k,v in d['ms'].items():
    if 'step' in k or 'pair' in k: print(k, v)
print(d['equal'])"
exit $rc
