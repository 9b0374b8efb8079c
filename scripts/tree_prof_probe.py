import sys, os
sys.path.insert(0, os.getcwd())
import torch
from socceraction_amd import batch as B, ops, synthetic, trees
from bench import SPADL_DEFAULT
d = synthetic.spadl_games(2000)
ab = B.ActionBatch.from_columns(d)
fb = ops.features(ab, SPADL_DEFAULT, 3, bool_tile=1024, num_tile=128)
kinds = [k for _, k, _ in fb.plan.order]
m = trees.TreeEnsemble.from_xgboost_json(trees.synthetic_xgboost_json(len(kinds), 100, 3, 1, kinds))
for _ in range(3):
    p = m.predict_blocks(fb)
torch.cuda.synchronize()
print('ok', ab.n)
