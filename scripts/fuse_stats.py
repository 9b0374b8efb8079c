"""A/B diagnostics for the fused bool kernel (library built with SA_BOOL_MODE=4 SA_FUSE_STATS=1):
one bool-block launch over the cfg2 batch, then how many consumer waves waited for their
producer, fell back, or saw a producer flag from another XCD, and the total polls."""
import ctypes
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from socceraction_amd import _native, batch as B, catalog, ops, synthetic  # noqa: E402

SPADL_DEFAULT = ['actiontype_onehot', 'result_onehot', 'actiontype_result_onehot',
                 'bodypart_onehot', 'team']
lib = _native.load_library()
dev = B.device()
d = synthetic.spadl_games(10000)
ab = B.ActionBatch.from_columns(d, dev=dev)
plan = catalog.build_plan(SPADL_DEFAULT, 3)
out = ops.alloc_feature_blocks(plan, ab.n, dev)
s = ab.struct()
buf = (ctypes.c_ulonglong * 4)()
for rep in range(3):
    lib.sa_debug_fuse_stats(buf, 1)
    ops.features_into(s, out)
    torch.cuda.synchronize()
    lib.sa_debug_fuse_stats(buf, 1)
    print(json.dumps({'rep': rep, 'waited': buf[0], 'fallback': buf[1], 'other_xcd': buf[2],
                      'polls': buf[3], 'waves': (ab.n + 1023) // 1024 * 515}), flush=True)
