"""Run by tests/test_gpu_rccl.py in its own process: the multi-GPU xT paths through REAL RCCL
(backend nccl) with one rank on one GPU.  With world size 1 every collective is an identity,
but each call goes through RCCL with the device tensors, dtypes, shapes and split lists the
N-GPU run uses -- the nccl branches of shard._all_reduce / _all_gather / _all_to_all /
_reduce_scatter that gloo rehearsals never execute.  Results must equal the single-GPU fit bit
for bit (exact_order) or within the reordered-solve tolerance."""
import json
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from socceraction_amd import batch as B, ops, shard, synthetic  # noqa: E402


def main():
    torch.cuda.set_device(0)
    dist.init_process_group('nccl', device_id=torch.device('cuda', 0))
    assert dist.get_backend() == 'nccl' and dist.get_world_size() == 1
    out = {}
    bs = [B.ActionBatch.from_columns(synthetic.spadl_games(g, game_id0=100 * k)) for k, g in enumerate((30, 45))]
    # 1. the counts' all-reduce (all_reduce of the whole int32 count allocation, 16 x 12)
    acc = ops.xt_count_many(bs, 16, 12)
    ref = [t.clone() for t in (acc.shot, acc.goal, acc.move, acc.trans, acc.err)]
    shard.allreduce_xt_counts(acc)
    out['allreduce_equal'] = all(torch.equal(a, b) for a, b in zip(ref, (acc.shot, acc.goal, acc.move, acc.trans, acc.err)))
    # 2. the band-sharded 105 x 68 fit: header + key all_to_all_single (uneven split lists),
    #    band-offset all_to_all, all_gather_into_tensor of the vectors / row lengths / packs,
    #    the error word's all_reduce; compact solve and the row-sharded solve
    l, w = 105, 68
    single = ops.xt_solve(ops.xt_count_many(bs, l, w), transition=False, exact_order=True)
    for solve in ('compact', 'rows'):
        st = {}
        mats, heat, n_iter, err = shard.xt_fit_bands_sharded(bs, l, w, solve=solve, exact_order=True, stats=st)
        out[f'bands_{solve}_equal'] = bool(n_iter == single.n_iter and torch.equal(mats, single.mats)
                                           and torch.equal(heat, single.heatmaps))
        out[f'bands_{solve}_exchange'] = st.get('exchange')
    # 3. the row-sharded solve from counts: reduce_scatter_tensor of the transition rows,
    #    all_gather_into_tensor of x per iteration, the MAX all_reduce of the flags
    acc = ops.xt_zero_counts(l, w, bs[0].device, row_blocks=1)
    for b in bs:
        ops.xt_count(b, l, w, acc)
    mats, heat, n_iter = shard.xt_solve_sharded(acc)
    out['rows_sharded_equal'] = bool(n_iter == single.n_iter and torch.equal(mats, single.mats))
    dist.destroy_process_group()
    print(json.dumps(out), flush=True)


if __name__ == '__main__':
    main()
