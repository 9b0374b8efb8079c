"""The headline step's one bounded experiment (round 6): the bench step's two VAEP launches -- the
numeric step pass (sa_vaep_step_f64: f64 / i64 blocks, goalscore, xT cell codes, labels, f64
formula) and the bool pass -- against ONE call of sa_vaep_step_f64 with both column families.
In the default library that call is the same two launches; in the SA_FUSED_STEP=1 probe build
(`python -m socceraction_amd.build -DSA_FUSED_STEP=1 --variant=fused`, selected with
SOCCERACTION_AMD_LIB) it is one launch whose bool and numeric workgroups are interleaved.
Times both forms with HIP events (median of --reps) on cfg2's 10k games and checks that the
one-call outputs equal the two-launch outputs byte for byte.  Prints one JSON line."""
import argparse
import copy
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from socceraction_amd import _native, batch as B, catalog, ops, synthetic  # noqa: E402
from step_pair import SPADL_DEFAULT  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--games', type=int, default=10000)
    ap.add_argument('--reps', type=int, default=30)
    args = ap.parse_args()
    ab = B.ActionBatch.from_columns(synthetic.spadl_games(args.games))
    plan = catalog.build_plan(SPADL_DEFAULT, 3, False)
    n, dev = ab.n, ab.device
    s = ab.struct()
    p = synthetic.probabilities(n)
    ps = torch.from_numpy(p['scores']).to(dev)
    pc = torch.from_numpy(p['concedes']).to(dev)
    ld = (n + 15) // 16 * 16

    def outputs():
        out = ops.alloc_feature_blocks(plan, n, dev, 1024, 128, contiguous=True)
        lab_buf = torch.zeros((3, ld), dtype=torch.uint8, device=dev)
        lab = ops.LabelBlocks(n, lab_buf[0], lab_buf[1], lab_buf[2])
        val = torch.zeros((3, ld), dtype=torch.float64, device=dev)
        cells = ops.xt_cells_buffer(n, dev)
        return out, lab, lab_buf, val, cells

    def only(out, keep):
        q = copy.copy(plan)
        q.struct = copy.deepcopy(plan.struct)
        for x in range(len(q.struct.bool_col)):
            if keep == 'num':
                q.struct.bool_col[x] = -1
            else:
                q.struct.f64_col[x] = -1
                q.struct.i64_col[x] = -1
        o = copy.copy(out)
        o.plan = q
        return o

    sep, one = outputs(), outputs()
    numo, boolo = only(sep[0], 'num'), only(sep[0], 'bool')

    def two_launches():
        ops.step_into(s, numo, ps, pc, 10, sep[1], sep[3], xt_cells=(16, 12, sep[4]))
        ops.features_into(s, boolo)

    def one_call():
        ops.step_into(s, one[0], ps, pc, 10, one[1], one[3], xt_cells=(16, 12, one[4]))

    def timed(fn):
        for _ in range(3):
            fn()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in range(args.reps)]
        torch.cuda.synchronize()
        for a, b in ev:
            a.record()
            fn()
            b.record()
        torch.cuda.synchronize()
        t = sorted(a.elapsed_time(b) for a, b in ev)
        return t[len(t) // 2]

    rec = {'n': n, 'lib': os.path.basename(_native.LIB_PATH)}
    # interleave the two forms' timings (3 rounds) so clock drift hits both
    t2, t1 = [], []
    for _ in range(3):
        t2.append(timed(two_launches))
        t1.append(timed(one_call))
    rec['two_launches_ms'] = round(min(t2), 4)
    rec['one_call_ms'] = round(min(t1), 4)
    rec['one_over_two'] = round(min(t1) / min(t2), 4)
    eq = {}
    for name, a, b in (('bool', sep[0].bool_block, one[0].bool_block),
                       ('f64', sep[0].f64_block, one[0].f64_block),
                       ('i64', sep[0].i64_block, one[0].i64_block),
                       ('labels', sep[2], one[2]), ('cells', sep[4][:n], one[4][:n])):
        eq[name] = bool(torch.equal(a.view(torch.uint8) if a.dtype != torch.uint8 else a,
                                    b.view(torch.uint8) if b.dtype != torch.uint8 else b))
    eq['values'] = bool(torch.equal(sep[3].view(torch.int64), one[3].view(torch.int64)))
    rec['equal'] = eq
    rec['bytes_per_action'] = 522 + 516  # bench BYTES: bool_features + num_step + 2-B cell code
    rec['one_call_GBs'] = round(n * rec['bytes_per_action'] / (min(t1) * 1e-3) / 1e9, 1)
    print(json.dumps(rec), flush=True)
    if not all(eq.values()):
        sys.exit(1)


if __name__ == '__main__':
    main()
