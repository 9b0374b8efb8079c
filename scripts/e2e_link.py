"""Where bench.py's end_to_end entry (pandas in -> pandas out, 1000 games) spends its time,
against the host link: pinned H2D / D2H GB/s measured in-process, then each stage of the
drop-in batched calls (encode + H2D, kernels, D2H, DataFrame assembly), synchronised between
stages.  Prints one JSON line."""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from socceraction_amd import ops, synthetic, vaep  # noqa: E402
from socceraction_amd.batch import ActionBatch  # noqa: E402


def link_rates(nbytes=1 << 30, reps=5):
    dev = torch.empty(nbytes, dtype=torch.uint8, device='cuda')
    host = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
    out = {}
    for name, dst, src in (('d2h', host, dev), ('h2d', dev, host)):
        t = []
        for _ in range(reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            dst.copy_(src, non_blocking=True)
            torch.cuda.synchronize()
            t.append(time.perf_counter() - t0)
        out[name + '_GBs'] = round(nbytes / min(t) / 1e9, 2)
    return out


def main():
    games = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
    rec = link_rates()
    d = synthetic.spadl_games(games)
    actions = synthetic.to_frame(d)
    gframe = synthetic.games_frame(d)
    home_of = gframe.set_index('game_id')['home_team_id']
    model = vaep.VAEP()
    n = len(actions)
    for _ in range(3):
        stage = {}
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ab = ActionBatch.from_frame(actions, home_team_id=home_of, segments='game')
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        fb = ops.features(ab, model._split_xfns()[0], 3)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        b, f, i = fb.to_numpy()
        t3 = time.perf_counter()
        from socceraction_amd.catalog import assemble_frame
        import pandas as pd
        X = assemble_frame(fb.plan, b, f, i, n, pd.RangeIndex(n))
        t4 = time.perf_counter()
        t5 = time.perf_counter()
        X2 = model.compute_features_batch(gframe, actions)
        t6 = time.perf_counter()
        Y = model.compute_labels_batch(gframe, actions)
        t7 = time.perf_counter()
        stage = {'encode_h2d_s': t1 - t0, 'kernels_s': t2 - t1, 'd2h_s': t3 - t2,
                 'assemble_s': t4 - t3, 'features_batch_s': t6 - t5, 'labels_batch_s': t7 - t6,
                 'd2h_bytes': int(b.nbytes + f.nbytes + i.nbytes)}
        assert X.shape == X2.shape == (n, 568) and len(Y) == n
    stage = {k: (round(v, 4) if isinstance(v, float) else v) for k, v in stage.items()}
    stage['d2h_GBs_in_path'] = round(stage['d2h_bytes'] / stage['d2h_s'] / 1e9, 2)
    print(json.dumps({'actions': n, **rec, **stage}), flush=True)


if __name__ == '__main__' and not (len(sys.argv) > 2 and sys.argv[2] == 'probe'):
    main()


def pipeline_probe(games: int = 1000):
    """VAEP.compute_batch's pieces: the pitched D2H alone (one chunk's blocks into the frame's
    host blocks) against a contiguous D2H of the same bytes, the host encode of one chunk, and
    the whole call with its chunk size varied."""
    from socceraction_amd import _native, catalog
    d = synthetic.spadl_games(games)
    actions = synthetic.to_frame(d)
    gframe = synthetic.games_frame(d)
    model = vaep.VAEP()
    n = len(actions)
    p = synthetic.probabilities(n)
    out = {}
    plan = catalog.build_plan(model._split_xfns()[0], 3, False)
    m = 1 << 18
    fb = ops.alloc_feature_blocks(plan, m, 'cuda')
    hb = torch.empty((plan.n_bool, n), dtype=torch.uint8, pin_memory=True)
    hb1 = torch.empty((plan.n_bool, m), dtype=torch.uint8, pin_memory=True)
    src = fb.bool_block[0]
    lib = _native.lib()
    s = torch.cuda.current_stream()
    def pitched(dst_off, src_off, width):
        return lambda: _native.check(lib.sa_copy2d_async(
            hb.data_ptr() + dst_off, n, src.data_ptr() + src_off, src.shape[-1], width, plan.n_bool,
            s.cuda_stream))
    cases = [('pitched_d2h_GBs', pitched(0, 0, m)),
             ('contiguous_d2h_GBs', lambda: hb1.copy_(src[:, :m], non_blocking=True))]
    for a in (1, 2, 4, 8, 16, 64, 256):  # dst and src offsets of a bytes (both), odd width
        cases.append((f'pitched_d2h_off_{a}_GBs', pitched(262144 + a, a, m - 257)))
    cases.append(('pitched_d2h_off_0_oddwidth_GBs', pitched(262144, 0, m - 257)))
    cases.append(('pitched_d2h_dstoff_4_srcoff_0_GBs', pitched(262144 + 4, 0, m - 257)))
    cases.append(('pitched_d2h_dstoff_0_srcoff_4_GBs', pitched(262144, 4, m - 257)))
    for name, fn in cases:
        t = []
        for _ in range(5):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            t.append(time.perf_counter() - t0)
        out[name] = round(plan.n_bool * m / min(t) / 1e9, 2)
    home_of = gframe.set_index('game_id')['home_team_id']
    t0 = time.perf_counter()
    sub = actions.iloc[:m]
    ab = ActionBatch.from_frame(sub, home_team_id=home_of, segments='game')
    torch.cuda.synchronize()
    out['encode_h2d_ms_per_256k_rows'] = round((time.perf_counter() - t0) * 1e3, 2)
    for chunk in (1 << 18, 1 << 21):
        model.compute_batch(gframe, actions, p['scores'], p['concedes'], chunk_rows=chunk)
        t = []
        for _ in range(3):
            t0 = time.perf_counter()
            model.compute_batch(gframe, actions, p['scores'], p['concedes'], chunk_rows=chunk)
            t.append(time.perf_counter() - t0)
        out[f'compute_batch_ms_chunk_{chunk}'] = round(min(t) * 1e3, 2)
    from socceraction_amd.pipeline import value_frames
    for ramp in ((4, 2), (), (8, 4, 2)):  # the first chunks' sizes: chunk_rows / ramp[i]
        t = []
        for _ in range(4):
            t0 = time.perf_counter()
            value_frames(model, gframe, actions, p['scores'], p['concedes'], chunk_rows=1 << 18, ramp=ramp)
            t.append(time.perf_counter() - t0)
        out[f'value_frames_ms_ramp_{"_".join(map(str, ramp)) or "none"}'] = round(min(t[1:]) * 1e3, 2)
    tl = []
    value_frames(model, gframe, actions, p['scores'], p['concedes'], chunk_rows=1 << 18, timeline=tl)
    out['timeline_chunk_262144'] = tl
    print(json.dumps({'pipeline_probe': out}), flush=True)


if __name__ == '__main__' and len(sys.argv) > 2 and sys.argv[2] == 'probe':
    pipeline_probe(int(sys.argv[1]))
