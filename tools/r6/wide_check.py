"""Round-6 WIDE bring-up check (GPU box): DREAM (Zipf, 5 replicas) and LOKI
bank 0 at several TOA binnings, WIDE forced and AUTO, current histogram vs
oracle/binning_ref.c on the same events.  Test infrastructure only."""
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))

import torch  # noqa: E402

from esslivedata_amd import projection, synthetic  # noqa: E402
from esslivedata_amd.engine import BinningEngine  # noqa: E402
from oracle import c_oracle  # noqa: E402
from oracle import scipp_semantics as ora  # noqa: E402

N = int(os.environ.get('WC_EVENTS', '5000000'))
threads = int(os.environ.get('OMP_NUM_THREADS', '16'))
specs = os.environ.get('WC_SPECS', 'dream:100:log,dream:164:log,dream:1000:log,dream:1000:log:0.01,'
                       'dream:10000:log,loki:164:linear,loki:1000:linear,loki:10000:linear').split(',')
strategies = os.environ.get('WC_STRATEGIES', 'wide,auto').split(',')
bad = 0
for spec in specs:
    f = spec.split(':')
    w, nb, sc = f[0], int(f[1]), f[2]
    st = float(f[3]) if len(f) > 3 else None
    inst = synthetic.dream_mantle() if w == 'dream' else synthetic.loki_bank0()
    inst = synthetic.with_toa_edges(inst, num_bins=nb, scale=sc, start=st)
    flip = w == 'loki'
    view = projection.geometric_lut(inst.detector_number, inst.coords, inst.resolution, flip_x=flip)
    edges = inst.edges.edges_ns()
    if w == 'dream':
        pid, toa = synthetic.dream_events(N, inst, seed=11)
    else:
        pid, toa = synthetic.uniform_events(N, 1, 802816, seed=12)
    rep = 1
    ps = ora.geometric_pixel_screen(inst.coords, inst.resolution, flip_x=flip)
    c = c_oracle.CDetectorView(inst.detector_number, ps, view.n_screen, edges, threads=threads)
    c.accumulate(pid, toa, rep)
    ref = c.hist.reshape(view.n_screen, nb).astype(np.float64)
    for strat in strategies:
        eng = BinningEngine(toa_edges_ns=edges, out_lut=view.lut, pid_offset=view.pid_offset,
                            n_screen=view.n_screen, strategy=strat)
        dp = torch.as_tensor(pid, device='cuda')
        dt = torch.as_tensor(toa, device='cuda')
        h = len(pid) // 3
        for k in range(2):  # second pass: tables already built
            eng.stage_tensors_batch([(dp[:h], dt[:h]), (dp[h:], dt[h:])])
            t0 = time.perf_counter()
            eng.accumulate(rep)
            torch.cuda.synchronize()
            dt_ms = 1e3 * (time.perf_counter() - t0)
            res = eng.finalize(hists=True)
        ok = np.array_equal(res.current_hist, ref)
        bad += not ok
        info = eng.info()
        cnt = {k: eng.counter(k) for k in ('wide_levels', 'wide_parts', 'wide_tree_words', 'wide_tree_lds')}
        print(f'{spec:22s} {strat:5s} -> {info["last_strategy"]:7s} exact={ok} {dt_ms:7.3f} ms '
              f'total {res.current_total} ref {int(ref.sum())} {cnt}', flush=True)
        if not ok:
            d = np.argwhere(res.current_hist != ref)
            print('   first diffs', d[:5].tolist(), res.current_hist[tuple(d[0])], ref[tuple(d[0])], flush=True)
        eng.close()
print('BAD' if bad else 'ALL EXACT', bad)
sys.exit(1 if bad else 0)
