"""Kernel-level timing sweep on the GPU (diagnostic tool, not the product)."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from esslivedata_amd import projection, synthetic
from esslivedata_amd.engine import BinningEngine

dev = torch.device('cuda', 0)
insts = {}


def run(workload, strategy, env, pulses=14, n_pulse=10_000_000, reps=5, check=None):
    for k, v in env.items():
        os.environ[k] = str(v)
    if workload not in insts:
        inst = synthetic.dream_mantle() if workload == 'dream' else synthetic.loki_bank0()
        view = projection.geometric_lut(inst.detector_number, inst.coords, inst.resolution)
        n = pulses * n_pulse
        if workload == 'dream':
            pid, toa = synthetic.torch_dream_events(n, inst, 7, dev)
        else:
            pid, toa = synthetic.torch_uniform_events(n, 1, 802816, 7, dev)
        insts[workload] = (inst, view, pid, toa)
    inst, view, pid, toa = insts[workload]
    eng = BinningEngine(toa_edges_ns=inst.edges.edges_ns(), out_lut=view.lut,
                        pid_offset=view.pid_offset, n_screen=view.n_screen, strategy=strategy,
                        stream=torch.cuda.current_stream().cuda_stream)

    def step(i):
        for p in range(pulses):
            eng.stage_tensors(pid[p * n_pulse:(p + 1) * n_pulse], toa[p * n_pulse:(p + 1) * n_pulse])
        eng.accumulate(i % view.n_replicas)
    step(0)
    ref = eng.read_histogram('current')
    eng.finalize(images=False)
    torch.cuda.synchronize()
    eng.timing_enable(True)
    t0 = time.perf_counter()
    for i in range(reps):
        step(i)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / reps
    st = {k: eng.kernel_stats(k) for k in ('atomic', 'partition', 'plan', 'tile_accumulate', 'paged', 'page_plan', 'page_accumulate', 'binning')}
    eng.close()
    for k in env:
        del os.environ[k]
    ev = pulses * n_pulse
    out = {'workload': workload, 'strategy': strategy, 'env': env, 'wall_ms': round(dt * 1e3, 4),
           'Gev_s': round(ev / dt / 1e9, 2), 'pipeline_frac': round(ev * 8 / dt / 8e12, 4)}
    out.update({k: round(v[0] / max(v[1], 1), 4) for k, v in st.items()})
    if check is not None:
        out['match'] = bool(np.array_equal(ref, check))
    print(json.dumps(out), flush=True)
    return ref


if __name__ == '__main__':
    mode = sys.argv[1] if len(sys.argv) > 1 else 'sweep'
    if mode == 'prof':  # one config for rocprof
        run(sys.argv[2] if len(sys.argv) > 2 else 'dream', 'partition', {}, reps=3)
        sys.exit(0)
    variants = [dict(LDE_TILE_BITS=13), dict(LDE_TILE_BITS=15), dict(LDE_SUBC=1)]
    ablations = []
    for wl in ('dream', 'loki'):
        base = run(wl, 'partition', {})
        for v in variants:
            run(wl, 'paged', v, check=base)
        run(wl, 'paged', {}, check=base)
        for v in ablations:
            run(wl, 'partition', v)
        run(wl, 'atomic', {}, reps=1, pulses=14, check=base)
    print('sweep done')
