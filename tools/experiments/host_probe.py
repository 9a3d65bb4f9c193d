"""Host-side cost of one bench step (diagnostic): wall time of the staging
calls, accumulate and finalize, with and without kernel timing events."""
import sys, time
from pathlib import Path
sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch
from esslivedata_amd import projection, synthetic
from esslivedata_amd.engine import BinningEngine

dev = torch.device('cuda', 0)
torch.cuda.set_stream(torch.cuda.Stream(dev))  # as bench.py
inst = synthetic.dream_mantle()
view = projection.geometric_lut(inst.detector_number, inst.coords, inst.resolution)
eng = BinningEngine(toa_edges_ns=inst.edges.edges_ns(), out_lut=view.lut, pid_offset=view.pid_offset,
                    n_screen=view.n_screen, strategy='auto', device=0,
                    stream=torch.cuda.current_stream(dev).cuda_stream)
n_pulse, pulses = 10_000_000, 14
pid, toa = synthetic.torch_dream_events(n_pulse * pulses, inst, 7, dev)
msgs = [(pid[p * n_pulse:(p + 1) * n_pulse], toa[p * n_pulse:(p + 1) * n_pulse]) for p in range(pulses)]
torch.cuda.synchronize()
import os
for timing in (False, True):
    eng.timing_enable(timing)
    acc = {'stage': 0.0, 'accumulate': 0.0, 'finalize': 0.0}
    for i in range(25):
        t0 = time.perf_counter()
        eng.stage_tensors_batch(msgs)
        t1 = time.perf_counter()
        eng.accumulate(i % view.n_replicas)
        t2 = time.perf_counter()
        eng.finalize(images=True)
        t3 = time.perf_counter()
        if i >= 5:
            acc['stage'] += t1 - t0
            acc['accumulate'] += t2 - t1
            acc['finalize'] += t3 - t2
    print('timing' if timing else 'no timing', {k: round(v / 20 * 1e3, 4) for k, v in acc.items()},
          'ms/step total', round(sum(acc.values()) / 20 * 1e3, 4), flush=True)

# GPU-side span of one step (events around the whole step on the engine stream)
eng.timing_enable(False)
s0 = torch.cuda.Event(enable_timing=True); s1 = torch.cuda.Event(enable_timing=True)
tot = 0.0
for i in range(20):
    s0.record()
    torch.cuda._sleep(2_000_000)  # the GPU is busy while the host enqueues the step
    eng.stage_tensors_batch(msgs)
    eng.accumulate(i % view.n_replicas)
    eng.finalize(images=True)
    s1.record()
    s1.synchronize()
    tot += s0.elapsed_time(s1)
tot_sleep = 0.0
for i in range(20):
    s0.record()
    torch.cuda._sleep(2_000_000)
    s1.record()
    s1.synchronize()
    tot_sleep += s0.elapsed_time(s1)
print('gpu span per step (ms), host enqueue hidden behind a sleep:', round((tot - tot_sleep) / 20, 4))

# host cost of the staging call alone, split
import numpy as np
t0 = time.perf_counter()
for _ in range(200):
    rows = [(p.data_ptr(), t.data_ptr(), t.numel()) for p, t in msgs]
t1 = time.perf_counter()
for _ in range(200):
    for p, t in msgs:
        (t.dtype is torch.int32, t.is_contiguous(), t.is_cuda)
t2 = time.perf_counter()
print('data_ptr rows us', round((t1 - t0) / 200 * 1e6, 2), 'checks us', round((t2 - t1) / 200 * 1e6, 2))

# finalize alone with the GPU idle: launch + kernels + D2H + wait + host copies
tf = []
for i in range(20):
    eng.stage_tensors_batch(msgs)
    eng.accumulate(i % view.n_replicas)
    eng.synchronize()
    t0 = time.perf_counter()
    eng.finalize(images=True)
    tf.append(time.perf_counter() - t0)
print('finalize with idle GPU (us): median', round(sorted(tf)[10] * 1e6, 1), 'min', round(min(tf) * 1e6, 1))
import ctypes
buf = np.empty(25600 * 2, dtype=np.float64)
src = np.ones(25600 * 2, dtype=np.float64)
t0 = time.perf_counter()
for _ in range(200):
    np.copyto(buf, src)
print('host copy of 410 KB (us):', round((time.perf_counter() - t0) / 200 * 1e6, 2))

# python-side cost of the finalize wrapper around the C call (GPU idle)
import ctypes
from esslivedata_amd import _native
tw = []
for i in range(20):
    eng.stage_tensors_batch(msgs)
    eng.accumulate(i % view.n_replicas)
    eng.synchronize()
    out = _native.LdeOutputs()
    a1 = np.empty(view.n_screen); a2 = np.empty(view.n_screen)
    out.current_image = a1.ctypes.data; out.cumulative_image = a2.ctypes.data
    t0 = time.perf_counter()
    eng._lib.lde_finalize(eng._h, ctypes.byref(out))
    t1 = time.perf_counter()
    tw.append(t1 - t0)
print('raw lde_finalize with idle GPU (us): median', round(sorted(tw)[10] * 1e6, 1))
del eng
