import os, numpy as np
from esslivedata_amd import projection, synthetic, _native
from esslivedata_amd.engine import BinningEngine
print('lib', _native.LIB_PATH)
inst = synthetic.dream_mantle()
view = projection.geometric_lut(inst.detector_number, inst.coords, inst.resolution)
pid, toa = synthetic.dream_events(3_000_000, inst, seed=3)
eng = BinningEngine(toa_edges_ns=inst.edges.edges_ns(), out_lut=view.lut, pid_offset=view.pid_offset, n_screen=view.n_screen, strategy='split', device=0)
eng.stage(pid, toa); eng.accumulate(0); r = eng.finalize(hists=True); print('ok', r.current_total)
