import sys, os
sys.path.insert(0, os.environ.get('GRAFT_REPO_ROOT', '/root/repo'))
import torch
from esslivedata_amd import projection, synthetic, wavelength
from esslivedata_amd.edges import WavelengthEdges
from esslivedata_amd.engine import BinningEngine
dev = torch.device('cuda', 0)
inst = synthetic.dream_mantle()
view = projection.geometric_lut(inst.detector_number, inst.coords, inst.resolution)
tab = synthetic.dream_wavelength_table()
lt = wavelength.pixel_ltotal(inst.positions, source_position=(0, 0, -synthetic.DREAM_L1))
d = wavelength.distance_per_pid(inst.detector_number, lt, view.pid_offset, view.lut.shape[1])
edges = WavelengthEdges(start=0.2, stop=3.6, num_bins=100).get_edges()
eng = BinningEngine(toa_edges_ns=edges, out_lut=view.lut, pid_offset=view.pid_offset, n_screen=view.n_screen)
eng.set_coordinate_lut(d, tab.table, dist0=tab.distance0, dist_step=tab.distance_step, time0=tab.time0, time_step=tab.time_step)
pid, toa = synthetic.torch_dream_events(14 * 10**7, inst, 7, dev)
msgs = [(pid[p*10**7:(p+1)*10**7], toa[p*10**7:(p+1)*10**7]) for p in range(14)]
for i in range(6):
    eng.timing_enable(True)
    eng.stage_tensors_batch(msgs); eng.accumulate(i % 5); eng.finalize(images=True)
    torch.cuda.synchronize()
    names = ('paged', 'page_plan', 'page_accumulate', 'split', 'split_aux', 'coord', 'binning')
    print(i, eng.info()['last_strategy'], {k: round(eng.kernel_stats(k)[0], 4) for k in names}, flush=True)
