# round 5: where torch puts the bench's event arrays (pointer distances)
import torch
from esslivedata_amd import synthetic
inst = synthetic.dream_mantle()
dev = torch.device('cuda', 0)
keep = []
for b in range(3):
    pid, toa = synthetic.torch_dream_events(140_000_000, inst, 7 + 17 * b, dev)
    keep.append((pid, toa))
    print('batch', b, hex(pid.data_ptr()), hex(toa.data_ptr()), 'diff', toa.data_ptr() - pid.data_ptr())
