"""B-sweep of the fused value-head scan (VTRACE target + UPGO adv): GB/s vs HBM peak."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from bench import time_scan, HBM_PEAK_GBS

from handyrl_amd import _native

dev = torch.device('cuda', 0)
lib = _native.load()
for T, forms in ((32, (1,)), (9, (1, 2, 0))):
    for form in forms:     # T <= 16: 1 the default choice, 2 the lane-per-column kernel, 0 the chunked kernel
        lib.hrl_targets_set_short_form(form)
        for B in (4096, 1 << 14, 1 << 16, 1 << 18, 1 << 20):
            cold = B >= (1 << 18)
            r = time_scan(dev, B, T, 50 if cold else 200, cold=cold)
            print('T=%3d B=%8d %-4s form %d %9.2f us  %8.1f GB/s  %5.1f%%' % (
                T, B, 'cold' if cold else 'hot', form, r['us_per_launch'], r['GBps'],
                100 * r['GBps'] / HBM_PEAK_GBS), flush=True)
lib.hrl_targets_set_short_form(1)

# launch floor: the same graph timing around a 1-element torch kernel
x = torch.zeros(1, device=dev)
g = torch.cuda.CUDAGraph()
x.add_(1)
torch.cuda.synchronize()
with torch.cuda.graph(g):
    for _ in range(200):
        x.add_(1)
g.replay()
torch.cuda.synchronize()
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
s.record(); g.replay(); e.record(); e.synchronize()
print('graph launch floor (1-element add): %.2f us' % (s.elapsed_time(e) * 1e3 / 200), flush=True)
