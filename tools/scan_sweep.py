"""B-sweep of the fused value-head scan (VTRACE target + UPGO adv): GB/s vs HBM peak."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from bench import time_scan, HBM_PEAK_GBS

dev = torch.device('cuda', 0)
for T in (32, 9):
    for B in (4096, 1 << 14, 1 << 16, 1 << 18, 1 << 20):
        cold = B >= (1 << 18)
        r = time_scan(dev, B, T, 50 if cold else 200, cold=cold)
        print('T=%3d B=%8d %-4s %9.2f us  %8.1f GB/s  %5.1f%%' % (T, B, 'cold' if cold else 'hot', r['us_per_launch'],
              r['GBps'], 100 * r['GBps'] / HBM_PEAK_GBS), flush=True)
