"""Time one scan configuration (for rocprofv3 kernel-trace runs): python tools/scan_one.py B T [iters] [cold]."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from bench import time_scan, HBM_PEAK_GBS

B, T = int(sys.argv[1]), int(sys.argv[2])
iters = int(sys.argv[3]) if len(sys.argv) > 3 else 200
cold = len(sys.argv) > 4 and sys.argv[4] == 'cold'
r = time_scan(torch.device('cuda', 0), B, T, iters, cold=cold)
print('T=%d B=%d %s %.2f us %.1f GB/s %.1f%%' % (T, B, 'cold' if cold else 'hot', r['us_per_launch'], r['GBps'],
      100 * r['GBps'] / HBM_PEAK_GBS), flush=True)
