"""Launch one hrl_gboard convolution back to back (for rocprofv3 --pmc passes) at the learner's per-step game
count: 'h' the DRC cells' grouped h halves (3 x 32 -> 128), 'adj' the K-split input gradient (4 x 32 -> 32,
nn.gboard_adjoint_split's grouped launch).

    python tools/gboard_pmc.py h|adj [--N 256] [--iters 20] [--whole 1]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from handyrl_amd import _native, nn as hnn  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('which', choices=['h', 'adj'])
    ap.add_argument('--N', type=int, default=256)
    ap.add_argument('--iters', type=int, default=20)
    ap.add_argument('--whole', type=int, default=1)
    ap.add_argument('--nctw', type=int, default=0)
    opts = ap.parse_args()
    dev = torch.device('cuda', 0)
    _native.load().hrl_gboard_set_whole_ring(opts.whole)
    _native.load().hrl_gboard_set_nctw(opts.nctw)
    g = torch.Generator(device=dev).manual_seed(1)
    N = opts.N
    if opts.which == 'h':
        x = torch.randn(N, 96, 6, 6, device=dev, generator=g)
        pk = hnn.gboard_pack(torch.randn(384, 32, 3, 3, device=dev, generator=g) * 0.1)
        y = torch.empty(N, 384, 6, 6, device=dev)
        launch = lambda: hnn.gboard_conv(x, pk, 384, 32, 3, out=y)   # noqa: E731
    else:
        dy = torch.randn(N, 128, 6, 6, device=dev, generator=g)
        w = torch.randn(128, 64, 3, 3, device=dev, generator=g) * 0.1
        pk = hnn.gboard_pack_adjoint_split(w, 32, 32)
        y = torch.empty(N, 128, 6, 6, device=dev)
        launch = lambda: hnn.gboard_conv(dy, pk, 128, 32, 4, out=y)   # noqa: E731
    for _ in range(opts.iters):
        launch()
    torch.cuda.synchronize(dev)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(opts.iters):
        launch()
    e.record()
    e.synchronize()
    print('%s N=%d whole=%d nctw=%d: %.2f us per launch' % (opts.which, N, opts.whole, opts.nctw, s.elapsed_time(e) * 1e3 / opts.iters))


if __name__ == '__main__':
    main()
