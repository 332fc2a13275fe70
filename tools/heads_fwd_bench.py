"""The heads forward (csrc/hrl_heads.hip heads_fwd_kernel) standalone at the bench size with the body's last BN
fused in front, as the step runs it: per-launch microseconds from HIP events over --iters launches, and the HBM
rate of its algorithmic bytes (151 MB of h read, 19 MB of activations and outputs written).  Run it under
`rocprofv3 --pmc FETCH_SIZE` to compare the fetched bytes with the algorithmic ones.

    python tools/heads_fwd_bench.py [--n 131072] [--iters 50]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from handyrl_amd import _native  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--n', type=int, default=131072)
    ap.add_argument('--iters', type=int, default=50)
    o = ap.parse_args()
    dev = torch.device('cuda', 0)
    lib = _native.load()
    P = _native.ptr
    N = o.n
    g = torch.Generator(device=dev).manual_seed(0)
    h = torch.randn(N, 32, 3, 3, device=dev, generator=g)
    w1p, b1p = torch.randn(2, 32, device=dev, generator=g), torch.randn(2, device=dev, generator=g)
    w1v, b1v = torch.randn(1, 32, device=dev, generator=g), torch.randn(1, device=dev, generator=g)
    wp, wv = torch.randn(9, 18, device=dev, generator=g), torch.randn(1, 9, device=dev, generator=g)
    al, be = torch.rand(32, device=dev, generator=g) + 0.5, torch.randn(32, device=dev, generator=g) * 0.1
    a_p, a_v = torch.empty(N, 18, device=dev), torch.empty(N, 9, device=dev)
    p_out, v_out = torch.empty(N, 9, device=dev), torch.empty(N, 1, device=dev)
    stream = _native.stream_of(dev)

    def launch():
        _native.check(lib.hrl_heads_forward(P(h), N, P(w1p), P(b1p), P(w1v), P(b1v), P(wp), P(wv), P(al), P(be),
                                            P(a_p), P(a_v), P(p_out), P(v_out), 1, stream), 'hrl_heads_forward')

    def timed():
        for _ in range(3):
            launch()
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(o.iters):
            launch()
        b.record()
        torch.cuda.synchronize()
        return a.elapsed_time(b) / o.iters * 1e3

    rd, wr = h.numel() * 4, (a_p.numel() + a_v.numel() + p_out.numel() + v_out.numel()) * 4
    us = timed()
    print(json.dumps({'N': N, 'us': round(us, 2), 'read_bytes': rd, 'write_bytes': wr,
                      'TBps': round((rd + wr) / us / 1e6, 2)}))


if __name__ == '__main__':
    main()
