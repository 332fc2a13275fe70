"""The heads backward (csrc/hrl_heads.hip heads_bwd2_kernel + its reduce) standalone at the bench size with the
body's last BN fused in front, as the step runs it: per-call microseconds from HIP events over --iters calls and the
HBM rate of the kernel's algorithmic bytes (h read and dh written, 151 MB each).  HRL_LIB_PATH selects another build.

    python tools/heads_bwd_bench.py [--n 131072] [--iters 50]
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
    r = lambda *s: torch.randn(*s, device=dev, generator=g)   # noqa: E731
    h = r(N, 32, 3, 3)
    w1p, w1v, wp, wv = r(2, 32), r(1, 32), r(9, 18), r(1, 9)
    al, be, mu = torch.rand(32, device=dev, generator=g) + 0.5, r(32) * 0.1, r(32) * 0.1
    a_p, a_v, dp, dv, vt = r(N, 18), r(N, 9), r(N, 9), r(N, 1), torch.tanh(r(N, 1))
    dh = torch.empty_like(h)
    dws = [torch.empty(2, 32, device=dev), torch.empty(2, device=dev), torch.empty(1, 32, device=dev),
           torch.empty(1, device=dev), torch.empty(9, 18, device=dev), torch.empty(1, 9, device=dev)]
    part = torch.empty(lib.hrl_heads_bn_parts(N) * 64, dtype=torch.float64, device=dev)
    ws_bytes = lib.hrl_heads_workspace_bytes(N)
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
    stream = _native.stream_of(dev)

    def launch():
        _native.check(lib.hrl_heads_backward(P(h), N, P(w1p), P(w1v), P(wp), P(wv), P(al), P(be), P(mu), P(part),
                                             P(a_p), P(a_v), P(dp), P(dv), P(vt), P(dh), *(P(t) for t in dws),
                                             P(ws), ws_bytes, stream), 'hrl_heads_backward')

    for _ in range(3):
        launch()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(o.iters):
        launch()
    b.record()
    torch.cuda.synchronize()
    us = a.elapsed_time(b) / o.iters * 1e3
    byt = 2 * h.numel() * 4
    print(json.dumps({'N': N, 'lib': os.path.basename(_native.LIB_PATH), 'us': round(us, 2),
                      'TBps': round(byt / us / 1e6, 2), 'dh_sum': float(dh.double().sum()),
                      'part_sum': float(part.sum())}))


if __name__ == '__main__':
    main()
