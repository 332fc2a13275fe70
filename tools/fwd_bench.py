"""Time the chain's forward conv (hrl_conv3x3_forward_ex, epilogue 1, BN+ReLU prologue, packed weights) per fwd form,
M = 131,072 rows of random data, HIP events on the launch stream.  HRL_LIB_PATH selects a diagnostic build.

    python tools/fwd_bench.py [--forms 2,1,0] [--iters 50]
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
    ap.add_argument('--M', type=int, default=131072)
    ap.add_argument('--iters', type=int, default=50)
    ap.add_argument('--forms', default='2')
    opts = ap.parse_args()
    dev = torch.device('cuda', 0)
    lib = _native.load()
    P = _native.ptr
    stream = _native.stream_of(dev)
    M = opts.M
    g0 = torch.Generator(device=dev).manual_seed(1)
    x = torch.randn(M, 288, device=dev, generator=g0)
    w = torch.randn(32, 32, 3, 3, device=dev, generator=g0) * 0.1
    a, b = torch.rand(32, device=dev, generator=g0) + 0.5, torch.randn(32, device=dev, generator=g0) * 0.2
    packed = torch.empty(1, 2, 9216, device=dev)
    _native.check(lib.hrl_conv3x3_pack_n(_native.ptr_array([w]), 1, P(packed), stream), 'pack')
    ws_bytes = lib.hrl_conv3x3_workspace_bytes(M)
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
    part = torch.empty(lib.hrl_conv3x3_stats_blocks(M) * 64, dtype=torch.float64, device=dev)
    y = torch.empty_like(x)
    out = {'M': M, 'lib': os.path.basename(_native.LIB_PATH)}
    for f in [int(v) for v in opts.forms.split(',')]:
        prev = lib.hrl_conv3x3_set_fwd_form(f)

        def launch():
            _native.check(lib.hrl_conv3x3_forward_ex(P(x), M, P(a), P(b), P(packed[0, 0]), None, 2, P(y), 1, None,
                                                     None, None, None, P(part), P(ws), ws_bytes, stream), 'fwd')
        for _ in range(3):
            launch()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize(dev)
        s.record()
        for _ in range(opts.iters):
            launch()
        e.record()
        e.synchronize()
        out['fwd_form%d_us' % f] = round(s.elapsed_time(e) * 1e3 / opts.iters, 2)
        lib.hrl_conv3x3_set_fwd_form(prev)
    print(json.dumps(out))


if __name__ == '__main__':
    main()
