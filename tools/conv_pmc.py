"""Launch one board-conv kernel form back to back (for rocprofv3 --pmc passes): the chain's forward conv
(hrl_conv3x3_forward_ex, epilogue 1, with prologue) or one chain block's backward (hrl_conv3x3_block_backward,
epilogue 2), M = 131,072 rows, random data.

    python tools/conv_pmc.py fwd|bwd FORM [--iters 10]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from handyrl_amd import _native  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('which', choices=['fwd', 'bwd'])
    ap.add_argument('form', type=int)
    ap.add_argument('--iters', type=int, default=10)
    ap.add_argument('--M', type=int, default=131072)
    opts = ap.parse_args()
    dev = torch.device('cuda', 0)
    lib = _native.load()
    P = _native.ptr
    stream = _native.stream_of(dev)
    M = opts.M
    g0 = torch.Generator(device=dev).manual_seed(1)
    rnd = lambda *s: torch.randn(*s, device=dev, generator=g0)   # noqa: E731
    g, y, x = rnd(M, 288), rnd(M, 288), rnd(M, 288)
    w = rnd(32, 32, 3, 3) * 0.1
    c = [rnd(32).abs() + 0.5 for _ in range(11)]
    packed = torch.empty(1, 2, 9216, device=dev)
    _native.check(lib.hrl_conv3x3_pack_n(_native.ptr_array([w]), 1, P(packed), stream), 'pack')
    ws_bytes = lib.hrl_conv3x3_workspace_bytes(M)
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
    part = torch.empty(max(lib.hrl_conv3x3_stats_blocks(M), lib.hrl_conv3x3_block_sum_blocks(M)) * 64,
                       dtype=torch.float64, device=dev)
    dw, out = torch.empty(32, 32, 3, 3, device=dev), torch.empty_like(g)
    if opts.which == 'fwd':
        lib.hrl_conv3x3_set_fwd_form(opts.form)

        def launch():
            _native.check(lib.hrl_conv3x3_forward_ex(P(x), M, P(c[0]), P(c[1]), P(packed[0, 0]), None, 2, P(out), 1,
                                                     None, None, None, None, P(part), P(ws), ws_bytes, stream), 'fwd')
    else:
        lib.hrl_conv3x3_set_block_form(opts.form)

        def launch():
            _native.check(lib.hrl_conv3x3_block_backward(
                P(g), P(y), M, *[P(t) for t in c[:6]], P(x), P(c[6]), P(c[7]), P(packed[0, 1]), P(dw), P(out), 2,
                P(c[8]), P(c[9]), P(c[10]), P(part), P(ws), ws_bytes, stream), 'block')
    for _ in range(opts.iters):
        launch()
    torch.cuda.synchronize(dev)


if __name__ == '__main__':
    main()
