"""Time one chain block's backward: the fused hrl_conv3x3_block_backward (the default two-workgroup form 2, the
tile-shared form 1 and the per-wave form 0) vs the three launches it replaces.

    python tools/block_bench.py [--M 131072] [--iters 20]
HRL_LIB_PATH selects another build of libhrl.so (diagnostic variants).  HIP events on the launch stream.
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
    ap.add_argument('--iters', type=int, default=20)
    ap.add_argument('--epi', type=int, default=2, help='epilogue of the fused launch: 0, 2 (BN sums) or 3 (mask)')
    ap.add_argument('--forms', default='', help='only these block forms (comma list), e.g. 2,1')
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
    dw, gin, dy = torch.empty(32, 32, 3, 3, device=dev), torch.empty_like(g), torch.empty_like(g)

    def fused():
        _native.check(lib.hrl_conv3x3_block_backward(
            P(g), P(y), M, *[P(t) for t in c[:6]], P(x), P(c[6]), P(c[7]), P(packed[0, 1]), P(dw), P(gin),
            opts.epi, P(c[8]), P(c[9]), P(c[10]), P(part) if opts.epi == 2 else None, P(ws), ws_bytes, stream),
            'block')

    def three():
        _native.check(lib.hrl_bn_backward_apply(P(y), P(g), M, 32, 9, P(c[0]), P(c[1]), P(c[2]), P(c[3]), 1,
                                                P(c[4]), P(c[5]), P(dy), stream), 'apply')
        _native.check(lib.hrl_conv3x3_wgrad_ex(P(x), P(c[6]), P(c[7]), P(dy), M, P(dw), P(ws), ws_bytes, stream),
                      'wgrad')
        _native.check(lib.hrl_conv3x3_forward_ex(P(dy), M, None, None, P(packed[0, 1]), None, 3, P(gin), 2, P(x),
                                                 P(c[8]), P(c[9]), P(c[10]), P(part), P(ws), ws_bytes, stream),
                      'dgrad')

    out = {'M': M, 'lib': os.path.basename(_native.LIB_PATH), 'epi': opts.epi}
    only = {int(f) for f in opts.forms.split(',')} if opts.forms else None

    def form(f):
        def run():
            prev = lib.hrl_conv3x3_set_block_form(f)
            fused()
            lib.hrl_conv3x3_set_block_form(prev)
        return run
    cases = [('fused_two_wg_us', form(2), 2), ('fused_tile_shared_us', form(1), 1), ('fused_per_wave_us', form(0), 0),
             ('three_launches_us', three, None)]
    if only is None:
        cases = [('fused_us', fused, None)] + cases
    for name, fn, f in cases:
        if only is not None and f not in only:
            continue
        for _ in range(3):
            fn()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize(dev)
        s.record()
        for _ in range(opts.iters):
            fn()
        e.record()
        e.synchronize()
        out[name] = round(s.elapsed_time(e) * 1e3 / opts.iters, 2)
    print(json.dumps(out))


if __name__ == '__main__':
    main()
