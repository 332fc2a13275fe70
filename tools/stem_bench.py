"""The stem forward (csrc/hrl_stem.hip) standalone at the bench size, each form, beside torch writing the same
bytes (fill) and copying them (copy_): per-launch microseconds from HIP events over --iters launches.

    python tools/stem_bench.py [--n 131072] [--iters 50]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from handyrl_amd import _native  # noqa: E402


def timed(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--n', type=int, default=131072)
    ap.add_argument('--iters', type=int, default=50)
    o = ap.parse_args()
    dev = torch.device('cuda', 0)
    lib = _native.load()
    P = _native.ptr
    N = o.n
    x = (torch.rand(N, 3, 3, 3, device=dev) < 0.5).float()
    w = torch.randn(32, 3, 3, 3, device=dev)
    b = torch.randn(32, device=dev)
    y = torch.empty(N, 32, 3, 3, device=dev)
    y2 = torch.empty_like(y)
    stream = _native.stream_of(dev)
    res = {'N': N, 'bytes_out': y.numel() * 4}
    for form in (1, 2):
        prev = lib.hrl_stem_set_fwd_form(form)
        res['form%d_us' % form] = round(timed(lambda: _native.check(
            lib.hrl_stem_forward(P(x), N, 3, P(w), P(b), P(y), stream), 'stem'), o.iters), 2)
        lib.hrl_stem_set_fwd_form(prev)
    res['torch_fill_us'] = round(timed(lambda: y2.fill_(0.5), o.iters), 2)
    res['torch_copy_us'] = round(timed(lambda: y2.copy_(y), o.iters), 2)
    for k in ('form1_us', 'form2_us', 'torch_fill_us'):
        res[k.replace('_us', '_TBps')] = round(res['bytes_out'] / res[k] / 1e6, 2)
    print(json.dumps(res))


if __name__ == '__main__':
    main()
