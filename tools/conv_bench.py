"""Time the 3x3-board MFMA conv kernels (csrc/hrl_conv.hip) at the headline shape.

    python tools/conv_bench.py --M 131072 --iters 50
M = B*T*Pp rows of 32x3x3 NCHW activations (headline: 4096*32).  Prints
microseconds per launch (HIP events on the launch stream) and the achieved
fp32 MFMA rate on the algorithmic FLOPs (49 on-board 32x32 tap blocks per
sample, 2 FLOP per MAC).
"""

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from handyrl_amd import _native  # noqa: E402

PEAK_TFLOPS = 157.3   # MI355X dense fp32 MFMA


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--M', type=int, default=131072)
    ap.add_argument('--iters', type=int, default=50)
    ap.add_argument('--split', type=int, default=1, help='forward/input-gradient arithmetic: 1 split-bf16, 0 fp32 MFMA')
    opts = ap.parse_args()
    dev = torch.device('cuda', 0)
    lib = _native.load()
    lib.hrl_conv3x3_set_split(opts.split)
    M = opts.M
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(M, 288, device=dev, generator=g)
    dy = torch.randn(M, 288, device=dev, generator=g)
    w = torch.randn(32, 32, 3, 3, device=dev, generator=g) * 0.1
    b = torch.randn(32, device=dev, generator=g)
    y = torch.empty_like(x)
    dw = torch.empty_like(w)
    ws_bytes = lib.hrl_conv3x3_workspace_bytes(M)
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
    stream = _native.stream_of(dev)
    P = _native.ptr
    flops = 2.0 * M * 49 * 32 * 32

    def fwd():
        _native.check(lib.hrl_conv3x3_forward(P(x), M, 32, 32, P(w), P(b), 0, P(y), P(ws), ws_bytes, stream), 'fwd')

    def dgrad():
        _native.check(lib.hrl_conv3x3_forward(P(dy), M, 32, 32, P(w), None, 1, P(y), P(ws), ws_bytes, stream),
                      'dgrad')

    def wgrad():
        _native.check(lib.hrl_conv3x3_wgrad(P(x), P(dy), M, 32, 32, P(dw), P(ws), ws_bytes, stream), 'wgrad')

    # fused variants (conv -> BN -> ReLU chains, nn._BoardChain)
    nblk = lib.hrl_conv3x3_stats_blocks(M)
    part = torch.empty(nblk * 64, dtype=torch.float64, device=dev)
    al = torch.rand(32, device=dev) + 0.5
    be = torch.randn(32, device=dev) * 0.1
    mu = torch.randn(32, device=dev) * 0.1
    ref = torch.randn(M, 288, device=dev, generator=g)

    def fwd_pro_stats():
        _native.check(lib.hrl_conv3x3_forward_ex(P(x), M, P(al), P(be), P(w), None, 0, P(y), 1, None, None, None,
                                                 None, P(part), P(ws), ws_bytes, stream), 'fwd_pro_stats')

    def dgrad_bnred():
        _native.check(lib.hrl_conv3x3_forward_ex(P(dy), M, None, None, P(w), None, 1, P(y), 2, P(ref), P(mu), P(al),
                                                 P(be), P(part), P(ws), ws_bytes, stream), 'dgrad_bnred')

    def dgrad_mask():
        _native.check(lib.hrl_conv3x3_forward_ex(P(dy), M, None, None, P(w), None, 1, P(y), 3, P(ref), None, None,
                                                 None, None, P(ws), ws_bytes, stream), 'dgrad_mask')

    def wgrad_pro():
        _native.check(lib.hrl_conv3x3_wgrad_ex(P(x), P(al), P(be), P(dy), M, P(dw), P(ws), ws_bytes, stream),
                      'wgrad_pro')

    # correctness spot check against torch (fp32)
    fwd()
    ref = torch.nn.functional.conv2d(x.view(M, 32, 3, 3), w, b, padding=1).view(M, 288)
    err = float((y - ref).abs().max())
    # error against an fp64 reference, beside torch's own fp32 conv
    r64 = torch.nn.functional.conv2d(x.view(M, 32, 3, 3).double(), w.double(), b.double(), padding=1).view(M, 288)
    scale = float(r64.abs().max())
    res = {'M': M, 'split': opts.split, 'fwd_max_abs_err_vs_torch32': err,
           'fwd_max_err_vs_fp64_rel_to_max': float((y.double() - r64).abs().max()) / scale,
           'torch32_max_err_vs_fp64_rel_to_max': float((ref.double() - r64).abs().max()) / scale,
           'fwd_rms_rel_err_vs_fp64': float(((y.double() - r64).norm() / r64.norm())),
           'torch32_rms_rel_err_vs_fp64': float(((ref.double() - r64).norm() / r64.norm()))}
    dgrad()
    d64 = torch.nn.grad.conv2d_input((M, 32, 3, 3), w.double(), dy.view(M, 32, 3, 3).double(), padding=1).view(M, 288)
    res['dgrad_max_err_vs_fp64_rel_to_max'] = float((y.double() - d64).abs().max()) / float(d64.abs().max())
    for name, fn in (('fwd', fwd), ('dgrad', dgrad), ('wgrad', wgrad), ('fwd_pro_stats', fwd_pro_stats),
                     ('dgrad_bnred', dgrad_bnred), ('dgrad_mask', dgrad_mask), ('wgrad_pro', wgrad_pro),
                     ('fwd_again', fwd)):
        for _ in range(3):
            fn()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize(dev)
        s.record()
        for _ in range(opts.iters):
            fn()
        e.record()
        torch.cuda.synchronize(dev)
        us = s.elapsed_time(e) * 1e3 / opts.iters
        res[name + '_us'] = round(us, 2)
        res[name + '_tflops'] = round(flops / us / 1e6, 1)
        res[name + '_frac'] = round(flops / us / 1e6 / PEAK_TFLOPS, 3)
    print(json.dumps(res), flush=True)


if __name__ == '__main__':
    main()
