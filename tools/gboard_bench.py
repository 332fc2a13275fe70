"""Time GeisterNet's self-play convolutions (E games, 6x6 board) on csrc/hrl_gboard.hip against F.conv2d
(the vendor convolution the inference forward used before).

    python tools/gboard_bench.py [--E 2048] [--iters 20]
HIP events on the current stream; one JSON line per shape.
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from handyrl_amd import nn as hnn  # noqa: E402


def timed(fn, iters):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) * 1e3 / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--E', type=int, default=2048)
    ap.add_argument('--iters', type=int, default=20)
    opts = ap.parse_args()
    dev = torch.device('cuda', 0)
    E = opts.E
    for name, cin, cout, groups in (('stem', 25, 32, 1), ('x_halves', 32, 384, 1), ('h_halves', 32, 384, 3),
                                    ('move_head', 64, 8, 1)):
        x = torch.randn(E, cin * groups, 6, 6, device=dev)
        w = torch.randn(cout, cin, 3, 3, device=dev) * 0.1
        pk = hnn.gboard_pack(w)
        y = torch.empty(E, cout, 6, 6, device=dev)
        t_hip = timed(lambda: hnn.gboard_conv(x, pk, cout, cin, groups, out=y), opts.iters)
        t_ref = timed(lambda: F.conv2d(x, w, None, padding=1, groups=groups), opts.iters)
        flop = 2.0 * E * 256 * cin * cout   # 256 real (cell, tap) pairs of the 6x6 board
        err = (y - F.conv2d(x, w, None, padding=1, groups=groups)).abs().max().item()
        print(json.dumps({'conv': name, 'E': E, 'gboard_us': round(t_hip, 2), 'F_conv2d_us': round(t_ref, 2),
                          'gboard_tflops': round(flop / t_hip / 1e6, 1), 'max_abs_diff': err}))


if __name__ == '__main__':
    main()
