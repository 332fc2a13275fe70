"""The learner step (bench.py's workload: TicTacToe net, B=4096 T=32, HIP graph) with the chain's forward conv in
each form (hrl_conv3x3_set_fwd_form: 0 per-wave conv3x3_kernel, 1 the tile-shared block-backward form, 2 the
LDS-DMA ring form), then each form's kernel alone (HIP events over back-to-back launches at M = B*T).

    python tools/fwd_form_bench.py [--steps 20]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from handyrl_amd import _native  # noqa: E402
from handyrl_amd.envs.tictactoe import SimpleConv2dModel  # noqa: E402
from handyrl_amd.synthetic import default_args, tictactoe_batch  # noqa: E402
from handyrl_amd.trainer import LearnerStep  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--steps', type=int, default=20)
    ap.add_argument('--forms', default='1,2,1,2')
    opts = ap.parse_args()
    dev = torch.device('cuda', 0)
    lib = _native.load()
    B, T = 4096, 32
    forms = [int(f) for f in opts.forms.split(',')]
    for form in forms:
        prev = lib.hrl_conv3x3_set_fwd_form(form)
        torch.manual_seed(0)
        net = SimpleConv2dModel().to(dev)
        batch = tictactoe_batch(B, T, dev, seed=1000)
        learner = LearnerStep(net, default_args(T, B), dev, graph=True)
        for _ in range(5):
            learner.step(batch)
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(opts.steps):
            out = learner.step(batch)
        torch.cuda.synchronize(dev)
        ms = (time.perf_counter() - t0) / opts.steps * 1e3
        lib.hrl_conv3x3_set_fwd_form(prev)
        print(json.dumps({'fwd_form': form, 'ms_per_step': round(ms, 4), 'env_steps_per_s': round(B * T / ms * 1e3),
                          'loss_total': float(out['total'])}), flush=True)
    # the kernel alone: M = B*T rows, with the BN + ReLU prologue, 20 back-to-back launches
    P = _native.ptr
    stream = _native.stream_of(dev)
    M = B * T
    g0 = torch.Generator(device=dev).manual_seed(5)
    x = torch.randn(M, 288, device=dev, generator=g0)
    w = torch.randn(32, 32, 3, 3, device=dev, generator=g0) * 0.1
    alpha, beta = torch.rand(32, device=dev, generator=g0) + 0.5, torch.randn(32, device=dev, generator=g0) * 0.3
    packed = torch.empty(1, 2, 9216, device=dev)
    _native.check(lib.hrl_conv3x3_pack_n(_native.ptr_array([w]), 1, P(packed), stream), 'pack')
    ws_bytes = lib.hrl_conv3x3_workspace_bytes(M)
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
    part = torch.empty(lib.hrl_conv3x3_stats_blocks(M) * 64, dtype=torch.float64, device=dev)
    y = torch.empty_like(x)
    for form in sorted(set(forms)):
        prev = lib.hrl_conv3x3_set_fwd_form(form)

        def launch():
            _native.check(lib.hrl_conv3x3_forward_ex(P(x), M, P(alpha), P(beta), P(packed[0, 0]), None, 2, P(y), 1,
                                                     None, None, None, None, P(part), P(ws), ws_bytes, stream), 'fwd')
        for _ in range(3):
            launch()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize(dev)
        s.record()
        for _ in range(20):
            launch()
        e.record()
        e.synchronize()
        lib.hrl_conv3x3_set_fwd_form(prev)
        us = s.elapsed_time(e) * 1e3 / 20
        print(json.dumps({'fwd_form': form, 'kernel_us': round(us, 2), 'M': M,
                          'hbm_frac': round(2 * M * 288 * 4 / (us * 1e-6) / 8e12, 4)}), flush=True)


if __name__ == '__main__':
    main()
