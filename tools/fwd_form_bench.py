"""The learner step (bench.py's workload: TicTacToe net, B=4096 T=32, HIP graph) with the chain's forward conv in
each form (hrl_conv3x3_set_fwd_form: 0 per-wave conv3x3_kernel, 1 the tile-shared block-backward form).

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
    opts = ap.parse_args()
    dev = torch.device('cuda', 0)
    lib = _native.load()
    B, T = 4096, 32
    for form in (0, 1, 0, 1):
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


if __name__ == '__main__':
    main()
