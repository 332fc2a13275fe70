"""The learner step (bench.py's workload: TicTacToe net, B=4096 T=32, HIP graph) with the chain's BatchNorm finalizes
as launches of their own (nn.FOLD_BN = False) and folded into their consumers' prologues (True), alternating in one
process so both run on the same clocks; the loss of the last step is printed to show the two are bit-identical.

    python tools/fold_bench.py [--steps 40] [--rounds 3] [--fwd-form 2]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from handyrl_amd import _native, nn as hnn  # noqa: E402
from handyrl_amd.envs.tictactoe import SimpleConv2dModel  # noqa: E402
from handyrl_amd.synthetic import default_args, tictactoe_batch  # noqa: E402
from handyrl_amd.trainer import LearnerStep  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--steps', type=int, default=40)
    ap.add_argument('--rounds', type=int, default=3)
    ap.add_argument('--fwd-form', type=int, default=2)
    opts = ap.parse_args()
    dev = torch.device('cuda', 0)
    lib = _native.load()
    lib.hrl_conv3x3_set_fwd_form(opts.fwd_form)
    B, T = 4096, 32
    for r in range(opts.rounds):
        for fold in (False, True):
            hnn.FOLD_BN = fold
            torch.manual_seed(0)
            net = SimpleConv2dModel().to(dev)
            batch = tictactoe_batch(B, T, dev, seed=1000)
            learner = LearnerStep(net, default_args(T, B), dev, graph=True)
            for _ in range(20):
                out = learner.step(batch)
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            for _ in range(opts.steps):
                out = learner.step(batch)
            torch.cuda.synchronize(dev)
            ms = (time.perf_counter() - t0) / opts.steps * 1e3
            print(json.dumps({'round': r, 'fold_bn': fold, 'fwd_form': opts.fwd_form, 'ms_per_step': round(ms, 4),
                              'env_steps_per_s': round(B * T / ms * 1e3), 'loss_total': float(out['total'])}),
                  flush=True)


if __name__ == '__main__':
    main()
