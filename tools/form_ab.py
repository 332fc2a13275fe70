"""The learner step (bench.py's workload: TicTacToe net, B=4096 T=32, HIP graph) under each setting of one
process-wide kernel-form switch of libhrl.so, alternating, so the forms are compared on the same box in one run.

    python tools/form_ab.py --setter hrl_heads_set_bwd_form --forms 1,2,1,2 [--steps 20]
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
    ap.add_argument('--setter', required=True)
    ap.add_argument('--forms', default='1,2,1,2')
    ap.add_argument('--steps', type=int, default=50)
    ap.add_argument('--warmup', type=int, default=30)
    ap.add_argument('--seq', type=int, default=32)
    opts = ap.parse_args()
    dev = torch.device('cuda', 0)
    lib = _native.load()
    setter = getattr(lib, opts.setter)
    B, T = 4096, opts.seq
    for form in [int(f) for f in opts.forms.split(',')]:
        prev = setter(form)
        torch.manual_seed(0)
        net = SimpleConv2dModel().to(dev)
        batch = tictactoe_batch(B, T, dev, seed=1000)
        learner = LearnerStep(net, default_args(T, B), dev, graph=True)
        for _ in range(opts.warmup):   # past the first graph replays, which run slow while the clocks settle
            learner.step(batch)
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(opts.steps):
            out = learner.step(batch)
        torch.cuda.synchronize(dev)
        ms = (time.perf_counter() - t0) / opts.steps * 1e3
        setter(prev)
        print(json.dumps({'setter': opts.setter, 'form': form, 'T': T, 'ms_per_step': round(ms, 4),
                          'env_steps_per_s': round(B * T / ms * 1e3), 'loss_total': float(out['total'])}),
              flush=True)
        del learner, net, batch
        torch.cuda.empty_cache()


if __name__ == '__main__':
    main()
