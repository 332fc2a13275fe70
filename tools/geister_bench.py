"""Time the recurrent (GeisterNet, config C3) learner step on the GPU.

    python tools/geister_bench.py --B 256 1024 --T 16 --graph 0 1

One step = forward_prediction unrolled over T (3 ConvLSTM cells x 3 repeats
per step) + compute_loss + backward + clip + Adam on a synthetic Geister
batch (handyrl_amd.synthetic.geister_batch), hidden state zero at the window
start (train.py:375).
"""

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from handyrl_amd.envs.geister import GeisterNet  # noqa: E402
from handyrl_amd.synthetic import geister_batch, default_args  # noqa: E402
from handyrl_amd.trainer import LearnerStep  # noqa: E402


def to_dev(h, device):
    return ([x.to(device) for x in h[0]], [x.to(device) for x in h[1]])


def run(B, T, graph, steps, warmup, device):
    args = default_args(T, B)
    torch.manual_seed(0)
    net = GeisterNet().to(device)
    batch = geister_batch(B, T, device, seed=5)
    hidden = to_dev(net.init_hidden([B, 2]), device)
    learner = LearnerStep(net, args, device, graph=bool(graph))
    for _ in range(warmup):
        learner.step(batch, hidden)
    torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    for _ in range(steps):
        learner.step(batch, hidden)
    torch.cuda.synchronize(device)
    dt = (time.perf_counter() - t0) / steps
    sums, n = learner.pop_stats()
    return {'B': B, 'T': T, 'graph': graph, 'ms_per_step': round(dt * 1e3, 3),
            'env_steps_per_s': round(B * T / dt, 1), 'loss_total_mean': sums.get('total', 0.0) / max(n, 1)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--B', type=int, nargs='+', default=[256, 1024])
    ap.add_argument('--T', type=int, nargs='+', default=[16])
    ap.add_argument('--graph', type=int, nargs='+', default=[0, 1])
    ap.add_argument('--steps', type=int, default=10)
    ap.add_argument('--warmup', type=int, default=3)
    ap.add_argument('--flat', type=int, nargs='+', default=[1], help='train.FLAT_HIDDEN values to compare')
    opts = ap.parse_args()
    device = torch.device('cuda', 0)
    if 'HRL_GBOARD_WHOLE' in os.environ:   # hrl_gboard's whole-k-step ring on (default) / off
        from handyrl_amd import _native
        _native.load().hrl_gboard_set_whole_ring(int(os.environ['HRL_GBOARD_WHOLE']))
    import handyrl_amd.train as train_mod
    for flat in opts.flat:
        train_mod.FLAT_HIDDEN = bool(flat)
        for T in opts.T:
            for B in opts.B:
                for g in opts.graph:
                    r = run(B, T, g, opts.steps, opts.warmup, device)
                    r['flat_hidden'] = flat
                    print(json.dumps(r), flush=True)


if __name__ == '__main__':
    main()
