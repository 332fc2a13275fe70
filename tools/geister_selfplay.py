"""Geister self-play training on one GPU: device rollout -> HBM replay -> recurrent learner.

    python tools/geister_selfplay.py --rounds 3 --games 2048 --steps 20
Prints per-round losses and timings, then the generation / learner split.
"""

import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from handyrl_amd.envs.geister import GeisterNet, GeisterBatch  # noqa: E402
from handyrl_amd.loop import SelfPlayTrainer  # noqa: E402
from handyrl_amd.synthetic import default_args  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--rounds', type=int, default=3)
    ap.add_argument('--games', type=int, default=2048)
    ap.add_argument('--steps', type=int, default=20)
    ap.add_argument('--batch', type=int, default=256)
    ap.add_argument('--seq', type=int, default=16)
    ap.add_argument('--graph', type=int, default=1)
    opts = ap.parse_args()
    dev = torch.device('cuda', 0)
    torch.manual_seed(0)
    net = GeisterNet().to(dev)
    args = default_args(opts.seq, opts.batch)
    tr = SelfPlayTrainer(net, args, dev, games_per_round=opts.games, capacity=8 * opts.games,
                         graph=bool(opts.graph), env_cls=GeisterBatch)
    tg = tl = 0.0
    for r in range(opts.rounds):
        t0 = time.perf_counter()
        ep = tr.generate()
        torch.cuda.synchronize(dev)
        t1 = time.perf_counter()
        tr.train_steps(opts.steps)
        torch.cuda.synchronize(dev)
        t2 = time.perf_counter()
        sums, n = tr.learner.pop_stats()
        dcnt = max(sums.get('dcnt', 1.0), 1e-9)
        oc = ep['outcome'][:, 0]
        print('round %d: %d games, mean plies %.1f, black win %.3f draw %.3f | gen %.2fs learn %.2fs | %s' % (
            r, opts.games, float(ep['length'].float().mean()), float((oc > 0).float().mean()),
            float((oc == 0).float().mean()), t1 - t0, t2 - t1,
            ' '.join('%s:%.4f' % (k, sums[k] / dcnt) for k in ('p', 'v', 'r', 'ent') if k in sums)), flush=True)
        if r:
            tg += t1 - t0
            tl += t2 - t1
    print('steady state: generation %.2fs/round, learner %.1f ms/step' % (
        tg / max(opts.rounds - 1, 1), 1e3 * tl / max((opts.rounds - 1) * opts.steps, 1)))


if __name__ == '__main__':
    main()
