"""Time the reference's own CPU learner step on the Geister net (this container only).

Imports handyrl from /root/reference (read-only, never shipped) and times
compute_loss + backward + clip_grad_norm_ + Adam exactly as
Trainer.train does it (train.py:357-401), on the synthetic Geister batch of
handyrl_amd.synthetic.geister_batch moved to the CPU.

    PYTHONDONTWRITEBYTECODE=1 python tools/ref_geister_cpu.py --B 64 --T 16 --threads 1 8
"""

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(1, '/root/reference')

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--B', type=int, default=64)
    ap.add_argument('--T', type=int, default=16)
    ap.add_argument('--threads', type=int, nargs='+', default=[1, 8])
    ap.add_argument('--steps', type=int, default=3)
    opts = ap.parse_args()

    from handyrl import train as ref_train
    from handyrl.envs.geister import GeisterNet
    from handyrl.model import ModelWrapper
    from handyrl_amd.synthetic import geister_batch, default_args

    B, T = opts.B, opts.T
    args = default_args(T, B)
    batch = geister_batch(B, T, torch.device('cpu'), seed=5)
    for th in opts.threads:
        torch.set_num_threads(th)
        torch.manual_seed(0)
        model = ModelWrapper(GeisterNet())
        opt = torch.optim.Adam(model.parameters(), lr=1e-5, weight_decay=1e-5)
        times = []
        for _ in range(opts.steps + 1):
            t0 = time.perf_counter()
            hidden = model.init_hidden([B, 2])
            losses, dcnt = ref_train.compute_loss(batch, model, hidden, args)
            opt.zero_grad()
            losses['total'].backward()
            torch.nn.utils.clip_grad_norm_(model.parameters(), 4.0)
            opt.step()
            times.append(time.perf_counter() - t0)
        dt = min(times[1:])
        print(json.dumps({'B': B, 'T': T, 'threads': th, 's_per_step': round(dt, 3),
                          'env_steps_per_s': round(B * T / dt, 1)}), flush=True)


if __name__ == '__main__':
    main()
