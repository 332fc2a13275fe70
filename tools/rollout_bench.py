"""Wall time per self-play ply vs GPU kernel time (Geister or TicTacToe device rollout).

    python tools/rollout_bench.py --env geister --games 2048 --reps 2
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from handyrl_amd.nn import accelerate  # noqa: E402
from handyrl_amd.rollout import DeviceGenerator, TicTacToeBatch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--env', default='geister')
    ap.add_argument('--games', type=int, default=2048)
    ap.add_argument('--reps', type=int, default=2)
    ap.add_argument('--graph', type=int, default=1, help='1: one HIP graph per ply (default), 0: eager plies')
    opts = ap.parse_args()
    dev = torch.device('cuda', 0)
    torch.manual_seed(0)
    if opts.env == 'geister':
        from handyrl_amd.envs.geister import GeisterNet, GeisterBatch
        net, env = accelerate(GeisterNet().to(dev)), GeisterBatch(opts.games, dev)
    else:
        from handyrl_amd.envs.tictactoe import SimpleConv2dModel
        net, env = accelerate(SimpleConv2dModel().to(dev)), TicTacToeBatch(opts.games, dev)
    gen = DeviceGenerator(env, net, graph=bool(opts.graph))
    g = torch.Generator(device=dev).manual_seed(0)
    gen.generate(generator=g)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    plies = loops = 0
    for _ in range(opts.reps):
        ep = gen.generate(generator=g)
        plies += int(ep['length'].sum())
        loops += int(ep['length'].max())
    torch.cuda.synchronize(dev)
    dt = time.perf_counter() - t0
    print(json.dumps({'env': opts.env, 'games': opts.games, 'graph': opts.graph, 'env_steps_per_s': round(plies / dt, 1),
                      'ms_per_ply_loop': round(dt / loops * 1e3, 3), 'ply_loops': loops}), flush=True)


if __name__ == '__main__':
    main()
