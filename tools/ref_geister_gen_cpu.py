"""Time the reference's own Geister self-play generator on the CPU (this container only).

One process, GeisterNet inference per ply (generation.py:20-88,
model.py:43-53), as one reference worker runs it.  Reports plies/s.

    PYTHONDONTWRITEBYTECODE=1 python tools/ref_geister_gen_cpu.py --episodes 6 --threads 1
"""

import argparse
import json
import sys
import time

sys.path.insert(0, '/root/reference')

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--episodes', type=int, default=6)
    ap.add_argument('--threads', type=int, default=1)
    opts = ap.parse_args()
    torch.set_num_threads(opts.threads)
    from handyrl.environment import make_env
    from handyrl.generation import Generator
    from handyrl.model import ModelWrapper
    env = make_env({'env': 'Geister'})
    torch.manual_seed(0)
    model = ModelWrapper(env.net()())
    gen = Generator(env, {'observation': False, 'gamma': 0.8, 'compress_steps': 4})
    plies, t0 = 0, time.perf_counter()
    for _ in range(opts.episodes):
        ep = gen.generate({0: model, 1: model}, {'player': [0, 1]})
        plies += ep['steps']
    dt = time.perf_counter() - t0
    print(json.dumps({'episodes': opts.episodes, 'plies': plies, 'threads': opts.threads,
                      'plies_per_s': round(plies / dt, 1)}))


if __name__ == '__main__':
    main()
