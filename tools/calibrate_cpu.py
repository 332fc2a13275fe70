"""D4 calibration: the CPU port vs the reference learner, timed here.

bench.py's ``cpu_baseline`` runs on the GPU box, where the reference cannot
go, so it times the port ``oracle.learner.CpuLearner``.  This script (build
container only; it imports /root/reference read-only) times both on the same
synthetic TicTacToe batch, same seeded net, 1 torch thread as shipped
(model.py:8, main.py:10), the body of Trainer.train (train.py:375-385:
compute_loss, backward, clip_grad_norm_(4.0), Adam), and writes
profiles/r02_cpu_calibration.json.

    PYTHONDONTWRITEBYTECODE=1 python tools/calibrate_cpu.py
"""

import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(1, os.environ.get('HANDYRL_REF', '/root/reference'))
sys.dont_write_bytecode = True

import torch  # noqa: E402
import torch.nn as nn  # noqa: E402


def time_steps(step, n):
    step()                      # warm-up
    t0 = time.perf_counter()
    for _ in range(n):
        step()
    return (time.perf_counter() - t0) / n


def main():
    from handyrl import train as ref_train
    from handyrl.envs.tictactoe import SimpleConv2dModel as RefNet
    from handyrl.model import ModelWrapper
    from handyrl_amd.envs.tictactoe import SimpleConv2dModel
    from handyrl_amd.synthetic import tictactoe_batch, default_args
    from oracle.learner import CpuLearner

    torch.set_num_threads(1)
    rows = []
    for B, T, n in ((4096, 32, 3), (4096, 9, 5), (2048, 32, 3)):
        args = default_args(T, B)
        batch = tictactoe_batch(B, T, torch.device('cpu'), seed=11)

        torch.manual_seed(0)
        ref_model = ModelWrapper(RefNet())
        params = list(ref_model.parameters())
        opt = torch.optim.Adam(params, lr=3e-8 * B * T, weight_decay=1e-5)
        ref_model.train()

        def ref_step():
            losses, _ = ref_train.compute_loss(batch, ref_model, None, args)
            opt.zero_grad()
            losses['total'].backward()
            nn.utils.clip_grad_norm_(params, 4.0)
            opt.step()
        t_ref = time_steps(ref_step, n)

        torch.manual_seed(0)
        port = CpuLearner(SimpleConv2dModel(), args)
        t_port = time_steps(lambda: port.step(batch), n)
        rows.append({'B': B, 'T': T, 'steps': n, 'reference_ms': t_ref * 1e3, 'port_ms': t_port * 1e3,
                     'reference_env_steps_per_s': B * T / t_ref, 'port_env_steps_per_s': B * T / t_port,
                     'port_vs_reference': t_port / t_ref})
        print(json.dumps(rows[-1]))
    import platform
    out = {'host': platform.processor() or platform.machine(), 'cpus': os.cpu_count(), 'threads': 1,
           'torch': torch.__version__, 'rows': rows,
           'note': 'same synthetic batch and seeded net; body of Trainer.train (train.py:375-385); the port is '
                   'within +-15% of the reference when port_vs_reference is in [0.85, 1.15]'}
    with open(os.path.join(ROOT, 'profiles', 'r02_cpu_calibration.json'), 'w') as f:
        json.dump(out, f, indent=1)


if __name__ == '__main__':
    main()
