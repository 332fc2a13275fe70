"""Two kernel forms of one learner step, side by side: the flat gradient of the first step (max abs / rel difference)
and the loss trajectory over --steps updates on the same batch (bench.py's workload), to tell rounding-order drift
from a real difference.

    python tools/diag_forms.py --setter hrl_heads_set_bwd_form --forms 1,2 [--steps 25] [--graph]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from handyrl_amd import _native  # noqa: E402
from handyrl_amd.envs.tictactoe import SimpleConv2dModel  # noqa: E402
from handyrl_amd.synthetic import default_args, tictactoe_batch  # noqa: E402
from handyrl_amd.trainer import LearnerStep  # noqa: E402


def run(setter, form, steps, graph, B, T, dev):
    prev = setter(form)
    try:
        torch.manual_seed(0)
        net = SimpleConv2dModel().to(dev)
        batch = tictactoe_batch(B, T, dev, seed=1000)
        learner = LearnerStep(net, default_args(T, B), dev, graph=graph)
        traj, first = [], None
        for s in range(steps):
            out = learner.step(batch)
            if s == 0:
                first = learner.grads.flat.detach().clone()
            traj.append((float(out['total']), float(out['grad_norm'])))
        return first, traj
    finally:
        setter(prev)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--setter', required=True)
    ap.add_argument('--forms', default='1,2')
    ap.add_argument('--steps', type=int, default=25)
    ap.add_argument('--graph', action='store_true')
    ap.add_argument('--batch', type=int, default=4096)
    ap.add_argument('--seq', type=int, default=32)
    o = ap.parse_args()
    dev = torch.device('cuda', 0)
    setter = getattr(_native.load(), o.setter)
    fa, fb = [int(f) for f in o.forms.split(',')]
    ga, ta = run(setter, fa, o.steps, o.graph, o.batch, o.seq, dev)
    gb, tb = run(setter, fb, o.steps, o.graph, o.batch, o.seq, dev)
    d = (ga - gb).abs()
    rel = d / gb.abs().clamp_min(1e-30)
    print('first-step flat gradient: max |diff| %.3e at %d (%.6e vs %.6e), max rel %.3e, n differing %d of %d'
          % (float(d.max()), int(d.argmax()), float(ga[d.argmax()]), float(gb[d.argmax()]), float(rel.max()),
             int((d > 0).sum()), d.numel()))
    for s, (a, b) in enumerate(zip(ta, tb)):
        print('step %2d  total %.6f %.6f  norm %.6f %.6f' % (s, a[0], b[0], a[1], b[1]))


if __name__ == '__main__':
    main()
