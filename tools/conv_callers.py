"""Which vendor convolutions does one eager Geister learner step still call?  torch.profiler over one LearnerStep
(B=256, T=16, eager), printing every aten convolution op with its input shapes and the Python frames above it.

    python tools/conv_callers.py
"""
import collections
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
from torch.profiler import profile, ProfilerActivity  # noqa: E402

from handyrl_amd.envs.geister import GeisterNet  # noqa: E402
from handyrl_amd.synthetic import geister_batch, default_args  # noqa: E402
from handyrl_amd.trainer import LearnerStep  # noqa: E402


def main():
    dev = torch.device('cuda', 0)
    B, T = 256, 16
    torch.manual_seed(0)
    net = GeisterNet().to(dev)
    batch = geister_batch(B, T, dev, seed=5)
    hidden = tuple([x.to(dev) for x in h] for h in net.init_hidden([B, 2]))
    step = LearnerStep(net, default_args(T, B), dev, graph=False)
    step.step(batch, hidden)
    torch.cuda.synchronize(dev)
    with profile(activities=[ProfilerActivity.CPU], record_shapes=True, with_stack=True) as prof:
        step.step(batch, hidden)
        torch.cuda.synchronize(dev)
    seen = collections.Counter()
    for ev in prof.events():
        if 'conv' not in ev.name or ev.name.startswith('aten::_conv') is False and 'convolution' not in ev.name:
            continue
        stack = [f for f in (ev.stack or []) if 'handyrl_amd' in f][:3]
        seen[(ev.name, str(ev.input_shapes)[:160], ' <- '.join(stack))] += 1
    for (name, shapes, stack), n in seen.most_common():
        print(n, name, shapes, '|', stack)


if __name__ == '__main__':
    main()
