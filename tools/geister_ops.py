"""Where the Geister learner step's torch launches come from: one eager step of the recurrent learner
(GeisterNet, B=256 T=16).  Two views:
  * torch.profiler: the aten ops that launched GPU kernels, counted (the autograd engine's own gradient sums
    included);
  * a TorchFunctionMode over the same step: every torch call made from Python (forward code and the HIP
    Functions' backward code) on a CUDA tensor, attributed to its innermost handyrl_amd frame (file:line).

    python tools/geister_ops.py [--B 256] [--T 16]
"""
import argparse
import collections
import os
import sys
import traceback

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
from torch.overrides import TorchFunctionMode  # noqa: E402
from torch.profiler import ProfilerActivity, profile  # noqa: E402

from handyrl_amd.envs.geister import GeisterNet  # noqa: E402
from handyrl_amd.synthetic import default_args, geister_batch  # noqa: E402
from handyrl_amd.trainer import LearnerStep  # noqa: E402

QUIET = {'view', 'reshape', 'size', 'dim', 'stride', 'data_ptr', 'is_contiguous', 'contiguous', 'element_size',
         'numel', 'shape', 'dtype', 'device', 'is_cuda', 'requires_grad', 'grad', 'grad_fn', 'detach', 'split',
         '__getitem__', 'storage_offset', 'select', 'narrow', 'unbind', 'chunk', 'transpose', 't', 'permute',
         'expand', 'view_as', '__get__', 'unsqueeze', 'squeeze', 'is_floating_point', 'item', '__len__',
         'untyped_storage', 'new_empty', 'empty_like', 'empty', 'layout', 'is_leaf', 'ndim', 'T', 'data',
         'requires_grad_', '_version', 'nelement', 'get_device', 'is_sparse', '__hash__', '__eq__', 'apply',
         'register_hook', 'flatten'}


class Calls(TorchFunctionMode):
    def __init__(self):
        super().__init__()
        self.sites = collections.Counter()

    def __torch_function__(self, func, types, args=(), kwargs=None):
        name = getattr(func, '__name__', str(func))
        if name not in QUIET:
            leaves = [a for a in list(args) + list((kwargs or {}).values()) if isinstance(a, torch.Tensor)]
            leaves += [t for a in args if isinstance(a, (list, tuple)) for t in a if isinstance(t, torch.Tensor)]
            if any(t.is_cuda for t in leaves):
                site = '?'
                for fr in reversed(traceback.extract_stack()[:-1]):
                    if 'handyrl_amd' in fr.filename and 'tools' not in fr.filename:
                        site = '%s:%d %s' % (fr.filename.split('handyrl_amd/')[-1], fr.lineno, fr.name)
                        break
                self.sites[(name, site)] += 1
        return func(*args, **(kwargs or {}))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--B', type=int, default=256)
    ap.add_argument('--T', type=int, default=16)
    o = ap.parse_args()
    dev = torch.device('cuda', 0)
    torch.manual_seed(0)
    net = GeisterNet().to(dev)
    batch = geister_batch(o.B, o.T, dev, seed=5)
    hidden = tuple([h.to(dev) for h in hs] for hs in net.init_hidden([o.B, 2]))
    learner = LearnerStep(net, default_args(o.T, o.B), dev, graph=False)
    for _ in range(3):
        learner.step(batch, hidden)
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
        learner.step(batch, hidden)
        torch.cuda.synchronize()
    ops = collections.Counter()
    nodes = collections.Counter()
    for ev in prof.events():
        if ev.device_type == torch.autograd.DeviceType.CPU and ev.name.startswith('aten::') and ev.kernels:
            ops[ev.name] += len(ev.kernels)
            # the autograd node (or the forward op) it ran under: the outermost non-aten ancestor
            par, node = ev.cpu_parent, None
            while par is not None:
                if par.name.startswith('autograd::engine::evaluate_function'):
                    node = par.name.split(': ', 1)[-1]
                    break
                par = par.cpu_parent
            top = ev
            while top.cpu_parent is not None and top.cpu_parent.name.startswith('aten::'):
                top = top.cpu_parent
            nodes[(ev.name, node or 'forward: ' + top.name)] += len(ev.kernels)
    print('aten ops with GPU kernels in one eager step: %d launches' % sum(ops.values()))
    for name, n in ops.most_common(30):
        print('%4d  %s' % (n, name))
    print('\nby autograd node (backward) or outermost aten op (forward):')
    for (name, node), n in nodes.most_common(60):
        print('%4d  %-22s %s' % (n, name, node))
    mode = Calls()
    # the mode sees the forward thread; the backward runs on the autograd engine's device thread, so the common
    # launching calls are also wrapped process-wide for the same step
    patched = []
    for owner, names in ((torch.Tensor, ('add_', 'add', 'sum', 'copy_', 'zero_', 'fill_', 'mul', 'mul_', 'sub',
                                         '__add__', '__mul__', '__sub__', '__rsub__', 'clone', 'index_select')),
                         (torch, ('cat', 'stack', 'zeros_like', 'zeros', 'matmul', 'mm', 'bmm', 'tensordot', 'sum',
                                  'tanh', 'flip', 'addmm'))):
        for n in names:
            orig = getattr(owner, n)

            def wrap(*a, _orig=orig, _n=n, **k):
                if torch.overrides._get_current_function_mode() is None:   # not already seen by the mode
                    leaves = [t for t in list(a) + list(k.values()) if isinstance(t, torch.Tensor)]
                    leaves += [t for x in a if isinstance(x, (list, tuple)) for t in x if isinstance(t, torch.Tensor)]
                    if any(t.is_cuda for t in leaves):
                        site = '?'
                        for fr in reversed(traceback.extract_stack()[:-1]):
                            if 'handyrl_amd' in fr.filename and 'tools' not in fr.filename:
                                site = '%s:%d %s' % (fr.filename.split('handyrl_amd/')[-1], fr.lineno, fr.name)
                                break
                        mode.sites[('bwd ' + _n, site)] += 1
                return _orig(*a, **k)
            setattr(owner, n, wrap)
            patched.append((owner, n, orig))
    try:
        with mode:
            learner.step(batch, hidden)
        torch.cuda.synchronize()
    finally:
        for owner, n, orig in patched:
            setattr(owner, n, orig)
    print('\ntorch calls on CUDA tensors from Python in one eager step, by handyrl_amd site:')
    for (name, site), n in sorted(mode.sites.items(), key=lambda kv: -kv[1])[:90]:
        print('%4d  %-24s %s' % (n, name, site))


if __name__ == '__main__':
    main()
