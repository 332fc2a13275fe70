"""Per-parameter gradient error of one GPU learner step against the fp64 CPU oracle (diagnostic).

    python tools/grad_diag.py ttt 9        # TicTacToe, B=4096, T=9
    python tools/grad_diag.py geese 64     # GeeseNet, B=512, T=64

Prints, per parameter, the norm-relative error of the fp32 CPU oracle and of the GPU step (block backward
forms 1 and 0 for TicTacToe) against the fp64 step, and for the TicTacToe stem the error of the stem's
weight-gradient kernel alone (its own output vs x^T dy in fp64 from the GPU's dy).
"""

import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from tests.test_learner_gpu import oracle_step_grads
    from handyrl_amd.trainer import LearnerStep
    from handyrl_amd import _native
    case, T = sys.argv[1], int(sys.argv[2])
    dev = torch.device('cuda', 0)
    if case == 'ttt':
        from handyrl_amd.envs.tictactoe import SimpleConv2dModel as cls
        from handyrl_amd.synthetic import tictactoe_batch, default_args
        B = 4096
        args = default_args(T, B)
        batch = tictactoe_batch(B, T, dev, seed=11 + T)
        torch.manual_seed(1)
    else:
        from handyrl_amd.envs.hungry_geese import GeeseNet as cls
        from handyrl_amd.synthetic import geese_batch, geese_args
        B = 512
        args = geese_args(T, B)
        batch = geese_batch(B, T, dev, seed=9)
        torch.manual_seed(2)
    state = cls().state_dict()
    r32, r64 = oracle_step_grads(cls, state, batch, args)
    cols = {}
    forms = [1, 0] if case == 'ttt' else [1]
    stem = {}
    for form in forms:
        _native.load().hrl_conv3x3_set_block_form(form)
        net = cls()
        net.load_state_dict(state)
        step = LearnerStep(net, args, dev, graph=False)
        if case == 'ttt' and form == 1:
            def fwd_hook(mod, inp, out):
                if out.requires_grad:
                    stem['x'] = inp[0].detach()
                    out.register_hook(lambda g: stem.__setitem__('dy', g.detach()))
            step.net.conv.register_forward_hook(fwd_hook)
        step.step(batch)
        torch.cuda.synchronize()
        cols['gpu%d' % form] = {n: p.grad.detach().cpu().double() for n, p in step.net.named_parameters()}
    _native.load().hrl_conv3x3_set_block_form(1)
    print('%-28s %12s %10s %10s %s' % ('param', '|g64|', 'cpu32', 'gpu f1', 'gpu f0' if len(forms) > 1 else ''))
    for n, g64 in r64['grads'].items():
        den = float(g64.norm())
        if den == 0:
            continue
        row = [float((r32['grads'][n] - g64).norm()) / den]
        for f in forms:
            row.append(float((cols['gpu%d' % f][n] - g64).norm()) / den)
        print('%-28s %12.4e ' % (n, den) + ' '.join('%10.3e' % v for v in row))
    if stem:
        # the stem kernel alone: its (unclipped) weight gradient vs fp64 x^T dy from the same dy
        x, dy = stem['x'].double(), stem['dy'].double()
        w64 = torch.nn.grad.conv2d_weight(x, (32, x.shape[1], 3, 3), dy, padding=1)
        print('stem dy: |sum| / sum|.| per channel (cancellation):',
              float((dy.sum((0, 2, 3)).abs() / dy.abs().sum((0, 2, 3))).max()))
        print('stem weight grad kernel alone: x^T dy cancellation ratio sum|x dy| / |x^T dy| = %.3e' %
              float(torch.nn.grad.conv2d_weight(x.abs(), (32, x.shape[1], 3, 3), dy.abs(), padding=1).sum()
                    / w64.abs().sum()))
        from handyrl_amd.nn import _StemConv  # noqa: F401  (the kernel under test)
        lib = _native.load()
        N, Cin = x.shape[0], x.shape[1]
        ws = torch.empty(lib.hrl_stem_workspace_bytes(N), dtype=torch.uint8, device=dev)
        dw = torch.empty(32, Cin, 3, 3, device=dev)
        db = torch.empty(32, device=dev)
        _native.check(lib.hrl_stem_wgrad(_native.ptr(stem['x']), _native.ptr(stem['dy'].contiguous()), N, Cin,
                                         _native.ptr(dw), _native.ptr(db), _native.ptr(ws), ws.numel(),
                                         _native.stream_of(dev)), 'hrl_stem_wgrad')
        torch.cuda.synchronize()
        print('stem kernel norm-rel error vs fp64 from the same dy: %.3e' %
              float((dw.double() - w64).norm() / w64.norm()))


if __name__ == '__main__':
    main()
