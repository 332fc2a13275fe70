"""One-launch gradient clipping (csrc/hrl_optim.hip) vs the reference's
nn.utils.clip_grad_norm_(params, 4.0) (handyrl/train.py:384), including
non-finite gradients: a NaN norm makes every gradient NaN, an inf norm scales
finite gradients to 0 (torch.clamp(coef, max=1) semantics)."""

import math

import pytest
import torch
import torch.nn as nn

from handyrl_amd.distributed import FlatGrads


def _params(shapes, scale, device, seed):
    g = torch.Generator().manual_seed(seed)
    ps = [nn.Parameter(torch.zeros(s)) for s in shapes]
    grads = [torch.randn(s, generator=g) * scale for s in shapes]
    return ps, grads


def _run_flat(shapes, grads, device, max_norm):
    ps = [nn.Parameter(torch.zeros(s, device=device)) for s in shapes]
    fg = FlatGrads(ps)
    for p, g in zip(ps, grads):
        p.grad.copy_(g.to(device))
    total = fg.clip_(max_norm)
    return [p.grad.detach().cpu() for p in ps], float(total)


def _run_torch(shapes, grads, max_norm):
    ps = [nn.Parameter(torch.zeros(s)) for s in shapes]
    for p, g in zip(ps, grads):
        p.grad = g.clone()
    total = nn.utils.clip_grad_norm_(ps, max_norm)
    return [p.grad for p in ps], float(total)


SHAPES = [(32, 3, 3, 3), (32,), (9, 27), (1,), (7, 5)]   # 5 tensors, ragged tail (not a multiple of 4)
# GeisterNet-sized (234 k floats, the two-launch multi-workgroup form above 64 k) with a ragged tail
BIG = [(128, 64, 3, 3), (128, 64, 3, 3), (32, 25, 3, 3), (70,), (3,)]


@pytest.mark.parametrize('scale', [1e-3, 1.0, 100.0])      # below, near and above the 4.0 threshold
def test_clip_matches_torch_cpu(scale):
    """Host form (FlatGrads.clip_ on CPU tensors)."""
    _, grads = _params(SHAPES, scale, 'cpu', 0)
    got, tg = _run_flat(SHAPES, grads, 'cpu', 4.0)
    ref, tr = _run_torch(SHAPES, grads, 4.0)
    assert abs(tg - tr) <= 1e-6 * tr
    for a, b in zip(got, ref):
        torch.testing.assert_close(a, b, rtol=1e-6, atol=0)


@pytest.mark.gpu
@pytest.mark.parametrize('scale', [1e-3, 1.0, 100.0])
def test_clip_kernel_matches_torch(cuda, scale):
    _, grads = _params(SHAPES, scale, cuda, 1)
    got, tg = _run_flat(SHAPES, grads, cuda, 4.0)
    ref, tr = _run_torch(SHAPES, grads, 4.0)
    assert abs(tg - tr) <= 1e-6 * tr
    for a, b in zip(got, ref):
        torch.testing.assert_close(a, b, rtol=1e-6, atol=0)


@pytest.mark.gpu
@pytest.mark.parametrize('scale', [1e-3, 100.0])
def test_clip_kernel_large_buffer_matches_torch(cuda, scale):
    """The two-launch form (per-workgroup fp64 partials folded in one order by every workgroup) at GeisterNet's
    size: norm and clipped gradients against torch, as the one-launch form."""
    _, grads = _params(BIG, scale, cuda, 3)
    got, tg = _run_flat(BIG, grads, cuda, 4.0)
    ref, tr = _run_torch(BIG, grads, 4.0)
    assert abs(tg - tr) <= 1e-6 * tr
    for a, b in zip(got, ref):
        torch.testing.assert_close(a, b, rtol=1e-6, atol=0)


@pytest.mark.gpu
@pytest.mark.parametrize('bad', [float('nan'), float('inf')])
@pytest.mark.parametrize('shapes', [SHAPES, BIG])
def test_clip_kernel_nonfinite_like_torch(cuda, bad, shapes):
    _, grads = _params(shapes, 1.0, cuda, 2)
    grads[2][3, 4] = bad
    got, tg = _run_flat(shapes, grads, cuda, 4.0)
    ref, tr = _run_torch(shapes, grads, 4.0)
    assert (math.isnan(tg) and math.isnan(tr)) or tg == tr
    for a, b in zip(got, ref):
        torch.testing.assert_close(a, b, rtol=0, atol=0, equal_nan=True)


@pytest.mark.gpu
@pytest.mark.parametrize('graph', [False, True])
def test_step_tail_matches_torch_clip_and_adam(cuda, graph):
    """trainer.StepTail (csrc/hrl_optim.hip: hrl_grad_fold_norm + hrl_adam_clip) over a flat gradient buffer vs
    nn.utils.clip_grad_norm_(4.0) + torch.optim.Adam(lr, weight_decay=1e-5, fused=True) on the same gradients for
    four steps (train.py:384-385): the norms, the clipped gradients (p.grad afterwards) and the parameters; a
    parameter marked dead (no gradient, reference semantics) is never touched; replayed from a HIP graph with a
    changed lr, as LearnerStep's step does."""
    from handyrl_amd.trainer import StepTail
    shapes = [(32, 3, 3, 3), (32,), (9, 18), (1,), (1, 9), (128, 64, 3, 3), (7, 5)]
    g = torch.Generator().manual_seed(5)
    init = [torch.randn(s, generator=g) * 0.1 for s in shapes]
    grads = [[torch.randn(s, generator=g) * sc for s in shapes] for sc in (0.5, 3.0, 0.01, 1.0)]
    live = [True, True, True, False, True, True, True]
    lrs = [1e-3, 1e-3, 5e-4, 5e-4]
    ref = [nn.Parameter(t.clone().to(cuda)) for t in init]
    opt = torch.optim.Adam([p for p, l in zip(ref, live) if l], lr=lrs[0], weight_decay=1e-5, fused=True)
    ps = [nn.Parameter(t.clone().to(cuda)) for t in init]
    fg = FlatGrads(ps)
    tail = StepTail(fg, lrs[0])
    tail.set_live(live)
    gr = None
    if graph:
        for p, t in zip(ps, grads[0]):
            p.grad.copy_(t.to(cuda))
        tg = torch.cuda.CUDAGraph()
        snap = [p.detach().clone() for p in ps]
        side = torch.cuda.Stream(cuda)
        side.wait_stream(torch.cuda.current_stream(cuda))
        with torch.cuda.stream(side):
            tail(None)                      # warm-up, then undone
        torch.cuda.current_stream(cuda).wait_stream(side)
        with torch.no_grad():
            for p, s in zip(ps, snap):
                p.copy_(s)
            for t in tail.state_tensors():
                t.zero_()
        with torch.cuda.graph(tg):
            gr = tail(None)
    for k in range(4):
        for i, (p, t) in enumerate(zip(ref, grads[k])):
            p.grad = t.to(cuda).clone() if live[i] else None
        for group in opt.param_groups:
            group['lr'] = lrs[k]
        tr = float(nn.utils.clip_grad_norm_([p for p in ref if p.grad is not None], 4.0))
        opt.step()
        for p, t, l in zip(ps, grads[k], live):
            p.grad.copy_(t.to(cuda) if l else torch.zeros_like(t).to(cuda))
        tail.set_lr(lrs[k])
        if graph:
            tg.replay()
            tt = float(gr)
        else:
            tt = float(tail(None))
        assert abs(tt - tr) <= 1e-6 * tr, (k, tt, tr)
        for i, (a, b) in enumerate(zip(ps, ref)):
            if live[i]:
                torch.testing.assert_close(a.grad, b.grad, rtol=1e-6, atol=0)
                torch.testing.assert_close(a.detach(), b.detach(), rtol=2e-6, atol=2e-7)
            else:
                assert torch.equal(a.detach().cpu(), init[i])


@pytest.mark.gpu
def test_grad_fold_norm_folds_partials(cuda):
    """hrl_grad_fold_norm's deferred folds: mode 0 columns of partial rows and mode 1 (a 32x32x3x3 conv weight from
    [tap][ci][co] rows) summed over the rows into their destinations of the flat buffer, the rest untouched; the
    per-block sums of squares add up to the squared norm; the step count advances once and each counter by its
    increment (a recurrent unroll's per-step BatchNorm counts T)."""
    import ctypes
    from handyrl_amd import _native
    lib = _native.load()
    P = _native.ptr
    g0 = torch.Generator(device=cuda).manual_seed(2)
    n = 9216 + 300 + 41
    flat = torch.randn(n, device=cuda, generator=g0)
    before = flat.clone()
    p1 = torch.randn(256, 9216, device=cuda, generator=g0)             # conv partials [tap][ci][co]
    p0 = torch.randn(1000, 270, device=cuda, generator=g0)             # heads-like partial rows
    step = torch.zeros((), device=cuda)
    ctr = [torch.zeros((), dtype=torch.int64, device=cuda) for _ in range(3)]
    nb = lib.hrl_grad_fold_norm_blocks(n)
    norm_part = torch.empty(nb, dtype=torch.float64, device=cuda)
    folds = [(p1, 9216, 0, 256, 0, 9216, 1), (p0, 270, 99, 1000, 9216 + 10, 162, 0),
             (p0, 270, 261, 1000, 9216 + 200, 9, 0)]
    i64 = _native.i64_array
    _native.check(lib.hrl_grad_fold_norm(
        P(flat), n, _native.ptr_array([f[0] for f in folds]), i64([f[1] for f in folds]), i64([f[2] for f in folds]),
        i64([f[3] for f in folds]), i64([f[4] for f in folds]), i64([f[5] for f in folds]),
        (ctypes.c_int * 3)(*[f[6] for f in folds]), 3, P(step), _native.ptr_array(ctr), i64([1, 16, 3]), 3,
        P(norm_part), nb * 8, _native.stream_of(cuda)), 'fold')
    torch.cuda.synchronize(cuda)
    ref = before.double().cpu()
    conv = p1.double().sum(0).view(9, 32, 32).permute(2, 1, 0).reshape(-1)   # (tap, ci, co) -> (co, ci, tap)
    # folds ADD into their destinations (another use of the parameter may have added its gradient there)
    ref[:9216] += conv.cpu()
    ref[9226:9226 + 162] += p0.double().sum(0)[99:261].cpu()
    ref[9416:9425] += p0.double().sum(0)[261:270].cpu()
    got = flat.double().cpu()
    assert float((got - ref).abs().max()) <= 1e-5 * float(ref.abs().max())
    assert torch.equal(got[9216:9226], before[9216:9226].double().cpu())
    tot = float(norm_part.sum())
    assert abs(tot - float((got ** 2).sum())) <= 1e-9 * tot
    assert float(step) == 1.0 and [int(c) for c in ctr] == [1, 16, 3]   # each counter by its increment


def _twice_stem_net():
    """The TicTacToe net with its stem applied twice (to the board and to its mirror image): the stem's HIP
    Function is reached twice, so one use may leave its weight gradient as deferred partials while autograd adds
    the other use's gradient into the same p.grad during the backward."""
    import torch.nn.functional as F
    from handyrl_amd.envs.tictactoe import SimpleConv2dModel

    class TwiceStem(SimpleConv2dModel):
        def forward(self, x, hidden=None):
            h = F.relu(self.conv(x)) + F.relu(self.conv(x.flip(-1)))
            for blk in self.blocks:
                h = F.relu(blk(h))
            return {'policy': self.head_p(h), 'value': torch.tanh(self.head_v(h))}
    return TwiceStem()


@pytest.mark.gpu
@pytest.mark.parametrize('case', ['shared_stem', 'nine_blocks'])
def test_deferred_folds_match_unfolded_step(cuda, case):
    """LearnerStep with the step tail's deferred folds vs the same step with every Function folding its own
    partials (fold_deferral off): a parameter used twice in the step (the fold adds to what autograd accumulated,
    ADVICE r5) and a 9-block chain, whose 9 + 6 + 2 folds and 9 BatchNorm counters overflow the tail's tables
    (16 / 8): the Functions past the limit fold with their own launch, the counters advance by their own add."""
    from handyrl_amd.envs.tictactoe import SimpleConv2dModel
    from handyrl_amd.synthetic import tictactoe_batch, default_args
    from handyrl_amd.trainer import LearnerStep
    B, T = 64, 9
    args = default_args(T, B)
    make = _twice_stem_net if case == 'shared_stem' else (lambda: SimpleConv2dModel(layers=9))
    torch.manual_seed(0)
    a = make()
    torch.manual_seed(0)
    b = make()
    sa, sb = LearnerStep(a, args, cuda), LearnerStep(b, args, cuda)
    assert sa.fold_deferral and sa.tail is not None
    sb.fold_deferral = False
    for s in range(2):
        batch = tictactoe_batch(B, T, cuda, seed=7 + s)
        oa, ob = sa.step(batch), sb.step(batch)
        ga, gb = float(oa['grad_norm']), float(ob['grad_norm'])
        assert abs(ga - gb) <= 1e-5 * gb, (s, ga, gb)
    for (k, va), vb in zip(a.state_dict().items(), b.state_dict().values()):
        if k.endswith('num_batches_tracked'):
            assert int(va) == int(vb) == 2, k
        else:
            torch.testing.assert_close(va, vb, rtol=1e-5, atol=1e-6, msg=k)
