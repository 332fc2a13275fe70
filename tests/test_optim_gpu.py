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
@pytest.mark.parametrize('bad', [float('nan'), float('inf')])
def test_clip_kernel_nonfinite_like_torch(cuda, bad):
    _, grads = _params(SHAPES, 1.0, cuda, 2)
    grads[2][3, 4] = bad
    got, tg = _run_flat(SHAPES, grads, cuda, 4.0)
    ref, tr = _run_torch(SHAPES, grads, 4.0)
    assert (math.isnan(tg) and math.isnan(tr)) or tg == tr
    for a, b in zip(got, ref):
        torch.testing.assert_close(a, b, rtol=0, atol=0, equal_nan=True)
