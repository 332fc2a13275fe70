"""Parity of the HIP return-target scans (libhrl.so) with the reference.

* every golden case produced by the reference's handyrl/losses.py must match
  BIT FOR BIT (the kernels replay the reference's float32 op order; the
  tolerance below is the north-star 1e-5 bound, the assertion on exactness
  is separate);
* the fused entry point against the pinned oracle for every (target, adv)
  pair;
* edge cases: ragged B, T=1, multi-chunk T, wide C, per-player rho, NaN,
  unaligned pointers, B=0;
* full BASELINE sizes (B=4096, T=32 and beyond) against the oracle.
"""

import numpy as np
import pytest
import torch

from oracle import targets as ot

pytestmark = pytest.mark.gpu

TOL = 1e-5  # north_star: targets match the reference to 1e-5 fp32
ALGS = ('MC', 'TD', 'UPGO', 'VTRACE')


def _t(x, dev):
    return None if x is None else torch.from_numpy(np.ascontiguousarray(x)).to(dev)


def _np(x):
    return x.detach().cpu().numpy()


def test_golden_targets_bit_exact(cuda, golden_targets):
    from handyrl_amd.losses import compute_target
    meta, arrays = golden_targets
    worst = 0.0
    for c in meta:
        p = '%d:' % c['id']
        rew = arrays[p + 'rewards'] if c['has_rewards'] else None
        args = [_t(arrays[p + k], cuda) for k in ('values', 'returns')]
        tgt, adv = compute_target(c['alg'], args[0], args[1], _t(rew, cuda), c['lmb'], c['gamma'],
                                  _t(arrays[p + 'rhos'], cuda), _t(arrays[p + 'cs'], cuda))
        torch.cuda.synchronize()
        assert tuple(tgt.shape) == arrays[p + 'target'].shape, c
        assert tuple(adv.shape) == arrays[p + 'adv'].shape, c
        dt = np.abs(_np(tgt) - arrays[p + 'target']).max()
        da = np.abs(_np(adv) - arrays[p + 'adv']).max()
        assert dt <= TOL and da <= TOL, (c, dt, da)
        worst = max(worst, dt, da)
    assert worst == 0.0, 'HIP scans are expected to be bit-exact; worst |diff| = %g' % worst


def _random_case(B, T, P, K, Pr, head, seed, dev):
    g = np.random.default_rng(seed)
    values = np.tanh(g.standard_normal((B, T, P, K))).astype(np.float32)
    rhos = np.clip(np.exp(0.5 * g.standard_normal((B, T, Pr, 1))), 0, 1).astype(np.float32)
    cs = np.clip(np.exp(0.5 * g.standard_normal((B, T, Pr, 1))), 0, 1).astype(np.float32)
    if head == 'value':
        returns = g.integers(-1, 2, (B, 1, P, K)).astype(np.float32)
        rewards, gamma = None, 1
    else:
        returns = g.standard_normal((B, T, P, K)).astype(np.float32)
        rewards = (0.01 * g.standard_normal((B, T, P, K))).astype(np.float32)
        gamma = 0.8
    return values, returns, rewards, rhos, cs, gamma


def _check_fused(dev, B, T, P, K, Pr, head, seed, tgt_alg, adv_alg, exact=True):
    from handyrl_amd.losses import compute_targets_fused
    values, returns, rewards, rhos, cs, gamma = _random_case(B, T, P, K, Pr, head, seed, dev)
    tgt, adv = compute_targets_fused(tgt_alg, adv_alg, _t(values, dev), _t(returns, dev), _t(rewards, dev),
                                     0.7, gamma, _t(rhos, dev), _t(cs, dev))
    rt, _ = ot.compute_target(tgt_alg, values, returns, rewards, 0.7, gamma, rhos, cs)
    _, ra = ot.compute_target(adv_alg, values, returns, rewards, 0.7, gamma, rhos, cs)
    tgt, adv = _np(tgt), _np(adv)
    assert tgt.shape == rt.shape and adv.shape == ra.shape
    np.testing.assert_allclose(tgt, rt, rtol=0, atol=TOL)
    np.testing.assert_allclose(adv, ra, rtol=0, atol=TOL)
    if exact:
        np.testing.assert_array_equal(tgt, rt)
        np.testing.assert_array_equal(adv, ra)


class _short_form:
    """hrl_targets_set_short_form(form) for the block (T <= 16: 2 = lane-per-column kernel, 0 = chunked, 1 = the
    default choice by batch size)."""

    def __init__(self, form):
        self.form = form

    def __enter__(self):
        from handyrl_amd import _native
        self.prev = _native.load().hrl_targets_set_short_form(self.form)

    def __exit__(self, *exc):
        from handyrl_amd import _native
        _native.load().hrl_targets_set_short_form(self.prev)
        return False


@pytest.mark.parametrize('form', [2, 0])
@pytest.mark.parametrize('tgt_alg', ALGS)
@pytest.mark.parametrize('adv_alg', ALGS)
@pytest.mark.parametrize('head', ['value', 'return'])
def test_fused_pairs(cuda, tgt_alg, adv_alg, head, form):
    with _short_form(form):
        _check_fused(cuda, 37, 9, 2, 1, 1, head, 11, tgt_alg, adv_alg)


@pytest.mark.parametrize('B,T,P,K,Pr', [
    (1, 1, 1, 1, 1),      # single step: targets are the bootstrap
    (33, 2, 2, 1, 1),     # ragged last wave
    (65, 31, 1, 1, 1),    # C=1: 64 trajectories per wave, ragged
    (40, 33, 2, 1, 2),    # two time chunks, ragged second chunk, per-player rho
    (17, 100, 2, 1, 1),   # four chunks (Geese/GRF-like length)
    (9, 64, 4, 1, 4),     # four players, exact chunks
    (11, 7, 3, 1, 3),     # C=3: wave holds 21 trajectories
    (13, 9, 2, 3, 2),     # K=3 trailing value dims, rho per player
    (5, 128, 1, 1, 1),    # GRF-like T=128
])
@pytest.mark.parametrize('head', ['value', 'return'])
def test_edge_shapes(cuda, B, T, P, K, Pr, head):
    for form in ((2, 0) if T <= 16 else (1,)):
        with _short_form(form):
            for tgt_alg, adv_alg in (('VTRACE', 'UPGO'), ('TD', 'VTRACE'), ('UPGO', 'MC'), ('MC', 'TD')):
                _check_fused(cuda, B, T, P, K, Pr, head, B * 1000 + T, tgt_alg, adv_alg)


@pytest.mark.parametrize('T', [9, 16])
def test_short_forms_identical_at_two_to_the_twenty(cuda, T):
    """configs[1]'s T=9 (and the longest short T) at B = 2^20: the lane-per-column kernel and the chunked
    kernel give bit-identical targets and advantages for the value head (V-trace + UPGO) and the return head
    (TD + V-trace with rewards), both checked against the oracle at B = 4096 in test_baseline_sizes."""
    from handyrl_amd.losses import compute_targets_fused
    B = 1 << 20
    g = torch.Generator(device=cuda).manual_seed(T)
    v = torch.tanh(torch.randn(B, T, 2, 1, device=cuda, generator=g))
    ret = torch.randint(-1, 2, (B, 1, 2, 1), device=cuda, generator=g).float()
    rew = 0.01 * torch.randn(B, T, 2, 1, device=cuda, generator=g)
    rho = torch.rand(B, T, 1, 1, device=cuda, generator=g)
    cs = torch.rand(B, T, 1, 1, device=cuda, generator=g)
    for args in (('VTRACE', 'UPGO', v, ret, None, 0.7, 1, rho, cs), ('TD', 'VTRACE', v, ret, rew, 0.7, 0.8, rho, cs)):
        out = {}
        for form in (2, 0):
            with _short_form(form):
                out[form] = compute_targets_fused(*args)
        for a, b in zip(out[2], out[0]):
            assert torch.equal(torch.nan_to_num(a), torch.nan_to_num(b))


def test_empty_batch(cuda):
    from handyrl_amd.losses import compute_target
    v = torch.zeros(0, 5, 2, 1, device=cuda)
    t, a = compute_target('VTRACE', v, torch.zeros(0, 1, 2, 1, device=cuda), None, 0.7, 1,
                          torch.zeros(0, 5, 1, 1, device=cuda), torch.zeros(0, 5, 1, 1, device=cuda))
    assert t.shape == v.shape and a.shape == v.shape


def test_unaligned_views(cuda):
    """Inputs at a 4-byte (not 16-byte) offset take the scalar path and still match."""
    from handyrl_amd.losses import compute_target
    values, returns, rewards, rhos, cs, gamma = _random_case(50, 16, 2, 1, 1, 'return', 3, cuda)
    def shifted(x):
        flat = torch.zeros(x.size + 1, dtype=torch.float32, device=cuda)
        flat[1:] = _t(x.reshape(-1), cuda)
        return flat[1:].view(*x.shape)
    for alg in ALGS:
        t, a = compute_target(alg, shifted(values), shifted(returns), shifted(rewards), 0.7, gamma,
                              shifted(rhos), shifted(cs))
        rt, ra = ot.compute_target(alg, values, returns, rewards, 0.7, gamma, rhos, cs)
        np.testing.assert_array_equal(_np(t), rt)
        np.testing.assert_array_equal(_np(a), ra)


def test_nan_propagates_like_torch_max(cuda):
    from handyrl_amd.losses import compute_target
    values, returns, rewards, rhos, cs, gamma = _random_case(4, 6, 2, 1, 1, 'return', 5, cuda)
    values[1, 3, 0, 0] = np.nan
    rt, ra = ot.compute_target('UPGO', values, returns, rewards, 0.7, gamma, rhos, cs)
    t, a = compute_target('UPGO', _t(values, cuda), _t(returns, cuda), _t(rewards, cuda), 0.7, gamma,
                          _t(rhos, cuda), _t(cs, cuda))
    np.testing.assert_array_equal(np.isnan(_np(t)), np.isnan(rt))
    np.testing.assert_array_equal(np.nan_to_num(_np(t)), np.nan_to_num(rt))


def test_invalid_arguments(cuda):
    from handyrl_amd.losses import compute_target
    v = torch.zeros(2, 3, 2, 1, device=cuda)
    with pytest.raises(ValueError):
        compute_target('GAE', v, v, None, 0.7, 1, v, v)
    with pytest.raises(TypeError):
        compute_target('TD', v.double(), v, None, 0.7, 1, v, v)
    with pytest.raises(RuntimeError):
        compute_target('TD', v.cpu(), v.cpu(), None, 0.7, 1, v.cpu(), v.cpu())
    assert compute_target('TD', None, v, None, 0.7, 1, v, v) == (None, 0)


@pytest.mark.parametrize('B,T', [(4096, 32), (4096, 9), (2048, 64), (1024, 128), (65536, 32)])
def test_baseline_sizes(cuda, B, T):
    """BASELINE.json configs (value + return heads) against the oracle, bit for bit."""
    _check_fused(cuda, B, T, 2, 1, 1, 'value', B + T, 'VTRACE', 'UPGO')
    _check_fused(cuda, B, T, 2, 1, 1, 'return', B + T + 1, 'VTRACE', 'UPGO')


def test_large_batch_properties(cuda):
    """B = 2^20 trajectories (0.5 GB working set): V-trace with rho = c = 1 and
    lambda = 1 telescopes to the discounted return, a size-independent identity."""
    from handyrl_amd.losses import compute_target
    B, T = 1 << 20, 8
    g = torch.Generator(device=cuda).manual_seed(0)
    v = torch.rand(B, T, 2, 1, device=cuda, generator=g)
    r = torch.rand(B, T, 2, 1, device=cuda, generator=g) * 0.1
    ret = torch.rand(B, T, 2, 1, device=cuda, generator=g)
    ones = torch.ones(B, T, 1, 1, device=cuda)
    vs, _ = compute_target('VTRACE', v, ret, r, 1.0, 0.9, ones, ones)
    # reference identity: vs[t] = r[t] + 0.9 * vs[t+1] (vs[T] := ret[T-1])
    expect = torch.empty_like(vs)
    nxt = ret[:, -1]
    for t in range(T - 1, -1, -1):
        expect[:, t] = r[:, t] + 0.9 * nxt
        nxt = expect[:, t]
    assert torch.allclose(vs, expect, atol=1e-5, rtol=0)
