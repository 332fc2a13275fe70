"""The CPU oracle (oracle/targets.py) reproduces the reference bit for bit.

The golden vectors were produced by importing the reference's
handyrl/losses.py (tests/golden/make_golden.py); this pins the oracle that
the GPU tests compare against.
"""

import numpy as np
import pytest

from oracle import targets as ot


def _case(arrays, c):
    p = '%d:' % c['id']
    rew = arrays[p + 'rewards'] if c['has_rewards'] else None
    return (arrays[p + 'values'], arrays[p + 'returns'], rew, arrays[p + 'rhos'], arrays[p + 'cs'],
            arrays[p + 'target'], arrays[p + 'adv'])


def test_targets_bit_exact(golden_targets):
    meta, arrays = golden_targets
    assert len(meta) >= 100
    for c in meta:
        v, ret, rew, rho, cs, tgt, adv = _case(arrays, c)
        t, a = ot.compute_target(c['alg'], v, ret, rew, c['lmb'], c['gamma'], rho, cs)
        assert t.shape == tgt.shape and a.shape == adv.shape, c
        np.testing.assert_array_equal(t, tgt, err_msg=str(c))
        np.testing.assert_array_equal(a, adv, err_msg=str(c))


def test_values_none_convention():
    assert ot.compute_target('TD', None, None, None, 0.7, 1, None, None) == (None, 0)


def test_unknown_algorithm():
    v = np.zeros((1, 2, 1, 1), np.float32)
    with pytest.raises(ValueError):
        ot.compute_target('GAE', v, v, None, 0.7, 1, v, v)


def test_loss_fixture_calls_match_oracle(golden_loss):
    """Every compute_target call recorded inside the reference compute_loss."""
    meta, arrays = golden_loss
    n = 0
    for c in meta:
        for j, call in enumerate(c['calls']):
            if call['values_none']:
                continue
            p = '%d:call%d.' % (c['id'], j)
            head = 'value' if j % 2 == 0 else 'return'
            b = '%d:batch.' % c['id']
            if head == 'value':
                ret, rew = arrays[b + 'outcome'], None
            else:
                ret, rew = arrays[b + 'return'], arrays[b + 'reward']
            rho = arrays[p + 'rhos']
            t, a = ot.compute_target(call['alg'], arrays[p + 'values'], ret, rew, call['lmb'], call['gamma'], rho, rho)
            np.testing.assert_array_equal(t, arrays[p + 'target'])
            np.testing.assert_array_equal(a, arrays[p + 'adv'])
            n += 1
    assert n >= 10
