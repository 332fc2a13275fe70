"""numpy float32 restatement of handyrl/losses.py — TEST INFRASTRUCTURE ONLY.

Each recurrence follows the reference operation by operation (same operand
order, one float32 rounding per torch op, Python scalars rounded to float32
exactly where torch rounds them), so it reproduces the reference bit for bit
on the golden vectors (tests/test_oracle_golden.py).

Shapes follow the reference: values (B,T,P,K), returns (B,1|T,P,K),
rewards (B,T,P,K) or None, rhos/cs (B,T,1|P,1) broadcast over P and K.
"""

import numpy as np

ALGS = ('MC', 'TD', 'UPGO', 'VTRACE')


def _coefs(lmb, gamma):
    # Python-float x float32-tensor arithmetic rounds the scalar to float32;
    # (1 - lmb) and gamma * lmb are formed in double first (losses.py:24,51).
    return (np.float32(1 - lmb), np.float32(lmb), np.float32(gamma), np.float32(gamma * lmb))


def monte_carlo(values, returns):
    """losses.py:16-17"""
    return returns, returns - values


def temporal_difference(values, returns, rewards, lmb, gamma):
    """losses.py:20-28: tv[T-1] = returns[:,-1]; tv[i] = r[i] + g((1-l)v[i+1] + l tv[i+1])."""
    a, l, g, _ = _coefs(lmb, gamma)
    T = values.shape[1]
    tv = np.empty(np.broadcast_shapes(values.shape, returns[:, -1:].shape), dtype=np.float32)
    tv[:, T - 1] = returns[:, -1]
    for i in range(T - 2, -1, -1):
        x = g * (a * values[:, i + 1] + l * tv[:, i + 1])
        tv[:, i] = (rewards[:, i] + x) if rewards is not None else (np.float32(0) + x)
    return tv, tv - values


def upgo(values, returns, rewards, lmb, gamma):
    """losses.py:31-40: tv[i] = r[i] + g max(v[i+1], (1-l)v[i+1] + l tv[i+1])."""
    a, l, g, _ = _coefs(lmb, gamma)
    T = values.shape[1]
    tv = np.empty(np.broadcast_shapes(values.shape, returns[:, -1:].shape), dtype=np.float32)
    tv[:, T - 1] = returns[:, -1]
    for i in range(T - 2, -1, -1):
        v1 = values[:, i + 1]
        x = g * np.maximum(v1, a * v1 + l * tv[:, i + 1])
        tv[:, i] = (rewards[:, i] + x) if rewards is not None else (np.float32(0) + x)
    return tv, tv - values


def vtrace(values, returns, rewards, lmb, gamma, rhos, cs):
    """losses.py:43-58 (V-trace, IMPALA); rho is applied to the advantage by the caller."""
    _, _, g, gl = _coefs(lmb, gamma)
    r = rewards if rewards is not None else np.float32(0)
    v1 = np.concatenate([values[:, 1:], np.broadcast_to(returns[:, -1:], values[:, -1:].shape)], axis=1)
    deltas = rhos * ((r + g * v1) - values)
    T = values.shape[1]
    acc = np.empty_like(deltas)
    acc[:, T - 1] = deltas[:, -1]
    for i in range(T - 2, -1, -1):
        acc[:, i] = deltas[:, i] + (gl * cs[:, i]) * acc[:, i + 1]
    vs = acc + values
    vs1 = np.concatenate([vs[:, 1:], np.broadcast_to(returns[:, -1:], vs[:, -1:].shape)], axis=1)
    adv = (r + g * vs1) - values
    return vs, adv


def compute_target(algorithm, values, returns, rewards, lmb, gamma, rhos, cs):
    """losses.py:61-74 dispatch, including the values-is-None convention."""
    if values is None:
        return None, 0
    if algorithm == 'MC':
        return monte_carlo(values, returns)
    if algorithm == 'TD':
        return temporal_difference(values, returns, rewards, lmb, gamma)
    if algorithm == 'UPGO':
        return upgo(values, returns, rewards, lmb, gamma)
    if algorithm == 'VTRACE':
        return vtrace(values, returns, rewards, lmb, gamma, rhos, cs)
    raise ValueError('No algorithm named %s' % algorithm)
