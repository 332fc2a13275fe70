"""Return targets and advantages on MI355X — drop-in for handyrl/losses.py.

``compute_target`` keeps the reference signature and conventions
(handyrl/losses.py:61-74):

* ``values is None``      -> ``(None, 0)``                    (losses.py:62-63)
* ``rewards is None``     -> rewards treated as 0             (losses.py:23,35,44)
* ``returns`` may have time extent 1 (the outcome); TD / UPGO / VTRACE read
  only ``returns[:, -1]``                                      (losses.py:21,32,45)
* ``rhos`` / ``cs`` broadcast over players when their player extent is 1
* MC returns ``returns`` itself as the target                  (losses.py:17)
* an unknown algorithm raises ``ValueError`` (the reference prints
  'No algorithm named ...' and returns None, which its caller then fails to
  unpack, losses.py:73-74)

Every recurrence runs in ONE launch of the HIP scan kernel
(csrc/hrl_targets.hip) through the C ABI of include/hrl_targets.h; the
outputs are detached, like the reference's (its callers pass detached
tensors, train.py:232).  There is no CPU path: CPU tensors are rejected.
"""

import torch

from . import _native

__all__ = ['compute_target', 'compute_targets_fused', 'target_layout']


def _alg_id(algorithm):
    alg = _native.ALG.get(algorithm)
    if alg is None:
        raise ValueError('No algorithm named %s' % algorithm)
    return alg


def _as_f32(t, name, device):
    if not isinstance(t, torch.Tensor):
        raise TypeError('%s must be a torch.Tensor' % name)
    if t.device != device:
        raise ValueError('%s is on %s, values on %s' % (name, t.device, device))
    if t.dtype != torch.float32:
        raise TypeError('%s must be float32 (got %s)' % (name, t.dtype))
    return t.detach().contiguous()


def target_layout(values, returns, rewards, rhos, cs):
    """Validate shapes and flatten to the kernel layout.

    Returns ``(v, ret, rew, rho, c, dims)`` with ``dims = (B, T, C, ret_T,
    rho_C, rho_div)``: values (B,T,C) with C = prod(values.shape[2:]);
    returns (B, 1|T, C); rhos/cs (B, T, rho_C) where value column ``c`` reads
    rho column ``c // rho_div``.
    """
    if values.dim() < 2:
        raise ValueError('values must be (B, T, ...), got %s' % (tuple(values.shape),))
    dev = values.device
    if dev.type != 'cuda':
        raise RuntimeError('handyrl_amd.compute_target runs on the GPU only (got a %s tensor)' % dev.type)
    B, T = values.shape[:2]
    rest = tuple(values.shape[2:])
    C = 1
    for d in rest:
        C *= d
    v = _as_f32(values, 'values', dev)

    ret = _as_f32(returns, 'returns', dev)
    if ret.dim() != values.dim() or ret.shape[0] != B or ret.shape[1] not in (1, T):
        raise ValueError('returns must be (B, 1|T, ...) matching values %s, got %s'
                         % (tuple(values.shape), tuple(returns.shape)))
    if tuple(ret.shape[2:]) != rest:
        ret = ret.expand(B, ret.shape[1], *rest).contiguous()
    ret_T = ret.shape[1]

    rew = None
    if rewards is not None:
        rew = _as_f32(rewards, 'rewards', dev)
        if tuple(rew.shape) != tuple(values.shape):
            rew = rew.expand(values.shape).contiguous()

    rho = c = None
    rho_C, rho_div = 1, C
    if rhos is not None and cs is not None:
        rho = _as_f32(rhos, 'rhos', dev)
        c = _as_f32(cs, 'cs', dev)
        if rho.shape != c.shape:
            c = c.expand(rho.shape).contiguous() if c.dim() == rho.dim() else c
        rshape = tuple(rho.shape)
        if rho.dim() != values.dim() or rshape[:2] != (B, T):
            raise ValueError('rhos must be (B, T, ...) matching values %s, got %s'
                             % (tuple(values.shape), rshape))
        rrest = rshape[2:]
        if all(d == 1 for d in rrest):
            rho_C, rho_div = 1, C                        # broadcast over every value column
        elif len(rest) >= 1 and rrest[0] == rest[0] and all(d == 1 for d in rrest[1:]):
            rho_C, rho_div = rest[0], C // rest[0]       # per player, broadcast over K
        else:
            rho = rho.expand(values.shape).contiguous()  # general broadcast: materialise
            c = c.expand(values.shape).contiguous()
            rho_C, rho_div = C, 1
        rho = rho.reshape(B, T, rho_C)
        c = c.reshape(B, T, rho_C)
    return v, ret, rew, rho, c, (B, T, C, ret_T, rho_C, rho_div)


def compute_targets_fused(target_algorithm, adv_algorithm, values, returns, rewards, lmb, gamma, rhos, cs):
    """One pass producing ``target_algorithm``'s targets and ``adv_algorithm``'s advantages.

    This is the learner's form of train.py:248-253: the reference calls
    compute_target for value_target (keeping targets and advantages) and,
    when policy_target differs, again for policy_target (keeping only the
    advantages).  Returns ``(targets, advantages)`` with the reference's
    shapes; ``(None, 0)`` when ``values is None``.
    """
    if values is None:
        return None, 0
    tgt_alg = _alg_id(target_algorithm)
    adv_alg = _alg_id(adv_algorithm)
    need_rho = 'VTRACE' in (target_algorithm, adv_algorithm)
    if need_rho and (rhos is None or cs is None):
        raise ValueError('VTRACE needs rhos and cs')
    v, ret, rew, rho, c, (B, T, C, ret_T, rho_C, rho_div) = target_layout(
        values, returns, rewards, rhos if need_rho else None, cs if need_rho else None)
    out_shape = tuple(values.shape)
    adv = torch.empty(out_shape, dtype=torch.float32, device=values.device)
    tgt = None if target_algorithm == 'MC' else torch.empty(out_shape, dtype=torch.float32, device=values.device)
    lib = _native.load()
    code = lib.hrl_compute_targets_fused(
        tgt_alg, adv_alg, _native.ptr(v), _native.ptr(ret), _native.ptr(rew), _native.ptr(rho), _native.ptr(c),
        B, T, C, ret_T, rho_C, rho_div, float(lmb), float(gamma), _native.ptr(tgt), _native.ptr(adv),
        _native.stream_of(values.device))
    _native.check(code, 'hrl_compute_targets_fused(%s, %s)' % (target_algorithm, adv_algorithm))
    if tgt is None:
        tgt = returns  # MC: the target IS returns (losses.py:17)
    return tgt, adv


def compute_target(algorithm, values, returns, rewards, lmb, gamma, rhos, cs):
    """Drop-in for handyrl.losses.compute_target (losses.py:61-74) on the GPU."""
    if values is None:
        return None, 0
    alg = _alg_id(algorithm)
    need_rho = algorithm == 'VTRACE'
    if need_rho and (rhos is None or cs is None):
        raise ValueError('VTRACE needs rhos and cs')
    v, ret, rew, rho, c, (B, T, C, ret_T, rho_C, rho_div) = target_layout(
        values, returns, rewards, rhos if need_rho else None, cs if need_rho else None)
    out_shape = tuple(values.shape)
    adv = torch.empty(out_shape, dtype=torch.float32, device=values.device)
    tgt = None if algorithm == 'MC' else torch.empty(out_shape, dtype=torch.float32, device=values.device)
    lib = _native.load()
    code = lib.hrl_compute_target(
        alg, _native.ptr(v), _native.ptr(ret), _native.ptr(rew), _native.ptr(rho), _native.ptr(c),
        B, T, C, ret_T, rho_C, rho_div, float(lmb), float(gamma), _native.ptr(tgt), _native.ptr(adv),
        _native.stream_of(values.device))
    _native.check(code, 'hrl_compute_target(%s)' % algorithm)
    if tgt is None:
        tgt = returns
    return tgt, adv
