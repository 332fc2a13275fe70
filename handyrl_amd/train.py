"""Learner math on MI355X — drop-in for the hot path of handyrl/train.py.

Public functions keep the reference signatures:

* ``forward_prediction(model, hidden, batch, args)``   train.py:136-185
* ``compose_losses(outputs, log_selected_policies, total_advantages, targets, batch, args)``
                                                       train.py:188-215
* ``compute_loss(batch, model, hidden, args) -> (losses, dcnt)``
                                                       train.py:218-258

The env network runs on PyTorch-ROCm.  Everything after it runs in the HIP
library (csrc/hrl_loss.hip): importance ratios, value preparation, the
return-target scans (the 2-4 ``compute_target`` calls of train.py:248-253
become one fused scan per value head), the advantages and the five loss sums
are one autograd Function whose backward is a single closed-form kernel.
``loss_terms`` is the sync-free core: it returns ``dcnt`` as a device tensor
so the learner step never waits on the host (the reference calls ``.item()``
at train.py:199 and :390).  ``compose_losses`` keeps the reference's
PyTorch formulation as a public function, and ``loss_terms_composed`` uses it
(with the HIP scans) for outputs the fused kernel does not take (value heads
wider than one scalar).
"""

import torch
import torch.distributions as dist
import torch.nn.functional as F

from . import _native
from .losses import compute_targets_fused
from .util import map_r, bimap_r, trimap_r

__all__ = ['forward_prediction', 'compose_losses', 'compute_loss', 'loss_terms', 'loss_terms_composed']


def forward_prediction(model, hidden, batch, args):
    """Network outputs over a (B, T, P, ...) batch (train.py:136-185).

    Feed-forward nets see all B*T*P' observations in one call; recurrent nets
    are unrolled over T with the hidden state masked by observation_mask and,
    in turn-based training without opponent observation, summed over players.
    Policies are reduced to the turn player and masked by action_mask; other
    heads are masked by observation_mask.
    """
    observations = batch['observation']
    tmask = batch['turn_mask']
    B, T = tmask.shape[:2]

    if hidden is None:
        obs = map_r(observations, lambda o: o.reshape(-1, *o.shape[3:]))
        outputs = model(obs, None)
    elif _flat_hidden_ok(hidden, tmask):
        outputs = _unroll_flat_hidden(model, hidden, batch, args)
    else:
        per_t = {}
        tbt_single = args['turn_based_training'] and not args['observation']
        for t in range(T):
            obs = map_r(observations, lambda o: o[:, t].reshape(-1, *o.shape[3:]))
            om_t = batch['observation_mask'][:, t]
            om = map_r(hidden, lambda h: om_t.view(*h.shape[:2], *([1] * (h.dim() - 2))))
            h_in = bimap_r(hidden, om, lambda h, m: h * m)
            if tbt_single:
                h_in = map_r(h_in, lambda h: h.sum(1))
            else:
                h_in = map_r(h_in, lambda h: h.reshape(-1, *h.shape[2:]))
            out_t = model(obs, h_in)
            next_hidden = None
            for k, o in out_t.items():
                if k == 'hidden':
                    next_hidden = o
                else:
                    per_t.setdefault(k, []).append(o)
            next_hidden = bimap_r(next_hidden, hidden, lambda nh, h: nh.view(h.shape[0], -1, *h.shape[2:]))
            hidden = trimap_r(hidden, next_hidden, om, lambda h, nh, m: h * (1 - m) + nh * m)
        outputs = {k: torch.stack(o, dim=1) for k, o in per_t.items() if o[0] is not None}

    result = {}
    fused = _output_mask_fusable(outputs, batch, B, T)
    if fused:
        result['policy'], result['value'] = _OutputMask.apply(
            outputs['policy'].view(B, T, -1, outputs['policy'].size(-1)),
            outputs['value'].view(B, T, -1, 1), tmask, batch['observation_mask'], batch['action_mask'])
    for k, o in outputs.items():
        if k == 'hidden' or o is None or (fused and k in ('policy', 'value')):
            continue
        o = o.view(B, T, -1, o.size(-1))
        if k == 'policy':
            result[k] = o.mul(tmask).sum(2, keepdim=True) - batch['action_mask']
        else:
            result[k] = o.mul(batch['observation_mask'])
    return result


def _output_mask_fusable(outputs, batch, B, T):
    """The common feed-forward case of the masking above, for _OutputMask: fp32 CUDA tensors, policy and
    value P-extents 1 or P, masks (B, T, P, 1), action_mask (B, T, 1, A)."""
    pol, val = outputs.get('policy'), outputs.get('value')
    if pol is None or val is None or not pol.is_cuda or pol.dtype != torch.float32 or val.dtype != torch.float32:
        return False
    tmask, omask, amask = batch['turn_mask'], batch['observation_mask'], batch['action_mask']
    if tmask.dim() != 4 or tmask.shape[-1] != 1 or omask.shape != tmask.shape:
        return False
    P, A = tmask.shape[2], pol.size(-1)
    if pol.numel() % (B * T * A) or val.size(-1) != 1 or val.numel() % (B * T):
        return False
    if pol.numel() // (B * T * A) not in (1, P) or val.numel() // (B * T) not in (1, P):
        return False
    if pol.numel() // (B * T * A) != val.numel() // (B * T):
        return False
    if tuple(amask.shape) != (B, T, 1, A) or amask.dtype != torch.float32:
        return False
    return all(t.is_contiguous() for t in (pol, val, tmask, omask, amask))


class _OutputMask(torch.autograd.Function):
    """train.py:176-183 for policy and value as csrc/hrl_loss.hip's out_mask kernels (one launch each way)."""

    @staticmethod
    def forward(ctx, opol, oval, tmask, omask, amask):
        B, T, Pq, A = opol.shape
        P = tmask.shape[2]
        pol = torch.empty(B, T, 1, A, dtype=opol.dtype, device=opol.device)
        val = torch.empty(B, T, P, 1, dtype=oval.dtype, device=oval.device)
        lib, p = _native.load(), _native.ptr
        _native.check(lib.hrl_output_mask_forward(p(opol), p(oval), p(tmask), p(omask), p(amask), B * T, P, Pq, A,
                                                  p(pol), p(val), _native.stream_of(opol.device)),
                      'hrl_output_mask_forward')
        ctx.save_for_backward(tmask, omask)
        ctx.pq, ctx.a = Pq, A
        return pol, val

    @staticmethod
    def backward(ctx, gpol, gval):
        tmask, omask = ctx.saved_tensors
        B, T, P = tmask.shape[:3]
        A = ctx.a
        gpol = torch.zeros(B, T, 1, A, dtype=tmask.dtype, device=tmask.device) if gpol is None else gpol.contiguous()
        gval = gval.contiguous() if gval is not None else None
        gopol = torch.empty(B, T, ctx.pq, A, dtype=gpol.dtype, device=gpol.device)
        goval = torch.empty(B, T, ctx.pq, 1, dtype=gpol.dtype, device=gpol.device) if gval is not None else None
        lib, p = _native.load(), _native.ptr
        _native.check(lib.hrl_output_mask_backward(p(gpol), p(gval) if gval is not None else None, p(tmask),
                                                   p(omask), B * T, P, ctx.pq, A, p(gopol),
                                                   p(goval) if goval is not None else None,
                                                   _native.stream_of(gpol.device)),
                      'hrl_output_mask_backward')
        return gopol, goval, None, None, None


def _leaves(x):
    if isinstance(x, (list, tuple)):
        return [l for v in x for l in _leaves(v)]
    if isinstance(x, dict):
        return [l for v in x.values() for l in _leaves(v)]
    return [x]


def _rebuild(template, it):
    if isinstance(template, (list, tuple)):
        return type(template)(_rebuild(v, it) for v in template)
    if isinstance(template, dict):
        return type(template)((k, _rebuild(v, it)) for k, v in template.items())
    return next(it)


FLAT_HIDDEN = True   # recurrent state plumbing through csrc/hrl_hidden.hip on the GPU (False: torch ops)
SEQUENCE_UNROLL = True   # nets with sequence_begin/step/end run their state-free parts once over all T


def _flat_hidden_ok(hidden, tmask):
    if not FLAT_HIDDEN:
        return False
    leaves = _leaves(hidden)
    if not (0 < len(leaves) <= 16) or not all(isinstance(h, torch.Tensor) for h in leaves):
        return False
    B, P = leaves[0].shape[:2]
    return (tmask.is_cuda and all(h.is_cuda and h.dtype == torch.float32 and h.dim() >= 2
                                  and tuple(h.shape[:2]) == (B, P) for h in leaves)
            and tmask.shape[0] == B and tmask.shape[2] == P)


# _unroll_flat_hidden's sequence path runs step t's state update and step t+1's gather as one fused Function
# (nn._HiddenUpdateGather); False: the two Functions (bit-identical; tests/test_geister.py)
FUSE_UPDATE_GATHER = True


def _unroll_flat_hidden(model, hidden, batch, args):
    """The recurrent branch on the GPU: the masking/summing and the mixing of every hidden tensor
    run as one HIP launch each per step (nn._HiddenGather / _HiddenUpdate), with the arithmetic of
    the torch formulation below (train.py:155-174).  The tensors stay separate autograd values, so
    state that never reaches an output is pruned exactly as with the torch ops."""
    from .nn import _HiddenGather, _HiddenUpdate
    observations = batch['observation']
    tmask = batch['turn_mask']
    B, T, P = tmask.shape[:3]
    leaves = _leaves(hidden)
    n = len(leaves)
    masks = batch['observation_mask'].reshape(B, T, P).transpose(0, 1).contiguous()   # (T, B, P)
    summed = args['turn_based_training'] and not args['observation']
    seq_ok = getattr(model, 'sequence_ok', None)
    if SEQUENCE_UNROLL and seq_ok is not None and seq_ok(map_r(observations, lambda o: o[:, 0])):
        # the net runs its state-free parts once over all T steps (e.g. GeisterNet.sequence_begin/end):
        # observations time-major, (T*N, ...) with N = B*P' in the per-step order
        from .nn import _HiddenUpdateGather
        obs = map_r(observations, lambda o: o.transpose(0, 1).reshape(-1, *o.shape[3:]))
        seq = model.sequence_begin(obs, T)
        h_lasts = []
        g = _HiddenGather.apply(masks[0], summed, B, P, *leaves)
        for t in range(T):
            m = masks[t]
            h_in = _rebuild(hidden, iter(g[:n]))
            h_last, next_hidden = model.sequence_step(seq, t, h_in)
            nh = _leaves(next_hidden)
            Pn = nh[0].shape[0] // B
            # the state continues through the gather's pass-through views, and the step output that is also a
            # new state leaf comes back from the update: every tensor has one consumer, the adjoints add
            k = next((i for i, x in enumerate(nh) if x is h_last), -1)
            if FUSE_UPDATE_GATHER and t + 1 < T:
                # this step's update and the next step's gather in one launch each way
                u = _HiddenUpdateGather.apply(m, masks[t + 1], summed, B, P, Pn, n, k, *g[n:], *nh)
                g = u[:2 * n]
                h_lasts.append(u[2 * n] if k >= 0 else h_last)
                continue
            u = _HiddenUpdate.apply(m, B, P, Pn, n, k, *g[n:], *nh)
            leaves = list(u[:n])
            h_lasts.append(u[n] if k >= 0 else h_last)
            if t + 1 < T:
                g = _HiddenGather.apply(masks[t + 1], summed, B, P, *leaves)
        out = model.sequence_end(seq, h_lasts)
        # (T*N, ...) -> (N, T, ...), the per-step loop's torch.stack(dim=1) layout
        return {k: o.view(T, -1, *o.shape[1:]).transpose(0, 1).contiguous() for k, o in out.items()
                if o is not None}
    per_t = {}
    for t in range(T):
        obs = map_r(observations, lambda o: o[:, t].reshape(-1, *o.shape[3:]))
        m = masks[t]
        g = _HiddenGather.apply(m, summed, B, P, *leaves)
        h_in = _rebuild(hidden, iter(g[:n]))
        out_t = model(obs, h_in)
        next_hidden = None
        for k, o in out_t.items():
            if k == 'hidden':
                next_hidden = o
            else:
                per_t.setdefault(k, []).append(o)
        nh = _leaves(next_hidden)
        Pn = nh[0].shape[0] // B
        leaves = list(_HiddenUpdate.apply(m, B, P, Pn, n, -1, *g[n:], *nh))
    return {k: torch.stack(o, dim=1) for k, o in per_t.items() if o[0] is not None}


def compose_losses(outputs, log_selected_policies, total_advantages, targets, batch, args):
    """Summed policy / value / return / entropy losses (train.py:188-215).

    Returns ``(losses, dcnt)`` with ``dcnt`` a Python float, as the reference
    (``tmasks.sum().item()``, train.py:199); the learner's sync-free path uses
    ``_compose_losses``, whose ``dcnt`` stays a 0-d device tensor.
    """
    losses, dcnt = _compose_losses(outputs, log_selected_policies, total_advantages, targets, batch, args)
    return losses, dcnt.item()


def _compose_losses(outputs, log_selected_policies, total_advantages, targets, batch, args):
    """compose_losses with ``dcnt`` as a 0-d device tensor (no host sync)."""
    tmasks = batch['turn_mask']
    omasks = batch['observation_mask']

    losses = {}
    dcnt = tmasks.sum()
    turn_advantages = total_advantages.mul(tmasks).sum(2, keepdim=True)

    losses['p'] = (-log_selected_policies * turn_advantages).sum()
    if 'value' in outputs:
        losses['v'] = ((outputs['value'] - targets['value']) ** 2).mul(omasks).sum() / 2
    if 'return' in outputs:
        losses['r'] = F.smooth_l1_loss(outputs['return'], targets['return'], reduction='none').mul(omasks).sum()

    entropy = dist.Categorical(logits=outputs['policy'], validate_args=False).entropy().mul(tmasks.sum(-1))
    losses['ent'] = entropy.sum()

    base_loss = losses['p'] + losses.get('v', 0) + losses.get('r', 0)
    entropy_loss = entropy.mul(1 - batch['progress'] * (1 - args['entropy_regularization_decay'])).sum() \
        * -args['entropy_regularization']
    losses['total'] = base_loss + entropy_loss
    return losses, dcnt


class _FusedLoss(torch.autograd.Function):
    """train.py:220-258 + compose_losses as csrc/hrl_loss.hip (forward 5 launches, backward 1)."""

    @staticmethod
    def forward(ctx, tpol, value, ret_out, bpol, action, emask, tmask, omask, progress, outcome, ret, reward,
                cfg):
        B, T, Pp, A = tpol.shape
        P = tmask.shape[2]
        lib = _native.load()
        ws_bytes = lib.hrl_loss_workspace_bytes(B, T, P, Pp)
        ws = torch.empty(ws_bytes, dtype=torch.uint8, device=tpol.device)
        losses = torch.empty(6, dtype=torch.float32, device=tpol.device)
        p = _native.ptr
        code = lib.hrl_loss_forward(
            p(tpol), p(bpol), p(action), B, T, P, Pp, A, p(emask), p(tmask), p(omask), p(progress),
            p(value), p(outcome), p(ret_out), p(ret), p(reward),
            cfg['value_target'], cfg['policy_target'], cfg['symmetrize'], cfg['lambda'], cfg['gamma'],
            cfg['ent_coef'], cfg['ent_decay'], p(ws), ws_bytes, p(losses), _native.stream_of(tpol.device))
        _native.check(code, 'hrl_loss_forward')
        ctx.cfg = cfg
        ctx.has_value, ctx.has_ret = value is not None, ret_out is not None
        ctx.save_for_backward(tpol, value, ret_out, action, emask, tmask, omask, progress, ws)
        return losses

    @staticmethod
    def backward(ctx, dlosses):
        tpol, value, ret_out, action, emask, tmask, omask, progress, ws = ctx.saved_tensors
        B, T, Pp, A = tpol.shape
        P = tmask.shape[2]
        dl = dlosses[:5].contiguous()
        g_tpol = torch.empty_like(tpol)
        g_value = torch.empty_like(value) if ctx.has_value else None
        g_ret = torch.empty_like(ret_out) if ctx.has_ret else None
        p = _native.ptr
        lib = _native.load()
        code = lib.hrl_loss_backward(
            p(tpol), p(action), B, T, P, Pp, A, p(emask), p(tmask), p(omask), p(progress),
            p(value), p(ret_out), ctx.cfg['ent_coef'], ctx.cfg['ent_decay'], p(ws), ws.numel(), p(dl),
            p(g_tpol), p(g_value), p(g_ret), _native.stream_of(tpol.device))
        _native.check(code, 'hrl_loss_backward')
        return (g_tpol, g_value, g_ret) + (None,) * 10


def _fusable(outputs, batch):
    pol = outputs.get('policy')
    if pol is None or not pol.is_cuda or pol.dtype != torch.float32 or pol.dim() != 4:
        return False
    for k in ('value', 'return'):
        o = outputs.get(k)
        if o is not None and (o.dim() != 4 or o.shape[-1] != 1 or o.dtype != torch.float32):
            return False
    P = batch['turn_mask'].shape[2]
    return pol.shape[2] in (1, P) and batch['turn_mask'].shape[-1] == 1


def loss_terms(outputs, batch, args):
    """train.py:220-258 and compose_losses on the HIP kernels; (losses, dcnt tensor), no host sync."""
    if not _fusable(outputs, batch):
        return loss_terms_composed(outputs, batch, args)
    alg = _native.ALG
    for k in ('value_target', 'policy_target'):
        if args[k] not in alg:
            raise ValueError('No algorithm named %s' % args[k])
    value, ret_out = outputs.get('value'), outputs.get('return')
    P = batch['turn_mask'].shape[2]
    cfg = {'value_target': alg[args['value_target']], 'policy_target': alg[args['policy_target']],
           'symmetrize': int(bool(args['turn_based_training']) and value is not None and P == 2),
           'lambda': float(args['lambda']), 'gamma': float(args['gamma']),
           'ent_coef': float(args['entropy_regularization']),
           'ent_decay': float(args['entropy_regularization_decay'])}
    c = lambda t: None if t is None else t.contiguous()  # noqa: E731
    with_ret = ret_out is not None
    vec = _FusedLoss.apply(c(outputs['policy']), c(value), c(ret_out), c(batch['policy'].detach()),
                           c(batch['action']), c(batch['episode_mask']), c(batch['turn_mask']),
                           c(batch['observation_mask']), c(batch['progress']),
                           c(batch['outcome']) if value is not None else None,
                           c(batch['return']) if with_ret else None, c(batch['reward']) if with_ret else None, cfg)
    losses = {'p': vec[0]}
    if value is not None:
        losses['v'] = vec[1]
    if with_ret:
        losses['r'] = vec[2]
    losses['ent'] = vec[3]
    total = vec[4]
    total._hrl_loss_vec = vec   # backward_total seeds the vector itself
    losses['total'] = total
    return losses, vec[5].detach()


_SEEDS = {}


def backward_total(losses, inputs=None, retain_graph=None):
    """``losses['total'].backward()``.  For the fused loss (loss_terms) the backward starts at the loss
    vector with a persistent one-hot seed on its total: autograd's ones fill for the scalar and the
    select backward's zeros fill and copy (three launches per step) do not run."""
    total = losses['total']
    vec = getattr(total, '_hrl_loss_vec', None)
    if vec is None:
        torch.autograd.backward(total, inputs=inputs, retain_graph=retain_graph)
        return
    key = (vec.device, vec.dtype)
    seed = _SEEDS.get(key)
    if seed is None:
        seed = torch.zeros(6, dtype=vec.dtype, device=vec.device)
        seed[4] = 1.0
        # cached only when made outside a graph capture (the eager warm-up): a seed made inside one lives in
        # the capture's pool and is the capture's own
        if not (vec.is_cuda and torch.cuda.is_current_stream_capturing()):
            _SEEDS[key] = seed
    torch.autograd.backward(vec, grad_tensors=seed, inputs=inputs, retain_graph=retain_graph)


def loss_terms_composed(outputs, batch, args):
    """IS ratios, value symmetrisation, fused HIP target scans, PyTorch-composed losses.

    train.py:220-258 without host synchronisation, for any output shapes.
    """
    actions = batch['action']
    emasks = batch['episode_mask']

    log_sel_b = F.log_softmax(batch['policy'], dim=-1).gather(-1, actions) * emasks
    log_sel_t = F.log_softmax(outputs['policy'], dim=-1).gather(-1, actions) * emasks

    rhos = torch.exp(log_sel_t.detach() - log_sel_b)
    clipped_rhos = torch.clamp(rhos, 0, 1.0)
    cs = torch.clamp(rhos, 0, 1.0)

    nograd = {k: o.detach() for k, o in outputs.items()}
    if 'value' in nograd:
        v = nograd['value']
        if args['turn_based_training'] and v.size(2) == 2:  # two-player zero-sum
            v_opp = -torch.stack([v[:, :, 1], v[:, :, 0]], dim=2)
            v = (v + v_opp) / (batch['observation_mask'].sum(dim=2, keepdim=True) + 1e-8)
        nograd['value'] = v * emasks + batch['outcome'] * (1 - emasks)

    lmb, gamma = args['lambda'], args['gamma']
    targets, advantages = {}, {}
    targets['value'], advantages['value'] = compute_targets_fused(
        args['value_target'], args['policy_target'],
        nograd.get('value'), batch['outcome'], None, lmb, 1, clipped_rhos, cs)
    targets['return'], advantages['return'] = compute_targets_fused(
        args['value_target'], args['policy_target'],
        nograd.get('return'), batch['return'], batch['reward'], lmb, gamma, clipped_rhos, cs)

    total_advantages = clipped_rhos * sum(advantages.values())
    return _compose_losses(outputs, log_sel_t, total_advantages, targets, batch, args)


def compute_loss(batch, model, hidden, args):
    """Drop-in for handyrl.train.compute_loss (train.py:218-258)."""
    outputs = forward_prediction(model, hidden, batch, args)
    losses, dcnt = loss_terms(outputs, batch, args)
    return losses, dcnt.item()
