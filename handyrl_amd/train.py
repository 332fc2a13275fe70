"""Learner math on MI355X — drop-in for the hot path of handyrl/train.py.

Public functions keep the reference signatures:

* ``forward_prediction(model, hidden, batch, args)``   train.py:136-185
* ``compose_losses(outputs, log_selected_policies, total_advantages, targets, batch, args)``
                                                       train.py:188-215
* ``compute_loss(batch, model, hidden, args) -> (losses, dcnt)``
                                                       train.py:218-258

The env network runs on PyTorch-ROCm.  The return-target scans run in the HIP
library: the 2-4 ``compute_target`` calls of train.py:248-253 become ONE
fused launch per value head (``compute_targets_fused``: value_target's
targets + policy_target's advantages).  ``loss_terms`` is the sync-free core:
it returns ``dcnt`` as a device tensor so the learner step never waits on the
host (the reference calls ``.item()`` at train.py:199 and :390).
"""

import torch
import torch.distributions as dist
import torch.nn.functional as F

from .losses import compute_targets_fused
from .util import map_r, bimap_r, trimap_r

__all__ = ['forward_prediction', 'compose_losses', 'compute_loss', 'loss_terms']


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
    for k, o in outputs.items():
        if k == 'hidden' or o is None:
            continue
        o = o.view(B, T, -1, o.size(-1))
        if k == 'policy':
            result[k] = o.mul(tmask).sum(2, keepdim=True) - batch['action_mask']
        else:
            result[k] = o.mul(batch['observation_mask'])
    return result


def compose_losses(outputs, log_selected_policies, total_advantages, targets, batch, args):
    """Summed policy / value / return / entropy losses (train.py:188-215).

    Returns ``(losses, dcnt)`` with ``dcnt`` a 0-d device tensor (the
    reference returns ``tmasks.sum().item()``; ``compute_loss`` converts).
    """
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


def loss_terms(outputs, batch, args):
    """IS ratios, value symmetrisation, fused HIP target scans, composed losses.

    train.py:220-258 without host synchronisation.
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
    return compose_losses(outputs, log_sel_t, total_advantages, targets, batch, args)


def compute_loss(batch, model, hidden, args):
    """Drop-in for handyrl.train.compute_loss (train.py:218-258)."""
    outputs = forward_prediction(model, hidden, batch, args)
    losses, dcnt = loss_terms(outputs, batch, args)
    return losses, dcnt.item()
