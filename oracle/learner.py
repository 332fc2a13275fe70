"""CPU restatement of the reference learner step — TEST INFRASTRUCTURE ONLY.

Restates, on the CPU with torch fp32 (autograd for the backward):
  * forward_prediction        handyrl/train.py:136-185
  * compute_loss              handyrl/train.py:218-258 (scans via oracle.targets)
  * compose_losses            handyrl/train.py:188-215
  * one Trainer.train step    handyrl/train.py:375-385
Pinned by tests/test_oracle_golden.py against the reference's own outputs
(tests/golden/loss.*, learner.*).  Used by the GPU parity tests as the checker
and by bench.py's cpu_baseline leg as the timed CPU learner ("port").
"""

import numpy as np
import torch
import torch.distributions as dist
import torch.nn as nn
import torch.nn.functional as F

from . import targets as ot


def _map(x, fn):
    if isinstance(x, (list, tuple)):
        return type(x)(_map(v, fn) for v in x)
    if isinstance(x, dict):
        return {k: _map(v, fn) for k, v in x.items()}
    return fn(x)


def _map2(x, y, fn):
    if isinstance(x, (list, tuple)):
        return type(x)(_map2(v, y[i], fn) for i, v in enumerate(x))
    if isinstance(x, dict):
        return {k: _map2(v, y[k], fn) for k, v in x.items()}
    return fn(x, y)


def _map3(x, y, z, fn):
    if isinstance(x, (list, tuple)):
        return type(x)(_map3(v, y[i], z[i], fn) for i, v in enumerate(x))
    if isinstance(x, dict):
        return {k: _map3(v, y[k], z[k], fn) for k, v in x.items()}
    return fn(x, y, z)


def forward_prediction(model, hidden, batch, args):
    """train.py:136-185"""
    obs_all = batch['observation']
    tm = batch['turn_mask']
    if hidden is None:
        outputs = model(_map(obs_all, lambda o: o.view(-1, *o.size()[3:])), None)
    else:
        seq = {}
        for t in range(tm.size(1)):
            obs = _map(obs_all, lambda o: o[:, t].reshape(-1, *o.size()[3:]))
            om_ = batch['observation_mask'][:, t]
            om = _map(hidden, lambda h: om_.view(*h.size()[:2], *([1] * (len(h.size()) - 2))))
            h_ = _map2(hidden, om, lambda h, m: h * m)
            if args['turn_based_training'] and not args['observation']:
                h_ = _map(h_, lambda h: h.sum(1))
            else:
                h_ = _map(h_, lambda h: h.view(-1, *h.size()[2:]))
            out = model(obs, h_)
            for k, o in out.items():
                if k == 'hidden':
                    nh = o
                else:
                    seq[k] = seq.get(k, []) + [o]
            nh = _map2(nh, hidden, lambda a, h: a.view(h.size(0), -1, *h.size()[2:]))
            hidden = _map3(hidden, nh, om, lambda h, a, m: h * (1 - m) + a * m)
        outputs = {k: torch.stack(o, dim=1) for k, o in seq.items() if o[0] is not None}
    res = {}
    for k, o in outputs.items():
        if k == 'hidden':
            continue
        o = o.view(*tm.size()[:2], -1, o.size(-1))
        if k == 'policy':
            res[k] = o.mul(tm).sum(2, keepdim=True) - batch['action_mask']
        else:
            res[k] = o.mul(batch['observation_mask'])
    return res


def _target(alg, values, returns, rewards, lmb, gamma, rhos, cs):
    if values is None:
        return None, 0
    f = lambda x: None if x is None else x.detach().numpy()  # noqa: E731
    t, a = ot.compute_target(alg, f(values), f(returns), f(rewards), lmb, gamma, f(rhos), f(cs))
    return torch.from_numpy(np.ascontiguousarray(t)), torch.from_numpy(np.ascontiguousarray(a))


def compose_losses(outputs, log_sel, total_adv, targets, batch, args):
    """train.py:188-215"""
    tm, om = batch['turn_mask'], batch['observation_mask']
    losses = {}
    dcnt = tm.sum().item()
    turn_adv = total_adv.mul(tm).sum(2, keepdim=True)
    losses['p'] = (-log_sel * turn_adv).sum()
    if 'value' in outputs:
        losses['v'] = ((outputs['value'] - targets['value']) ** 2).mul(om).sum() / 2
    if 'return' in outputs:
        losses['r'] = F.smooth_l1_loss(outputs['return'], targets['return'], reduction='none').mul(om).sum()
    ent = dist.Categorical(logits=outputs['policy']).entropy().mul(tm.sum(-1))
    losses['ent'] = ent.sum()
    base = losses['p'] + losses.get('v', 0) + losses.get('r', 0)
    ent_loss = ent.mul(1 - batch['progress'] * (1 - args['entropy_regularization_decay'])).sum() \
        * -args['entropy_regularization']
    losses['total'] = base + ent_loss
    return losses, dcnt


def loss_from_outputs(outputs, batch, args, record=None):
    """train.py:220-258 given the network outputs."""
    act, em = batch['action'], batch['episode_mask']
    lb = F.log_softmax(batch['policy'], dim=-1).gather(-1, act) * em
    lt = F.log_softmax(outputs['policy'], dim=-1).gather(-1, act) * em
    rhos = torch.exp(lt.detach() - lb)
    crho = torch.clamp(rhos, 0, 1.0)
    cs = torch.clamp(rhos, 0, 1.0)
    ng = {k: o.detach() for k, o in outputs.items()}
    if 'value' in ng:
        v = ng['value']
        if args['turn_based_training'] and v.size(2) == 2:
            v_opp = -torch.stack([v[:, :, 1], v[:, :, 0]], dim=2)
            v = (v + v_opp) / (batch['observation_mask'].sum(dim=2, keepdim=True) + 1e-8)
        ng['value'] = v * em + batch['outcome'] * (1 - em)
    vargs = ng.get('value', None), batch['outcome'], None, args['lambda'], 1, crho, cs
    rargs = ng.get('return', None), batch['return'], batch['reward'], args['lambda'], args['gamma'], crho, cs
    targets, advs = {}, {}
    targets['value'], advs['value'] = _target(args['value_target'], *vargs)
    targets['return'], advs['return'] = _target(args['value_target'], *rargs)
    if args['policy_target'] != args['value_target']:
        _, advs['value'] = _target(args['policy_target'], *vargs)
        _, advs['return'] = _target(args['policy_target'], *rargs)
    total_adv = crho * sum(advs.values())
    if record is not None:
        record.update(log_sel=lt.detach(), total_adv=total_adv, targets=targets, rhos=crho)
    return compose_losses(outputs, lt, total_adv, targets, batch, args)


def compute_loss(batch, model, hidden, args):
    """train.py:218-258"""
    return loss_from_outputs(forward_prediction(model, hidden, batch, args), batch, args)


class CpuLearner:
    """The reference learner step on the CPU (train.py:375-385)."""

    def __init__(self, net, args, lr=None):
        self.net = net
        self.args = args
        self.params = list(net.parameters())
        if lr is None:
            lr = 3e-8 * args['batch_size'] * args['forward_steps']
        self.opt = torch.optim.Adam(self.params, lr=lr, weight_decay=1e-5)

    def step(self, batch, hidden=None):
        self.net.train()
        losses, dcnt = compute_loss(batch, self.net, hidden, self.args)
        self.opt.zero_grad()
        losses['total'].backward()
        gn = nn.utils.clip_grad_norm_(self.params, 4.0)
        self.opt.step()
        out = {k: float(v.item()) for k, v in losses.items()}
        out['dcnt'] = dcnt
        out['grad_norm'] = float(gn)
        return out
