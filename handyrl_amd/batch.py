"""Training-batch assembly: the learner's input contract.

``make_batch(episodes, args)`` keeps the signature, the episode wire format
and the output layout of handyrl/train.py:33-133, so a reference Batcher can
feed the MI355X learner unchanged:

* an episode window is ``{'moment': [bz2(pickle(list of moments)), ...],
  'base', 'start', 'end', 'total', 'outcome', 'args'}`` (generation.py:79-86,
  train.py:296-301);
* the output maps key -> tensor of shape (B, T, P, ...):
  observation (B,T,P',*obs) [nested dict/list observations keep their
  structure], policy (B,T,P',A), value/reward/return (B,T,P,1), action
  (B,T,P',1) int64, outcome (B,1,P,1), episode_mask (B,T,1,1),
  turn_mask/observation_mask (B,T,P,1), action_mask (B,T,P',A), progress
  (B,T,1), with P' = 1 in turn-based training without opponent observation;
* windows shorter than forward_steps are padded as the reference pads them:
  zeros, except value (padded with the outcome), action_mask (1e32) and
  progress (1).

Solo training (turn_based_training=False) draws the trained player with
``random.choice`` once per episode, in the reference's order, so a seeded
``random`` reproduces the reference's batch exactly.
"""

import bz2
import pickle
import random

import numpy as np
import torch

__all__ = ['make_batch', 'episode_moments']


def episode_moments(ep):
    """The window's moments: decompressed blocks, cut to [start, end) (train.py:54-55)."""
    moments = []
    for block in ep['moment']:
        moments.extend(pickle.loads(bz2.decompress(block)))
    return moments[ep['start'] - ep['base']:ep['end'] - ep['base']]


def _leaf_map(fn, x):
    if isinstance(x, dict):
        return {k: _leaf_map(fn, v) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return type(x)(_leaf_map(fn, v) for v in x)
    return fn(x)


def _stack(template, items):
    """Stack structures shaped like `template` leaf by leaf (np.stack along a new axis 0)."""
    if isinstance(template, dict):
        return {k: _stack(v, [it[k] for it in items]) for k, v in template.items()}
    if isinstance(template, (list, tuple)):
        return type(template)(_stack(v, [it[i] for it in items]) for i, v in enumerate(template))
    return np.stack([np.asarray(it) for it in items])


def _pad_time(a, n, value):
    return np.concatenate([a, np.full((n,) + a.shape[1:], value, dtype=a.dtype)])


def _window(ep, args):
    moments = episode_moments(ep)
    players = list(moments[0]['observation'].keys())
    if not args['turn_based_training']:   # solo training: one random player (train.py:57-58)
        players = [random.choice(players)]
    first = moments[0]['turn'][0]
    obs_zero = _leaf_map(np.zeros_like, moments[0]['observation'][first])
    pol_zero = np.zeros_like(moments[0]['policy'][first])

    def pick(m, key, player, default):
        v = m[key][player]
        return default if v is None else v

    if args['turn_based_training'] and not args['observation']:
        slots = [[m['turn'][0]] for m in moments]        # the turn player only (P' = 1)
        obs = [[m['observation'][s[0]]] for m, s in zip(moments, slots)]
        pol = np.array([[m['policy'][s[0]]] for m, s in zip(moments, slots)])
        act = np.array([[m['action'][s[0]]] for m, s in zip(moments, slots)], dtype=np.int64)[..., None]
        amask = np.array([[m['action_mask'][s[0]]] for m, s in zip(moments, slots)])
    else:
        obs = [[pick(m, 'observation', p, obs_zero) for p in players] for m in moments]
        pol = np.array([[pick(m, 'policy', p, pol_zero) for p in players] for m in moments])
        act = np.array([[pick(m, 'action', p, 0) for p in players] for m in moments], dtype=np.int64)[..., None]
        amask = np.array([[pick(m, 'action_mask', p, pol_zero + 1e32) for p in players] for m in moments])

    T, P = len(moments), len(players)
    obs = _stack(obs_zero, [_stack(obs_zero, row) for row in obs])          # (T, P', ...)

    def per_player(key):
        return np.array([[pick(m, key, p, [0]) for p in players] for m in moments],
                        dtype=np.float32).reshape(T, P, -1)

    val, rew, ret = per_player('value'), per_player('reward'), per_player('return')
    oc = np.array([ep['outcome'][p] for p in players], dtype=np.float32).reshape(1, P, -1)
    emask = np.ones((T, 1, 1), dtype=np.float32)
    tmask = np.array([[[m['policy'][p] is not None] for p in players] for m in moments], dtype=np.float32)
    omask = np.array([[[m['value'][p] is not None] for p in players] for m in moments], dtype=np.float32)
    progress = np.arange(ep['start'], ep['end'], dtype=np.float32)[..., None] / ep['total']

    pad = args['forward_steps'] - T
    if pad > 0:                                                           # train.py:92-104
        obs = _leaf_map(lambda o: _pad_time(o, pad, 0), obs)
        pol = _pad_time(pol, pad, 0)
        val = np.concatenate([val, np.tile(oc, [pad, 1, 1])])
        act = _pad_time(act, pad, 0)
        rew, ret = _pad_time(rew, pad, 0), _pad_time(ret, pad, 0)
        emask, tmask, omask = _pad_time(emask, pad, 0), _pad_time(tmask, pad, 0), _pad_time(omask, pad, 0)
        amask = _pad_time(amask, pad, 1e32)
        progress = _pad_time(progress, pad, 1)
    return obs_zero, obs, (pol, val, act, oc, rew, ret, emask, tmask, omask, amask, progress)


def make_batch(episodes, args):
    """Drop-in for handyrl.train.make_batch (train.py:33-133): dict of CPU tensors."""
    obss, cols, template = [], [], None
    for ep in episodes:
        template, obs, data = _window(ep, args)
        obss.append(obs)
        cols.append(data)
    names = ('policy', 'value', 'action', 'outcome', 'reward', 'return', 'episode_mask', 'turn_mask',
             'observation_mask', 'action_mask', 'progress')
    stacked = {n: torch.from_numpy(np.ascontiguousarray(np.array([c[i] for c in cols])))
               for i, n in enumerate(names)}
    obs = _leaf_map(lambda a: torch.from_numpy(np.ascontiguousarray(a)), _stack(template, obss))
    return {
        'observation': obs,
        'policy': stacked['policy'], 'value': stacked['value'],
        'action': stacked['action'], 'outcome': stacked['outcome'],
        'reward': stacked['reward'], 'return': stacked['return'],
        'episode_mask': stacked['episode_mask'],
        'turn_mask': stacked['turn_mask'], 'observation_mask': stacked['observation_mask'],
        'action_mask': stacked['action_mask'],
        'progress': stacked['progress'],
    }
