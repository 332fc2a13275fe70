"""The per-player device rollout (handyrl_amd/rollout.py: DeviceGenerator with ``observation=True`` or a
simultaneous-move env, PlayerReplay) against the reference.

* tests/golden/generation.* holds the reference's own ``Generator.generate`` episodes (generation.py:20-88) of
  seeded games: TicTacToe with ``observation`` (every player infers every ply), ParallelTicTacToe (both players
  move every ply, one of them played at random; parallel_tictactoe.py:20-24) with and without ``observation``,
  and Geister (recurrent GeisterNet, every player's state advanced) with ``observation``.  The device generator,
  fed the same random-stream values (``reference_uniforms``: each turn player's ``random.choices`` draw, the
  simultaneous step's ``random.choice``), must reproduce every moment of every game: turn and observation
  masks, observations, values, masked policies, action masks, actions, rewards, returns, outcomes (policies and
  values within 1e-5, everything else exact) -- on the CPU here and through the HIP path on the GPU.
* ``PlayerReplay.gather`` equals ``make_batch`` (train.py:33-133, golden-pinned in tests/test_make_batch.py) on
  the same windows, with every player (turn-based training) and with one random player per window (solo).
"""

import json
import os

import numpy as np
import pytest
import torch

from handyrl_amd.rollout import (DeviceGenerator, ParallelTicTacToeBatch, TicTacToeBatch, PlayerReplay,
                                 player_episodes_to_wire, reference_uniforms)
from tests.test_hostgen import _net

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden')


@pytest.fixture(scope='module')
def gen_golden():
    with open(os.path.join(GOLD, 'generation.json')) as f:
        man = json.load(f)
    return man, np.load(os.path.join(GOLD, 'generation.npz'))


def _batch_env(name, E, device):
    if name == 'TicTacToe':
        return TicTacToeBatch(E, device)
    if name == 'ParallelTicTacToe':
        return ParallelTicTacToeBatch(E, device)
    from handyrl_amd.envs.geister import GeisterBatch
    return GeisterBatch(E, device)


def _replay_reference_games(gen_golden, name, device, graph=False):
    man, arr = gen_golden
    ci = [c['name'] for c in man].index(name)
    case = man[ci]
    net = _net(case, arr, device)
    E = len(case['seeds'])
    env = _batch_env(case['env'], E, device)
    P = len(case['players'])
    gen = DeviceGenerator(env, net, gamma=0.8, observation=case['observation'], graph=graph)
    u, sel = reference_uniforms(case['seeds'], env.MAX_PLIES, P, simultaneous=getattr(env, 'SIMULTANEOUS', False))
    ep = {k: (v.cpu() if isinstance(v, torch.Tensor) else {kk: vv.cpu() for kk, vv in v.items()})
          for k, v in gen.generate(reference=(u, sel)).items()}
    tol = 1e-5
    for k in range(E):
        pre = '%d:%d:' % (ci, k)
        L = int(case['steps'][k])
        assert int(ep['length'][k]) == L, (k, int(ep['length'][k]), L)
        np.testing.assert_array_equal(ep['outcome'][k].numpy(), arr[pre + 'outcome'])
        tmask, omask = ep['tmask'][k, :L].numpy(), ep['omask'][k, :L].numpy()
        np.testing.assert_array_equal(tmask, arr[pre + 'turn'])
        np.testing.assert_array_equal(tmask, arr[pre + 'tmask'])
        np.testing.assert_array_equal(omask, arr[pre + 'omask'])
        if case['obs_keys']:
            for kk in case['obs_keys']:
                np.testing.assert_array_equal(ep['observation'][kk][k, :L].numpy(), arr[pre + 'obs.' + kk])
        else:
            np.testing.assert_array_equal(ep['observation'][k, :L].numpy(), arr[pre + 'obs'])
        np.testing.assert_allclose(ep['value'][k, :L].numpy(), arr[pre + 'value'], rtol=tol, atol=tol)
        pol, ref_pol = ep['policy'][k, :L].numpy(), arr[pre + 'policy']
        np.testing.assert_allclose(pol, ref_pol, rtol=tol, atol=tol)
        np.testing.assert_array_equal(ep['action_mask'][k, :L].numpy()[tmask], arr[pre + 'amask'][tmask])
        np.testing.assert_array_equal(ep['action'][k, :L].numpy()[tmask], arr[pre + 'action'][tmask])
        rew = arr[pre + 'reward']
        has = ~np.isnan(rew)
        np.testing.assert_array_equal(ep['reward'][k, :L].numpy()[has], rew[has].astype(np.float32))   # fp32 out
        np.testing.assert_array_equal(ep['return'][k, :L].double().numpy(),
                                      arr[pre + 'return'].astype(np.float32).astype(np.float64))
    return ep


PLAYER_CASES = ['ttt_obs', 'pttt', 'pttt_obs', 'geister_obs']


@pytest.mark.parametrize('name', PLAYER_CASES)
def test_player_generation_matches_reference_cpu(gen_golden, name):
    _replay_reference_games(gen_golden, name, torch.device('cpu'))


@pytest.mark.gpu
@pytest.mark.parametrize('name', PLAYER_CASES)
@pytest.mark.parametrize('graph', [False, True])
def test_player_generation_matches_reference_gpu(gen_golden, name, graph, cuda):
    """The same games through the HIP inference layers, eager and as one captured ply graph."""
    _replay_reference_games(gen_golden, name, cuda, graph=graph)


@pytest.mark.parametrize('env_name,obs', [('TicTacToe', True), ('ParallelTicTacToe', False),
                                          ('ParallelTicTacToe', True)])
@pytest.mark.parametrize('tbt', [True, False])
@pytest.mark.parametrize('T', [4, 9])
def test_player_replay_gather_matches_make_batch(env_name, obs, tbt, T):
    """PlayerReplay.gather on device-generated per-player episodes == make_batch on the same windows of the same
    episodes in the reference wire format: every player (turn-based training), the first turn player's
    observation / policy / action / action mask beside every player's values (turn-based without observation,
    make_batch's first branch), one random player per window (solo, train.py:55-56, the same random.choice
    draws)."""
    import random
    from handyrl_amd.batch import make_batch
    from handyrl_amd.envs.tictactoe import SimpleConv2dModel
    dev = torch.device('cpu')
    torch.manual_seed(3)
    net = SimpleConv2dModel()
    env = _batch_env(env_name, 24, dev)
    ep = DeviceGenerator(env, net, gamma=0.8, observation=obs, graph=False).generate(
        generator=torch.Generator().manual_seed(T))
    rep = PlayerReplay(32, 9, (3, 3, 3), 9, 2, dev, solo=not tbt, mover=tbt and not obs)
    rep.add(ep)
    slots, start = rep.sample_windows(20, T, generator=torch.Generator().manual_seed(1))
    players = None
    if not tbt:
        random.seed(5)
        players = torch.tensor([random.choice([0, 1]) for _ in range(20)])
        random.seed(5)
    wire = player_episodes_to_wire(ep)
    windows = []
    for s, st in zip(slots.tolist(), start.tolist()):
        e = wire[s]
        windows.append({'args': {}, 'outcome': e['outcome'], 'moment': e['moment'], 'base': 0, 'start': st,
                        'end': min(st + T, e['steps']), 'total': e['steps']})
    ref = make_batch(windows, {'turn_based_training': tbt, 'observation': obs, 'forward_steps': T})
    batch = rep.gather(slots, start, T, players)
    for k, v in ref.items():
        got = batch[k]
        assert got.shape == v.shape and got.dtype == v.dtype, (k, got.shape, v.shape, got.dtype, v.dtype)
        np.testing.assert_array_equal(got.numpy(), v.numpy(), err_msg=k)
