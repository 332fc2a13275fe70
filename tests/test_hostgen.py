"""Host-env batched self-play (handyrl_amd.hostgen) against the reference's generation.py.

* tests/golden/generation.* holds episodes of the reference's own
  ``Generator.generate`` (generation.py:20-88) with seeded nets: TicTacToe with
  and without ``observation``, ParallelTicTacToe (simultaneous ``turns()``,
  ``random`` inside ``step``) with and without ``observation``, Geister
  (recurrent GeisterNet, every player's state advanced) with ``observation``.
  ``HostBatchGenerator(sampler='reference')`` plays the same seeded games
  several at a time (fewer slots than games, so slots restart) with one
  batched forward per ply and must reproduce every moment: turn players,
  observations, values, masked policies, action masks, actions, rewards,
  returns, outcomes.  On the CPU here and through the HIP inference path on
  the GPU (policies / values within 1e-5, everything else exact).
* ``MomentReplay.gather`` == ``make_batch`` (train.py:33-133, golden-pinned in
  tests/test_make_batch.py) on the same windows in all four training modes.
* the Gumbel sampler draws from softmax over the legal actions.
"""

import json
import os
import random

import numpy as np
import pytest
import torch

from handyrl_amd.batch import make_batch
from handyrl_amd.environment import make_env
from handyrl_amd.hostgen import HostBatchGenerator, MomentReplay, to_wire

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden')


@pytest.fixture(scope='module')
def gen_golden():
    with open(os.path.join(GOLD, 'generation.json')) as f:
        man = json.load(f)
    arr = np.load(os.path.join(GOLD, 'generation.npz'))
    return man, arr


def _net(case, arr, device):
    env = make_env({'env': case['env']})
    torch.manual_seed(case['net_seed'])
    net = env.net()()
    pre = 'net:%s:%d:' % (case['net_key'], case['net_seed'])
    stored = {k[len(pre):]: torch.from_numpy(arr[k]) for k in arr.files if k.startswith(pre)}
    if stored:
        net.load_state_dict(stored)
    for k, v in net.state_dict().items():   # the seeded init is the reference's (param sums recorded)
        assert abs(float(v.double().sum()) - case['param_sums'][k]) <= 1e-9 * max(1.0, abs(case['param_sums'][k])), k
    net = net.to(device)
    if device.type == 'cuda':
        from handyrl_amd.nn import accelerate
        accelerate(net)
    return net


def _check_episode(ep, case, arr, ci, k, players, tol):
    pre = '%d:%d:' % (ci, k)
    L = int(case['steps'][k])
    assert ep['steps'] == L
    np.testing.assert_array_equal([ep['outcome'][p] for p in players], arr[pre + 'outcome'])
    for t, m in enumerate(ep['moments']):
        for j, p in enumerate(players):
            assert (p in m['turn']) == arr[pre + 'turn'][t, j], (t, p)
            o = m['observation'][p]
            assert (o is not None) == arr[pre + 'omask'][t, j], (t, p)
            if o is not None:
                if case['obs_keys']:
                    for kk in case['obs_keys']:
                        np.testing.assert_array_equal(o[kk], arr[pre + 'obs.' + kk][t, j])
                else:
                    np.testing.assert_array_equal(o, arr[pre + 'obs'][t, j])
                np.testing.assert_allclose(np.asarray(m['value'][p]).reshape(-1)[0], arr[pre + 'value'][t, j],
                                           rtol=tol, atol=tol)
            else:
                assert m['value'][p] is None
            assert (m['policy'][p] is not None) == arr[pre + 'tmask'][t, j]
            if m['policy'][p] is not None:
                np.testing.assert_allclose(m['policy'][p], arr[pre + 'policy'][t, j], rtol=tol, atol=tol)
                np.testing.assert_array_equal(m['action_mask'][p], arr[pre + 'amask'][t, j])
                assert m['action'][p] == arr[pre + 'action'][t, j], (t, p)
            else:
                assert m['action'][p] is None and m['action_mask'][p] is None
            r = arr[pre + 'reward'][t, j]
            assert (m['reward'][p] is None) == bool(np.isnan(r))
            if m['reward'][p] is not None:
                assert m['reward'][p] == r
            assert m['return'][p] == arr[pre + 'return'][t, j], (t, p)


def _replay_case(gen_golden, ci, device, tol):
    man, arr = gen_golden
    case = man[ci]
    net = _net(case, arr, device)
    env_name = case['env']
    games = len(case['seeds'])
    E = max(1, min(3, games - 1)) if games > 1 else 1
    g = HostBatchGenerator(lambda: make_env({'env': env_name}), net,
                           {'observation': case['observation'], 'gamma': 0.8}, E=E, sampler='reference',
                           game_seeds=case['seeds'])
    state = random.getstate()
    eps = g.generate(games)
    assert random.getstate() == state            # the caller's random stream is left as it was
    assert len(eps) == games
    for k, ep in enumerate(eps):
        _check_episode(ep, case, arr, ci, k, case['players'], tol)


CASE_IDS = ['ttt_obs', 'ttt', 'pttt', 'pttt_obs', 'geister_obs']


@pytest.mark.parametrize('ci', range(len(CASE_IDS)), ids=CASE_IDS)
def test_generation_matches_reference_cpu(gen_golden, ci):
    _replay_case(gen_golden, ci, torch.device('cpu'), 1e-5)


@pytest.mark.gpu
@pytest.mark.parametrize('ci', range(len(CASE_IDS)), ids=CASE_IDS)
def test_generation_matches_reference_gpu(gen_golden, ci, cuda):
    """The same seeded games with the forward on the GPU (HIP inference layers, two groups in flight)."""
    _replay_case(gen_golden, ci, cuda, 1e-5)


def _windows_wire(eps, pick, start, T, compress_steps=4):
    """make_batch input for the windows MomentReplay picked (Batcher.select_episode's record, train.py:290-301)."""
    out = []
    for e, st in zip(pick.tolist(), start.tolist()):
        ep = to_wire(eps[e], compress_steps)
        ed = min(st + T, ep['steps'])
        sb, eb = st // compress_steps, (ed - 1) // compress_steps + 1
        out.append({'args': ep['args'], 'outcome': ep['outcome'], 'moment': ep['moment'][sb:eb],
                    'base': sb * compress_steps, 'start': st, 'end': ed, 'total': ep['steps']})
    return out


@pytest.mark.parametrize('env_name', ['TicTacToe', 'ParallelTicTacToe', 'Geister'])
@pytest.mark.parametrize('tbt,obs', [(True, False), (True, True), (False, False), (False, True)])
def test_moment_replay_gather_matches_make_batch(env_name, tbt, obs):
    torch.manual_seed(3)
    net = make_env({'env': env_name}).net()()
    n = 3 if env_name == 'Geister' else 10
    g = HostBatchGenerator(lambda: make_env({'env': env_name}), net, {'observation': obs, 'gamma': 0.8}, E=4,
                           seed=5)
    eps = g.generate(n)
    T = 12 if env_name == 'Geister' else 6
    args = {'turn_based_training': tbt, 'observation': obs, 'forward_steps': T, 'maximum_episodes': 1000}
    replay = MomentReplay(args, 'cpu', capacity=8)      # small: the ring grows while episodes arrive
    replay.add(eps[:n // 2])
    replay.add(eps[n // 2:])
    B = 16
    rng = torch.Generator().manual_seed(7)
    pick, start = replay.sample_windows(B, T, generator=rng)
    players = list(range(len(eps[0]['outcome'])))
    random.seed(11)
    saved = random.getstate()
    solo = None
    if not tbt:   # the players make_batch's random.choice will draw, window by window (train.py:57-58)
        solo = torch.tensor([random.choice(players) for _ in range(B)])
        random.setstate(saved)
    got = replay.gather(pick, start, T, solo)
    want = make_batch(_windows_wire(eps, pick, start, T), args)
    assert set(got) == set(want)
    for k in want:
        if isinstance(want[k], dict):
            for kk in want[k]:
                torch.testing.assert_close(got[k][kk], want[k][kk], rtol=0, atol=0)
        else:
            assert got[k].dtype == want[k].dtype, k
            torch.testing.assert_close(got[k], want[k], rtol=0, atol=0, msg=k)


def test_moment_replay_evicts_to_maximum_episodes():
    torch.manual_seed(0)
    net = make_env({'env': 'TicTacToe'}).net()()
    g = HostBatchGenerator(lambda: make_env({'env': 'TicTacToe'}), net, {'observation': False, 'gamma': 0.8}, E=4)
    args = {'turn_based_training': True, 'observation': False, 'forward_steps': 4, 'maximum_episodes': 7}
    replay = MomentReplay(args, 'cpu', capacity=4)
    all_eps = []
    for _ in range(4):
        eps = g.generate(5)
        all_eps += eps
        replay.add(eps)
        assert len(replay) == min(len(all_eps), 7)
    # the stored episodes are the 7 newest, oldest first
    start, length, oc = replay._device_tables()
    assert length.tolist() == [e['steps'] for e in all_eps[-7:]]
    assert oc[:, 0].tolist() == [float(e['outcome'][0]) for e in all_eps[-7:]]
    b = replay.sample(32, 4)
    assert b['policy'].shape == (32, 4, 1, 9)


def test_gumbel_sampler_is_softmax_over_legal():
    """Every turn player's action is argmax(p - log(-log u)): softmax over the legal actions."""
    class Fixed(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.w = torch.nn.Parameter(torch.tensor([0.5, -1.0, 2.0, 0.0, 1.0, -0.5, 0.3, 1.5, -2.0]))

        def forward(self, x, hidden=None):
            return {'policy': self.w.expand(x.shape[0], 9), 'value': torch.zeros(x.shape[0], 1)}

    class OnePly:
        def __init__(self):
            from handyrl_amd.envs.tictactoe import Environment
            self.env = Environment()

        def __getattr__(self, name):
            return getattr(self.env, name)

        def reset(self, args=None):
            self.env.reset()
            self.env.cells[[1, 4]] = 1      # cells 1 and 4 taken: 7 legal actions

        def terminal(self):
            return len(self.env.record) == 1

    g = HostBatchGenerator(OnePly, Fixed(), {'observation': False, 'gamma': 1.0}, E=64, seed=1)
    eps = g.generate(20000)
    counts = np.bincount([e['moments'][0]['action'][0] for e in eps], minlength=9)
    assert counts[1] == 0 and counts[4] == 0
    w = Fixed().w.detach().numpy().astype(np.float64)
    legal = [0, 2, 3, 5, 6, 7, 8]
    p = np.exp(w[legal] - w[legal].max())
    p /= p.sum()
    freq = counts[legal] / counts.sum()
    assert np.abs(freq - p).max() < 0.015, (freq, p)
