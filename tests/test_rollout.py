"""Device rollout and replay (handyrl_amd/rollout.py) vs the reference.

* TicTacToe rules: the batched env and the CPU plugin replay 60 random games
  recorded from the reference env (tests/golden/tictactoe_rules.*): legal
  actions, both players' observations, terminal plies and outcomes;
* the replay's window gather equals make_batch (bit-exact to the reference,
  tests/test_make_batch.py) on the same episodes converted to the
  reference's wire format;
* sampling: actions follow softmax over the legal actions; window choice
  follows the Batcher's recency weighting.
"""

import random

import numpy as np
import pytest
import torch

from tests.conftest import load_golden


@pytest.fixture(scope='module')
def rules():
    return load_golden('tictactoe_rules')


def test_cpu_env_matches_reference_rules(rules):
    from handyrl_amd.envs.tictactoe import Environment
    games, arrays = rules
    env = Environment()
    for g, game in enumerate(games):
        env.reset()
        for i, ply in enumerate(game['plies']):
            assert not env.terminal()
            assert env.turn() == ply['turn']
            assert env.legal_actions(env.turn()) == ply['legal']
            for p in (0, 1):
                np.testing.assert_array_equal(env.observation(p), arrays['%d:%d:obs%d' % (g, i, p)])
            env.play(ply['action'])
        assert env.terminal()
        assert [env.outcome()[0], env.outcome()[1]] == game['outcome']


def _replay_games(games, device):
    """Drive all games in parallel through TicTacToeBatch with the recorded actions."""
    from handyrl_amd.rollout import TicTacToeBatch
    E = len(games)
    env = TicTacToeBatch(E, device)
    T = max(len(g['plies']) for g in games)
    return env, T


@pytest.mark.parametrize('device', ['cpu', pytest.param('cuda', marks=pytest.mark.gpu)])
def test_batched_env_matches_reference_rules(rules, device):
    if device == 'cuda' and not torch.cuda.is_available():
        pytest.skip('no GPU')
    games, arrays = rules
    dev = torch.device(device)
    env, T = _replay_games(games, dev)
    for t in range(T):
        live = torch.tensor([t < len(g['plies']) for g in games], device=dev)
        assert torch.equal(~env.terminal(), live)
        acts = torch.zeros(len(games), dtype=torch.long, device=dev)
        for g, game in enumerate(games):
            if t < len(game['plies']):
                ply = game['plies'][t]
                assert int(env.turn()[g]) == ply['turn']
                assert torch.nonzero(env.legal()[g]).view(-1).tolist() == ply['legal']
                acts[g] = ply['action']
        for p in (0, 1):
            o = env.observation(torch.full((len(games),), p, dtype=torch.long, device=dev)).cpu().numpy()
            for g, game in enumerate(games):
                if t < len(game['plies']):
                    np.testing.assert_array_equal(o[g], arrays['%d:%d:obs%d' % (g, t, p)])
        env.step(acts, live)
    assert bool(env.terminal().all())
    assert env.outcome().cpu().tolist() == [[float(x) for x in g['outcome']] for g in games]


def _generate(device, E=64, seed=0):
    from handyrl_amd.envs.tictactoe import SimpleConv2dModel
    from handyrl_amd.rollout import TicTacToeBatch, DeviceGenerator
    torch.manual_seed(seed)
    net = SimpleConv2dModel().to(device)
    gen = DeviceGenerator(TicTacToeBatch(E, device), net)
    g = torch.Generator(device=device).manual_seed(seed)
    return gen.generate(generator=g)


@pytest.mark.parametrize('device', ['cpu', pytest.param('cuda', marks=pytest.mark.gpu)])
@pytest.mark.parametrize('T', [9, 4, 12])
def test_replay_gather_equals_make_batch(device, T):
    if device == 'cuda' and not torch.cuda.is_available():
        pytest.skip('no GPU')
    from handyrl_amd.batch import make_batch
    from handyrl_amd.rollout import DeviceReplay, episodes_to_wire
    dev = torch.device(device)
    ep = _generate(dev, E=48, seed=T)
    rep = DeviceReplay(64, 9, (3, 3, 3), 9, 2, dev)
    rep.add(ep)
    g = torch.Generator(device=dev).manual_seed(1)
    slots, start = rep.sample_windows(40, T, generator=g)
    batch = rep.gather(slots, start, T)
    wire = episodes_to_wire(ep)
    windows = []
    for s, st in zip(slots.tolist(), start.tolist()):
        e = wire[s]
        L = e['steps']
        ed = min(st + T, L)
        # the whole episode is stored from base 0 (compress blocks cover every ply)
        windows.append({'args': {}, 'outcome': e['outcome'], 'moment': e['moment'], 'base': 0,
                        'start': st, 'end': ed, 'total': L})
    ref = make_batch(windows, {'turn_based_training': True, 'observation': False, 'forward_steps': T})
    for k, v in ref.items():
        got = batch[k].cpu()
        assert got.shape == v.shape and got.dtype == v.dtype, (k, got.shape, v.shape)
        np.testing.assert_array_equal(got.numpy(), v.numpy(), err_msg=k)


def test_generated_games_are_legal_and_complete():
    ep = _generate(torch.device('cpu'), E=200, seed=3)
    L = ep['length']
    assert int(L.min()) >= 5 and int(L.max()) <= 9
    act, amask = ep['action'], ep['action_mask']
    t = torch.arange(9).view(1, -1)
    live = t < L.view(-1, 1)
    chosen = amask.gather(-1, act.unsqueeze(-1)).squeeze(-1)
    assert bool((chosen[live] == 0).all())             # every played action was legal
    # each square is played at most once per game
    for e in range(20):
        a = act[e, :int(L[e])].tolist()
        assert len(set(a)) == len(a)
    # turns alternate starting with player 0
    assert torch.equal(ep['turn'][live], (t.expand_as(live) % 2)[live])


def test_gumbel_sampling_matches_softmax_over_legal():
    """generation.py:53 samples random.choices(legal, weights=softmax(p[legal]))."""
    torch.manual_seed(0)
    logits = torch.tensor([0.5, -1.0, 2.0, 0.0, 0.3, -0.2, 1.0, 0.1, -2.0])
    legal = torch.tensor([1, 0, 1, 1, 0, 1, 1, 1, 0], dtype=torch.bool)
    m = torch.where(legal, 0.0, 1e32)
    p = logits - m
    n = 200000
    u = torch.rand(n, 9).clamp_(1e-20, 1.0)
    a = torch.argmax(p - torch.log(-torch.log(u)), dim=-1)
    freq = torch.bincount(a, minlength=9).float() / n
    expect = torch.softmax(logits.masked_fill(~legal, -float('inf')), 0)
    assert float(freq[~legal].sum()) == 0.0
    assert torch.allclose(freq, expect, atol=4e-3)


def test_window_choice_recency_weighting():
    """P(episode i of n) proportional to 1 - (n-1-i)/maximum_episodes (train.py:286-289)."""
    from handyrl_amd.rollout import DeviceReplay
    rep = DeviceReplay(10, 9, (3, 3, 3), 9, 2, torch.device('cpu'), maximum_episodes=20)
    rep.count, rep.ptr = 10, 0
    rep.length.fill_(9)
    g = torch.Generator().manual_seed(0)
    slots, start = rep.sample_windows(200000, 9, generator=g)
    freq = torch.bincount(slots, minlength=10).double() / slots.numel()
    w = 1 - (9 - torch.arange(10, dtype=torch.float64)) / 20
    assert torch.allclose(freq, w / w.sum(), atol=4e-3)
    assert int(start.max()) == 0     # 9-ply episodes, T=9: one window per episode


@pytest.mark.gpu
def test_selfplay_training_learns_tictactoe(cuda):
    """End to end on one GPU: device self-play -> HBM replay -> learner steps.

    The reference's learning signal, checked functionally: a randomly
    initialised TicTacToe net must beat a uniform random player after a few
    seconds of training (win >= 80 %, loss <= 5 %).
    """
    from handyrl_amd.envs.tictactoe import SimpleConv2dModel
    from handyrl_amd.loop import SelfPlayTrainer, evaluate_vs_random
    from handyrl_amd.synthetic import default_args
    torch.manual_seed(0)
    net = SimpleConv2dModel().to(cuda)
    args = default_args(9, 1024)
    args['maximum_episodes'] = 32768
    tr = SelfPlayTrainer(net, args, cuda, games_per_round=4096, capacity=32768)
    before = evaluate_vs_random(net, cuda)
    tr.run(25, 20)
    after = evaluate_vs_random(net, cuda)
    assert after['win'] >= 0.8 and after['loss'] <= 0.05, (before, after)
    assert after['win'] > before['win'] + 0.2


@pytest.mark.gpu
@pytest.mark.parametrize('env_name', ['tictactoe', 'geister'])
def test_graph_generate_equals_eager(cuda, env_name):
    """DeviceGenerator's HIP-graph ply (one capture per mover parity, replayed every ply) plays exactly the
    games of the eager ply loop on the same uniforms: every episode tensor bit-identical, over two calls (the
    second replays the graphs captured by the first)."""
    from handyrl_amd.rollout import TicTacToeBatch, DeviceGenerator
    from handyrl_amd.nn import accelerate
    if env_name == 'tictactoe':
        from handyrl_amd.envs.tictactoe import SimpleConv2dModel as Net
        env_cls, E = TicTacToeBatch, 512
    else:
        from handyrl_amd.envs.geister import GeisterNet as Net, GeisterBatch as env_cls
        E = 64
    torch.manual_seed(1)
    net = accelerate(Net().to(cuda))
    eager = DeviceGenerator(env_cls(E, cuda), net, graph=False)
    graph = DeviceGenerator(env_cls(E, cuda), net, graph=True)
    for call in range(2):
        a = eager.generate(generator=torch.Generator(device=cuda).manual_seed(call))
        b = graph.generate(generator=torch.Generator(device=cuda).manual_seed(call))
        assert graph._st['graphs'] is not None and eager._st['graphs'] is None
        assert set(a) == set(b)
        for k in a:
            if isinstance(a[k], dict):
                for kk in a[k]:
                    assert torch.equal(a[k][kk], b[k][kk]), (call, k, kk)
            else:
                assert torch.equal(a[k], b[k]), (call, k)
        assert int(a['length'].min()) > 0


@pytest.mark.gpu
@pytest.mark.parametrize('A', [9, 214])
def test_sample_record_hip_matches_torch(cuda, A):
    """csrc/hrl_selfplay.hip (one launch) vs the torch formulation of the ply tail on the same device tensors:
    sampled actions and every record slot bit-identical, including rows with no legal action (all logits
    -1e32: torch.argmax's tie order picks the lowest label), finished games (reset values) and untouched
    slots of other plies."""
    from handyrl_amd.rollout import sample_record_torch, sample_record_hip
    E, Tm, P = 300, 5, 2
    g = torch.Generator(device=cuda).manual_seed(A)

    def state():
        return {'policy': torch.full((E, Tm, A), 7.0, device=cuda), 'amask': torch.full((E, Tm, A), 3.0, device=cuda),
                'action': torch.full((E, Tm), 5, dtype=torch.long, device=cuda),
                'value': torch.full((E, Tm), 2.0, device=cuda),
                'turn': torch.full((E, Tm), 4, dtype=torch.long, device=cuda),
                'reward': torch.full((E, Tm, P), 9.0, dtype=torch.float64, device=cuda),
                'U': torch.rand(Tm, E, A, device=cuda, generator=g).clamp_(1e-20, 1.0),
                't': torch.tensor([3], device=cuda)}
    a_st = state()
    b_st = {k: v.clone() for k, v in a_st.items()}
    logits = torch.randn(E, A + 3, device=cuda, generator=g)[:, :A]          # strided rows
    legal = torch.rand(E, A, device=cuda, generator=g) < 0.4
    legal[:7] = False
    value = torch.randn(E, 1, device=cuda, generator=g)
    active = torch.rand(E, device=cuda, generator=g) < 0.8
    player = (torch.rand(E, device=cuda, generator=g) < 0.5).long()
    reward = torch.randn(E, P, device=cuda, generator=g, dtype=torch.float64)
    a = sample_record_torch(a_st, logits, legal, value, active, player, reward)
    b = sample_record_hip(b_st, logits, legal, value, active, player, reward)
    assert torch.equal(a, b)
    assert bool((a[:7] == 0).all())
    for k in ('policy', 'amask', 'action', 'value', 'turn', 'reward'):
        assert torch.equal(a_st[k], b_st[k]), k


@pytest.mark.gpu
def test_state_dependent_reward_is_read_after_the_step(cuda):
    """A batched env whose reward depends on the state (no REWARD_STATELESS) has it read after env.step, as
    generation.py:55-60 reads env.reward() after env.step: with a GeisterBatch whose reward is 0.001 x its ply
    counter, slot t of the reward record holds the reward of the state AFTER ply t for every game running at ply t
    (0 otherwise), and the returns are the fp64 discounted sums of those records (generation.py:73-77)."""
    from handyrl_amd.envs.geister import GeisterNet, GeisterBatch
    from handyrl_amd.rollout import DeviceGenerator
    from handyrl_amd.nn import accelerate

    class PlyReward(GeisterBatch):
        REWARD_STATELESS = False
        seen = None

        def reward(self):
            return (0.001 * (self.turn_count + 2).double()).view(-1, 1).expand(-1, 2).contiguous()

        def step(self, action, active):
            before = self.reward().clone()
            super().step(action, active)
            self.seen.append((before, self.reward().clone(), active.clone()))

    torch.manual_seed(3)
    net = accelerate(GeisterNet().to(cuda))
    E = 32
    env = PlyReward(E, cuda)
    env.seen = []
    gen = DeviceGenerator(env, net, graph=False, gamma=0.8)
    ep = gen.generate(generator=torch.Generator(device=cuda).manual_seed(0))
    reward = ep['reward'].cpu()          # the episode record's dtype (recorded in fp64, like the reference's floats)
    T = reward.shape[1]
    expect = torch.zeros(reward.shape, dtype=torch.float64)
    moved = False
    for t, (before, after, active) in enumerate(env.seen[:T]):
        a = active.cpu().view(-1, 1)
        expect[:, t] = torch.where(a, after.cpu(), 0.0)
        moved = moved or bool((a & (after.cpu() != before.cpu())).any())
    assert moved   # the reward does change with the step, so reading it before would differ
    bad = (reward != expect.to(reward.dtype)).any(-1).nonzero().tolist()
    assert not bad, (len(env.seen), T, ep['length'].tolist(),
                     [(n, t, reward[n, t].tolist(), expect[n, t].tolist()) for n, t in bad[:6]])
    ret = torch.zeros(E, 2, dtype=torch.float64)
    rets = torch.zeros(E, T, 2, dtype=torch.float64)
    for k in range(T - 1, -1, -1):
        ret = expect[:, k] + 0.8 * ret
        rets[:, k] = ret
    assert torch.equal(ep['return'].cpu(), rets.to(ep['return'].dtype))   # fp64 sums, stored as the record's dtype
