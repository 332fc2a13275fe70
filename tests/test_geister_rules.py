"""Device-batched Geister rules (handyrl_amd.envs.geister.GeisterBatch) vs the reference env.

tests/golden/geister_rules.* holds 24 seeded random games played by the
reference Environment (geister.py:170-541): per ply the turn player, the
legal-action set, both players' observations and the action; per game the
outcome and ply count.  All games are replayed together in one GeisterBatch
(finished games stay frozen while the others go on) and every legal mask,
observation, terminal flag and outcome must be identical.  GeisterBatch is
plain tensor code, so the same test runs on the CPU and on cuda:0.
"""

import numpy as np
import pytest
import torch

from tests.conftest import load_golden
from handyrl_amd.envs.geister import GeisterBatch


@pytest.fixture(scope='module')
def games():
    meta, arrays = load_golden('geister_rules')
    out = []
    for g, m in enumerate(meta):
        pre = '%d:' % g
        L = m['plies']
        out.append({
            'turn': arrays[pre + 'turn'].astype(np.int64),
            'legal': np.unpackbits(arrays[pre + 'legal'], axis=-1)[:, :214].astype(bool),
            'action': arrays[pre + 'action'].astype(np.int64),
            'board': np.unpackbits(arrays[pre + 'board'], axis=-1)[..., :6].astype(np.float32),
            'scalar': arrays[pre + 'scalar'].astype(np.float32),
            'plies': L, 'outcome': m['outcome'], 'win': m['win_color'],
        })
    return out


def replay(games, device):
    E = len(games)
    env = GeisterBatch(E, device)
    Tm = max(g['plies'] for g in games)
    assert Tm <= GeisterBatch.MAX_PLIES
    for t in range(Tm):
        live = np.array([t < g['plies'] for g in games])
        term = env.terminal().cpu().numpy()
        assert (term == ~live).all(), t
        turn = env.turn().cpu().numpy()
        legal = env.legal().cpu().numpy()
        obs = [env.observation(torch.full((E,), q, dtype=torch.long, device=device)) for q in (0, 1)]
        for e in np.nonzero(live)[0]:
            g = games[e]
            assert turn[e] == g['turn'][t], (e, t)
            assert (legal[e] == g['legal'][t]).all(), (e, t, np.nonzero(legal[e] != g['legal'][t]))
            for q in (0, 1):
                np.testing.assert_array_equal(obs[q]['board'][e].cpu().numpy(), g['board'][t, q], err_msg=str((e, t, q)))
                np.testing.assert_array_equal(obs[q]['scalar'][e].cpu().numpy(), g['scalar'][t, q], err_msg=str((e, t, q)))
        acts = torch.tensor([g['action'][t] if t < g['plies'] else 0 for g in games], device=device)
        env.step(acts, torch.tensor(live, device=device))
    assert env.terminal().all()
    np.testing.assert_array_equal(env.plies().cpu().numpy(), [g['plies'] for g in games])
    np.testing.assert_array_equal(env.outcome().cpu().numpy(), np.array([g['outcome'] for g in games], np.float32))
    np.testing.assert_array_equal(env.win.cpu().numpy(), [g['win'] for g in games])
    np.testing.assert_allclose(env.reward().cpu().numpy(), -0.01)


def test_rules_cpu(games):
    assert {g['win'] for g in games} == {0, 1, 2}   # black wins, white wins, 200-move draws
    replay(games, torch.device('cpu'))


@pytest.mark.gpu
def test_rules_gpu(games, cuda):
    replay(games, cuda)


def _generate(device, E, seed=0):
    from handyrl_amd.envs.geister import GeisterNet
    from handyrl_amd.rollout import DeviceGenerator
    torch.manual_seed(seed)
    net = GeisterNet().to(device)
    gen = DeviceGenerator(GeisterBatch(E, device), net, gamma=0.8)
    g = torch.Generator(device=device).manual_seed(seed)
    return net, gen.generate(generator=g)


@pytest.fixture(scope='module')
def generated():
    return _generate(torch.device('cpu'), E=12, seed=4)


def test_generated_geister_games(generated):
    _, ep = generated
    L = ep['length']
    Tm = GeisterBatch.MAX_PLIES
    assert int(L.min()) >= 3 and int(L.max()) <= Tm
    t = torch.arange(Tm).view(1, -1)
    live = t < L.view(-1, 1)
    chosen = ep['action_mask'].gather(-1, ep['action'].unsqueeze(-1)).squeeze(-1)
    assert bool((chosen[live] == 0).all())                       # every played action was legal
    assert bool((ep['action'][:, :2] >= 144).all())              # two layout plies first
    assert torch.equal(ep['turn'][live], (t.expand_as(live) % 2)[live])
    assert bool((ep['reward'][live] == np.float32(-0.01)).all()) and bool((ep['reward'][~live] == 0).all())
    for e in range(L.shape[0]):                                  # generation.py:73-77 in Python floats
        ret = 0.0
        for i in reversed(range(int(L[e]))):
            ret = -0.01 + 0.8 * ret
            assert float(ep['return'][e, i, 0]) == float(np.float32(ret))


def test_recurrent_inference_matches_per_game_loop(generated):
    """generation.py:23-41: one hidden state per player, advanced only on the player's own plies."""
    net, ep = generated
    _check_per_game(net, ep)


@pytest.mark.gpu
def test_gpu_selfplay_matches_per_game_loop(cuda):
    """The GPU self-play path (HIP graph per ply, HIP rules and ply tail, stacked player-major DRC state,
    fused BatchNorm + ReLU inference) against the reference's per-game loop run with the same weights on
    the CPU: every recorded value and legal policy logit of three games."""
    from handyrl_amd.nn import accelerate
    from handyrl_amd.rollout import DeviceGenerator
    from handyrl_amd.envs.geister import GeisterNet
    torch.manual_seed(6)
    cpu = GeisterNet()
    net = accelerate(GeisterNet().to(cuda))
    net.load_state_dict(cpu.state_dict())
    gen = DeviceGenerator(GeisterBatch(16, cuda), net, gamma=0.8)
    gen.generate(generator=torch.Generator(device=cuda).manual_seed(1))     # capture
    ep = gen.generate(generator=torch.Generator(device=cuda).manual_seed(2))
    assert gen._st['graphs'] is not None and gen._st['pmajor']
    ep = {k: ({kk: vv.cpu() for kk, vv in v.items()} if isinstance(v, dict) else v.cpu()) for k, v in ep.items()}
    _check_per_game(cpu, ep, games=(0, 7, 15))


@pytest.mark.gpu
def test_gpu_selfplay_2048_games_matches_per_game_loop(cuda):
    """BASELINE.json configs[2]: 2,048 concurrent games in one generate call (HIP graph per ply); three of
    them, first, middle and last, replayed through the reference's per-game loop on the CPU with the same
    weights: every recorded value, every legal policy logit (tolerance 1e-5 absolute + 1e-5 relative: the
    GPU convolutions run hrl_gboard's exact-split bf16 MFMA kernels, fp32-accurate but summed in another
    order than the CPU's) and the same recurrent-state plumbing."""
    from handyrl_amd.nn import accelerate
    from handyrl_amd.rollout import DeviceGenerator
    from handyrl_amd.envs.geister import GeisterNet
    torch.manual_seed(8)
    cpu = GeisterNet()
    net = accelerate(GeisterNet().to(cuda))
    net.load_state_dict(cpu.state_dict())
    gen = DeviceGenerator(GeisterBatch(2048, cuda), net, gamma=0.8)
    gen.generate(generator=torch.Generator(device=cuda).manual_seed(1))     # capture
    ep = gen.generate(generator=torch.Generator(device=cuda).manual_seed(3))
    assert gen._st['graphs'] is not None
    ep = {k: ({kk: vv.cpu() for kk, vv in v.items()} if isinstance(v, dict) else v.cpu()) for k, v in ep.items()}
    _check_per_game(cpu, ep, games=(0, 1023, 2047), atol=1e-5, rtol=1e-5)


def _check_per_game(net, ep, games=(0, 5), atol=1e-5, rtol=1e-5):
    net.eval()
    with torch.no_grad():
        for e in games:
            hidden = {p: net.init_hidden() for p in (0, 1)}
            for t in range(int(ep['length'][e])):
                p = int(ep['turn'][e, t])
                x = {k: v[e, t].unsqueeze(0) for k, v in ep['observation'].items()}
                h = ([torch.from_numpy(a).unsqueeze(0) for a in hidden[p][0]],
                     [torch.from_numpy(a).unsqueeze(0) for a in hidden[p][1]])
                out = net(x, h)
                hidden[p] = ([a.squeeze(0).numpy() for a in out['hidden'][0]],
                             [a.squeeze(0).numpy() for a in out['hidden'][1]])
                assert abs(float(out['value']) - float(ep['value'][e, t])) < 1e-5, (e, t)
                pol = out['policy'][0] - ep['action_mask'][e, t]
                legal = ep['action_mask'][e, t] == 0
                torch.testing.assert_close(pol[legal], ep['policy'][e, t][legal], rtol=rtol, atol=atol)


@pytest.mark.parametrize('T', [16, 5])
def test_geister_replay_gather_equals_make_batch(generated, T):
    from handyrl_amd.batch import make_batch
    from handyrl_amd.rollout import DeviceReplay, episodes_to_wire
    _, ep = generated
    dev = torch.device('cpu')
    rep = DeviceReplay(16, GeisterBatch.MAX_PLIES, GeisterBatch.OBS_SHAPE, 214, 2, dev, obs_dtype=torch.uint8)
    rep.add(ep)
    g = torch.Generator().manual_seed(T)
    slots, start = rep.sample_windows(10, T, generator=g)
    batch = rep.gather(slots, start, T)
    wire = episodes_to_wire(ep)
    windows = []
    for s, st in zip(slots.tolist(), start.tolist()):
        e = wire[s]
        windows.append({'args': {}, 'outcome': e['outcome'], 'moment': e['moment'], 'base': 0,
                        'start': st, 'end': min(st + T, e['steps']), 'total': e['steps']})
    ref = make_batch(windows, {'turn_based_training': True, 'observation': False, 'forward_steps': T})
    for k, v in ref.items():
        if isinstance(v, dict):
            for kk, vv in v.items():
                np.testing.assert_array_equal(batch[k][kk].numpy(), vv.numpy(), err_msg=k + kk)
                assert batch[k][kk].dtype == vv.dtype
        else:
            got = batch[k]
            assert got.shape == v.shape and got.dtype == v.dtype, (k, got.shape, v.shape)
            np.testing.assert_array_equal(got.numpy(), v.numpy(), err_msg=k)


@pytest.mark.gpu
@pytest.mark.parametrize('full', [False, True])
def test_hip_rules_match_torch_rules_random_games(cuda, full):
    """csrc/hrl_geister.hip (GeisterBatch on a GPU) vs the torch rules (GeisterBatch on the CPU, pinned to the
    reference games above): 512 random games side by side, every ply's legal mask, both players' views (and
    the complete-information view), the state tensors and the outcomes identical.  Exercises escapes,
    captures of both colours, the 200-move draw and frozen finished games far more often than 24 games."""
    E = 512
    gpu, cpu = GeisterBatch(E, cuda), GeisterBatch(E, torch.device('cpu'))
    g = torch.Generator().manual_seed(11 + full)
    for t in range(GeisterBatch.MAX_PLIES):
        for name in ('board', 'color', 'turn_count', 'win', 'cnt'):
            assert torch.equal(getattr(gpu, name).cpu(), getattr(cpu, name)), (t, name)
        assert torch.equal(gpu.active().cpu(), ~cpu.terminal()), t    # the live mask the HIP step keeps
        legal = cpu.legal()
        assert torch.equal(gpu.legal().cpu(), legal), t
        for q in (0, 1):
            pl = torch.full((E,), q, dtype=torch.long)
            a, b = gpu.observation(pl.to(cuda), full=full), cpu.observation(pl, full=full)
            for k in ('board', 'scalar'):
                assert torch.equal(a[k].cpu(), b[k]), (t, q, k)
        active = ~cpu.terminal()
        if not bool(active.any()):
            break
        # a random legal action per game (uniform over the legal labels); finished games pass action 0
        w = legal.float() + 1e-12
        act = torch.multinomial(w, 1, generator=g).view(-1)
        gpu.step(act.to(cuda), active.to(cuda))
        cpu.step(act, active)
    assert bool(cpu.terminal().all())
    wins = set(cpu.win.tolist())
    assert {0, 1, 2} <= wins, wins
    assert torch.equal(gpu.outcome().cpu(), cpu.outcome())


@pytest.mark.gpu
def test_observation_record_kernel(cuda):
    """GeisterBatch.observation_record: the same view as observation(), and slot t of the episode record holds
    it for active games and zeros for finished ones; the other slots are untouched."""
    from handyrl_amd.envs.geister import BOARD_PLANES, SCALARS
    E, Tm = 300, 6
    env = GeisterBatch(E, cuda)
    g = torch.Generator().manual_seed(5)
    for _ in range(9):   # a few random plies: layouts, then moves
        legal = env.legal().cpu()
        env.step(torch.multinomial(legal.float() + 1e-12, 1, generator=g).view(-1).to(cuda),
                 torch.ones(E, dtype=torch.bool, device=cuda))
    rec = {'board': torch.full((E, Tm, BOARD_PLANES, 6, 6), 7.0, device=cuda),
           'scalar': torch.full((E, Tm, SCALARS), 7.0, device=cuda)}
    t = torch.tensor([4], device=cuda)
    active = torch.rand(E, generator=g) < 0.7
    player = env.turn()
    o = env.observation_record(player, rec, t, active.to(cuda))
    ref = env.observation(player)
    for k in ('board', 'scalar'):
        assert torch.equal(o[k], ref[k]), k
        live = active.to(cuda).view(-1, *([1] * (ref[k].dim() - 1)))
        assert torch.equal(rec[k][:, 4], torch.where(live, ref[k], torch.zeros_like(ref[k]))), k
        assert bool((rec[k][:, :4] == 7.0).all()) and bool((rec[k][:, 5:] == 7.0).all()), k
