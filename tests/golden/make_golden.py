"""Golden-vector generator for the learner hot path.

Runs ONLY in the build container, where the reference HandyRL tree is mounted
read-only at ``$HANDYRL_REF`` (default ``/root/reference``).  It imports the
reference's own learner math and writes small ``.npz`` fixtures (inputs and
expected outputs, nothing else) next to this file.  The reference itself never
enters this repository and never travels to the GPU box: the tests only read
the fixtures.

Fixtures written
----------------
``targets.npz`` + ``targets.json``
    ``handyrl.losses.compute_target`` (losses.py:61-74) for MC / TD / UPGO /
    VTRACE on the value-head convention (returns = outcome (B,1,P,1),
    rewards=None, gamma=1; train.py:245) and the return-head convention
    (returns (B,T,P,1), rewards present, gamma=0.8; train.py:246), over
    T in {1,2,9,32}, P in {1,2}, rho P-extent in {1,P}, plus a trailing-dim
    K=2 case.
``loss.npz`` + ``loss.json``
    ``handyrl.train.compute_loss`` (train.py:218-258) on real ``make_batch``
    batches (train.py:33-133) built from seeded self-play episodes
    (generation.py:20-88) of TicTacToe and Geister, with fixed network
    outputs, recording every ``compute_target`` call, the composed advantages,
    the losses, ``dcnt`` and the gradients w.r.t. the network outputs.
``make_batch.npz`` + ``make_batch.json``
    ``handyrl.train.make_batch`` (train.py:33-133) on windows of seeded
    TicTacToe / Geister self-play episodes in the four training modes; the
    episodes are stored decompressed and pickle-free (JSON structure + npz
    arrays, ``encode_episode``), the outputs as arrays.
``geese_net.npz`` + ``geese_net.json``
    GeeseNet (handyrl/envs/kaggle/hungry_geese.py:23-57, config C4) with
    ``kaggle_environments`` stubbed in ``sys.modules`` (the module imports only
    ``make`` from it, :18, and the net never uses it): seeded initial weights,
    the train- and eval-mode forward, ``compute_loss`` in the solo layout
    (turn_based_training=False, P = Pp = 1) with every parameter's gradient,
    and three ``Trainer.train`` learner steps with the final state_dict.  The
    batch is ``handyrl_amd.synthetic.geese_batch`` (no Hungry Geese rules here),
    stored as input arrays.
``trainer.npz`` + ``trainer.json``
    ``Trainer.train`` (train.py:312-401) for two epochs of 2 and 3 batches
    over fixed TicTacToe ``make_batch`` batches (the batcher replaced by a
    list that raises ``update_flag`` at the epoch's last batch): the lr and
    ``data_cnt_ema`` after each epoch (the epoch-end schedule, :396-398) and
    the final weights.
``generation.npz`` + ``generation.json``
    ``handyrl.generation.Generator.generate`` (generation.py:20-88) on seeded
    games with a seeded env network (batch-1 ``ModelWrapper.inference``,
    model.py:43-53): TicTacToe with and without ``observation``,
    ParallelTicTacToe (simultaneous ``turns()``; its step draws from
    ``random``) with and without ``observation``, Geister (recurrent
    GeisterNet) with ``observation``.  Game k of a case runs after
    ``random.seed(seed + k)``.  Every moment is stored as arrays: turn players,
    observations / values (observation flags), masked policies, action masks,
    actions, rewards (None flags), returns, and the outcome.
``learner.npz`` + ``learner.json``
    Three learner steps of the TicTacToe ``SimpleConv2dModel`` exactly as
    ``Trainer.train`` runs them (train.py:375-385): loss, backward,
    ``clip_grad_norm_(4.0)``, ``Adam(lr=3e-8*B*T, weight_decay=1e-5)``.

Usage:  python tests/golden/make_golden.py
"""

import bz2
import json
import pickle
import os
import random
import sys

import numpy as np
import torch
import torch.nn as nn

REF = os.environ.get('HANDYRL_REF', '/root/reference')
OUT = os.path.dirname(os.path.abspath(__file__))

sys.dont_write_bytecode = True
sys.path.insert(0, REF)

from handyrl import losses as ref_losses            # noqa: E402
from handyrl import train as ref_train              # noqa: E402
from handyrl.model import ModelWrapper, RandomModel  # noqa: E402
from handyrl.generation import Generator            # noqa: E402
from handyrl.environment import make_env            # noqa: E402

torch.set_num_threads(1)


def _np(x):
    return None if x is None else x.detach().cpu().numpy().copy()


# ---------------------------------------------------------------------------
# 1. compute_target cases
# ---------------------------------------------------------------------------

def target_cases():
    g = torch.Generator().manual_seed(1234)
    arrays, manifest = {}, []
    shapes = []
    for T in (1, 2, 9, 32):
        for P, Pr in ((1, 1), (2, 1), (2, 2)):
            shapes.append((5, T, P, Pr, 1))
    shapes.append((3, 9, 2, 1, 2))   # trailing value dim K=2, rho broadcast over P and K
    shapes.append((4, 16, 4, 4, 1))  # four-player, per-player rho
    cid = 0
    for (B, T, P, Pr, K) in shapes:
        for head in ('value', 'return'):
            values = torch.tanh(torch.randn(B, T, P, K, generator=g))
            rhos = torch.clamp(torch.exp(0.5 * torch.randn(B, T, Pr, 1, generator=g)), 0, 1)
            cs = torch.clamp(torch.exp(0.5 * torch.randn(B, T, Pr, 1, generator=g)), 0, 1)
            if head == 'value':
                returns = torch.randint(-1, 2, (B, 1, P, K), generator=g).float()
                rewards, gamma = None, 1
            else:
                returns = torch.randn(B, T, P, K, generator=g)
                rewards = 0.1 * torch.randn(B, T, P, K, generator=g)
                gamma = 0.8
            lmb = 0.7
            for alg in ('MC', 'TD', 'UPGO', 'VTRACE'):
                tgt, adv = ref_losses.compute_target(alg, values, returns, rewards, lmb, gamma, rhos, cs)
                pre = '%d:' % cid
                arrays[pre + 'values'] = _np(values)
                arrays[pre + 'returns'] = _np(returns)
                if rewards is not None:
                    arrays[pre + 'rewards'] = _np(rewards)
                arrays[pre + 'rhos'] = _np(rhos)
                arrays[pre + 'cs'] = _np(cs)
                arrays[pre + 'target'] = _np(tgt)
                arrays[pre + 'adv'] = _np(adv)
                manifest.append({'id': cid, 'alg': alg, 'head': head, 'B': B, 'T': T, 'P': P,
                                 'Pr': Pr, 'K': K, 'gamma': gamma, 'lmb': lmb,
                                 'has_rewards': rewards is not None})
                cid += 1
    # values is None convention (losses.py:62-63)
    none_out = ref_losses.compute_target('VTRACE', None, None, None, 0.7, 1, None, None)
    assert none_out == (None, 0)
    return arrays, manifest


# ---------------------------------------------------------------------------
# 2. compute_loss cases on real make_batch batches
# ---------------------------------------------------------------------------

def gen_episodes(env_name, n, obs_flag, seed, net_cls=None):
    random.seed(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)
    env = make_env({'env': env_name})
    if net_cls is not None:
        model = ModelWrapper(net_cls())
    else:
        model = ModelWrapper(RandomModel(env))
    gargs = {'observation': obs_flag, 'gamma': 0.8, 'compress_steps': 4}
    gen = Generator(env, gargs)
    eps = []
    while len(eps) < n:
        ep = gen.generate({p: model for p in env.players()}, {'player': env.players()})
        if ep is not None:
            eps.append(ep)
    return eps


def select_windows(episodes, B, T, compress_steps, seed):
    """Window choice as Batcher.select_episode (train.py:284-302), uniform over episodes."""
    rnd = random.Random(seed)
    out = []
    for _ in range(B):
        ep = episodes[rnd.randrange(len(episodes))]
        turn_candidates = 1 + max(0, ep['steps'] - T)
        st = rnd.randrange(turn_candidates)
        ed = min(st + T, ep['steps'])
        st_block = st // compress_steps
        ed_block = (ed - 1) // compress_steps + 1
        out.append({'args': ep['args'], 'outcome': ep['outcome'], 'moment': ep['moment'][st_block:ed_block],
                    'base': st_block * compress_steps, 'start': st, 'end': ed, 'total': ep['steps']})
    return out


class FixedOutputs(nn.Module):
    """A 'network' whose outputs are its parameters, so d(loss)/d(output) is a param grad."""

    def __init__(self, N, A, has_return, seed):
        super().__init__()
        g = torch.Generator().manual_seed(seed)
        self.p = nn.Parameter(torch.randn(N, A, generator=g))
        self.v = nn.Parameter(torch.tanh(torch.randn(N, 1, generator=g)))
        self.r = nn.Parameter(torch.randn(N, 1, generator=g)) if has_return else None

    def forward(self, x, hidden=None):
        out = {'policy': self.p, 'value': self.v}
        if self.r is not None:
            out['return'] = self.r
        return out


def loss_cases():
    arrays, manifest = {}, []
    specs = [
        # name, env, tbt, obs, B, T, policy_target, value_target, has_return
        ('ttt_tbt', 'TicTacToe', True, False, 6, 16, 'UPGO', 'VTRACE', False),
        ('ttt_tbt_T9', 'TicTacToe', True, False, 8, 9, 'VTRACE', 'VTRACE', False),
        ('ttt_tbt_td', 'TicTacToe', True, False, 6, 5, 'TD', 'MC', False),
        ('ttt_obs', 'TicTacToe', True, True, 5, 4, 'UPGO', 'VTRACE', False),
        ('ttt_solo', 'TicTacToe', False, False, 6, 9, 'MC', 'TD', False),
        ('geister_ret', 'Geister', True, False, 4, 16, 'UPGO', 'VTRACE', True),
        ('geister_ret_td', 'Geister', True, False, 3, 8, 'TD', 'UPGO', True),
    ]
    from handyrl.envs.tictactoe import SimpleConv2dModel
    ep_cache = {}
    for ci, (name, env_name, tbt, obs, B, T, ptgt, vtgt, has_ret) in enumerate(specs):
        key = (env_name, obs)
        if key not in ep_cache:
            if env_name == 'TicTacToe':
                ep_cache[key] = gen_episodes(env_name, 24, obs, seed=7 + ci, net_cls=SimpleConv2dModel)
            else:
                ep_cache[key] = gen_episodes(env_name, 3, obs, seed=7 + ci)
        eps = select_windows(ep_cache[key], B, T, 4, seed=100 + ci)
        args = {'turn_based_training': tbt, 'observation': obs, 'forward_steps': T, 'compress_steps': 4,
                'lambda': 0.7, 'gamma': 0.8, 'policy_target': ptgt, 'value_target': vtgt,
                'entropy_regularization': 0.1, 'entropy_regularization_decay': 0.1}
        random.seed(500 + ci)  # make_batch draws a random player in solo mode (train.py:58)
        batch = ref_train.make_batch(eps, args)
        Pp = batch['action'].size(2)
        A = batch['policy'].size(-1)
        N = B * T * Pp
        net = FixedOutputs(N, A, has_ret, seed=900 + ci)

        calls = []
        orig_ct = ref_train.compute_target

        def spy_ct(alg, *a):
            out = orig_ct(alg, *a)
            calls.append((alg, a, out))
            return out

        captured = {}
        orig_cl = ref_train.compose_losses

        def spy_cl(outputs, log_sel, total_adv, targets, batch_, args_):
            captured['log_sel'] = log_sel.detach().clone()
            captured['total_adv'] = total_adv.detach().clone()
            return orig_cl(outputs, log_sel, total_adv, targets, batch_, args_)

        ref_train.compute_target = spy_ct
        ref_train.compose_losses = spy_cl
        try:
            losses, dcnt = ref_train.compute_loss(batch, net, None, args)
        finally:
            ref_train.compute_target = orig_ct
            ref_train.compose_losses = orig_cl
        losses['total'].backward()

        pre = '%d:' % ci
        for k, v in batch.items():
            if k == 'observation':
                continue
            arrays[pre + 'batch.' + k] = _np(v)
        arrays[pre + 'out.policy'] = _np(net.p)
        arrays[pre + 'out.value'] = _np(net.v)
        arrays[pre + 'grad.policy'] = _np(net.p.grad)
        arrays[pre + 'grad.value'] = _np(net.v.grad)
        if has_ret:
            arrays[pre + 'out.return'] = _np(net.r)
            arrays[pre + 'grad.return'] = _np(net.r.grad)
        arrays[pre + 'log_sel'] = _np(captured['log_sel'])
        arrays[pre + 'total_adv'] = _np(captured['total_adv'])
        call_meta = []
        for j, (alg, a, out) in enumerate(calls):
            values, returns, rewards, lmb, gamma, rhos, cs = a
            cpre = pre + 'call%d.' % j
            if values is not None:
                arrays[cpre + 'values'] = _np(values)
                arrays[cpre + 'target'] = _np(out[0])
                arrays[cpre + 'adv'] = _np(out[1])
            arrays[cpre + 'rhos'] = _np(rhos)
            call_meta.append({'alg': alg, 'values_none': values is None, 'gamma': gamma, 'lmb': lmb,
                              'has_rewards': rewards is not None})
        manifest.append({'id': ci, 'name': name, 'env': env_name, 'B': B, 'T': T, 'Pp': Pp, 'A': A,
                         'has_return': has_ret, 'args': args, 'dcnt': dcnt,
                         'losses': {k: float(v.item()) for k, v in losses.items()}, 'calls': call_meta})
    return arrays, manifest


# ---------------------------------------------------------------------------
# 3. learner steps with the TicTacToe net
# ---------------------------------------------------------------------------

def learner_case():
    from handyrl.envs.tictactoe import SimpleConv2dModel
    B, T = 16, 9
    eps = gen_episodes('TicTacToe', 32, False, seed=31, net_cls=SimpleConv2dModel)
    args = {'turn_based_training': True, 'observation': False, 'forward_steps': T, 'compress_steps': 4,
            'lambda': 0.7, 'gamma': 0.8, 'policy_target': 'UPGO', 'value_target': 'VTRACE',
            'entropy_regularization': 0.1, 'entropy_regularization_decay': 0.1}
    batch = ref_train.make_batch(select_windows(eps, B, T, 4, seed=77), args)

    torch.manual_seed(2024)
    net = SimpleConv2dModel()
    arrays = {}
    names = []
    for k, v in net.state_dict().items():
        arrays['init.' + k] = _np(v)
        names.append(k)
    for k, v in batch.items():
        arrays['batch.' + k] = _np(v)

    model = ModelWrapper(net)
    params = list(model.parameters())
    opt = torch.optim.Adam(params, lr=3e-8 * B * T, weight_decay=1e-5)
    model.train()
    step_losses = []
    for s in range(3):
        losses, dcnt = ref_train.compute_loss(batch, model, None, args)
        opt.zero_grad()
        losses['total'].backward()
        gn = nn.utils.clip_grad_norm_(params, 4.0)
        opt.step()
        step_losses.append({k: float(v.item()) for k, v in losses.items()})
        step_losses[-1]['grad_norm'] = float(gn)
        step_losses[-1]['dcnt'] = dcnt
    for k, v in net.state_dict().items():
        arrays['final.' + k] = _np(v)
    meta = {'B': B, 'T': T, 'args': args, 'lr': 3e-8 * B * T, 'steps': step_losses, 'state_names': names}
    return arrays, meta


# ---------------------------------------------------------------------------
# 4. make_batch on real episode windows
# ---------------------------------------------------------------------------

def encode(obj, arrays, prefix):
    """Pickle-free encoding: JSON structure, ndarrays into `arrays` (tests/golden/episodes.py decodes)."""
    if isinstance(obj, np.ndarray):
        key = '%s#%d' % (prefix, len(arrays))
        arrays[key] = obj
        return {'__nd__': key}
    if isinstance(obj, dict):
        return {'__dict__': [[k, encode(v, arrays, prefix)] for k, v in obj.items()]}
    if isinstance(obj, (list, tuple)):
        return [encode(v, arrays, prefix) for v in obj]
    if isinstance(obj, (np.floating, np.integer)):
        return obj.item()
    return obj


def make_batch_cases():
    import bz2
    import pickle
    from handyrl.envs.tictactoe import SimpleConv2dModel
    arrays, manifest = {}, []
    specs = [
        ('ttt_tbt', 'TicTacToe', True, False, 6, 16),
        ('ttt_tbt_short', 'TicTacToe', True, False, 5, 4),
        ('ttt_obs', 'TicTacToe', True, True, 5, 7),
        ('ttt_solo', 'TicTacToe', False, False, 6, 9),
        ('geister_tbt', 'Geister', True, False, 3, 12),
    ]
    for ci, (name, env_name, tbt, obs, B, T) in enumerate(specs):
        net = SimpleConv2dModel if env_name == 'TicTacToe' else None
        eps = gen_episodes(env_name, 6 if env_name == 'TicTacToe' else 2, obs, seed=60 + ci, net_cls=net)
        windows = select_windows(eps, B, T, 4, seed=200 + ci)
        args = {'turn_based_training': tbt, 'observation': obs, 'forward_steps': T, 'compress_steps': 4}
        random.seed(300 + ci)
        batch = ref_train.make_batch(windows, args)
        enc_windows = []
        for w in windows:
            moments = sum([pickle.loads(bz2.decompress(ms)) for ms in w['moment']], [])
            ew = {k: v for k, v in w.items() if k not in ('moment', 'args')}
            ew['moments'] = encode(moments, arrays, '%d:in' % ci)
            ew['outcome'] = encode(w['outcome'], arrays, '%d:in' % ci)
            enc_windows.append(ew)
        out_keys = []
        for k, v in batch.items():
            if isinstance(v, dict):
                for kk, vv in v.items():
                    arrays['%d:out.%s.%s' % (ci, k, kk)] = _np(vv)
                    out_keys.append('%s.%s' % (k, kk))
            else:
                arrays['%d:out.%s' % (ci, k)] = _np(v)
                out_keys.append(k)
        manifest.append({'id': ci, 'name': name, 'env': env_name, 'args': args, 'seed': 300 + ci,
                         'windows': enc_windows, 'out_keys': out_keys})
    return arrays, manifest


# ---------------------------------------------------------------------------
# 5. TicTacToe rules (handyrl/envs/tictactoe.py:72-172) on random games
# ---------------------------------------------------------------------------

def tictactoe_rules():
    env = make_env({'env': 'TicTacToe'})
    rnd = random.Random(2025)
    games = []
    arrays = {}
    for g in range(60):
        env.reset()
        plies = []
        while not env.terminal():
            legal = env.legal_actions(env.turn())
            a = rnd.choice(legal)
            key = '%d:%d' % (g, len(plies))
            arrays[key + ':obs0'] = env.observation(0)
            arrays[key + ':obs1'] = env.observation(1)
            plies.append({'turn': env.turn(), 'legal': legal, 'action': a})
            env.play(a)
        games.append({'plies': plies, 'outcome': [env.outcome()[0], env.outcome()[1]]})
    return arrays, games


def geister_rules(n_games=24, seed=2026):
    """Random Geister games (geister.py:170-541): per ply the turn player, legal-action
    mask, both players' observations (player given: opponent colours hidden), action;
    per game the outcome, the ply count and the reward."""
    env = make_env({'env': 'Geister'})
    rnd = random.Random(seed)
    arrays, games = {}, []
    for g in range(n_games):
        env.reset()
        turn, legal, acts, boards, scalars = [], [], [], [], []
        while not env.terminal():
            p = env.turn()
            la = env.legal_actions(p)
            m = np.zeros(env.action_length(), np.uint8)
            m[la] = 1
            o = [env.observation(q) for q in (0, 1)]
            a = rnd.choice(la)
            turn.append(p)
            legal.append(m)
            acts.append(a)
            boards.append(np.stack([o[0]['board'], o[1]['board']]).astype(np.uint8))
            scalars.append(np.stack([o[0]['scalar'], o[1]['scalar']]).astype(np.uint8))
            env.play(a)
        pre = '%d:' % g
        arrays[pre + 'turn'] = np.array(turn, np.int8)
        arrays[pre + 'legal'] = np.packbits(np.stack(legal), axis=-1)
        arrays[pre + 'action'] = np.array(acts, np.int16)
        arrays[pre + 'board'] = np.packbits(np.stack(boards), axis=-1)   # (L, 2, 7, 6, 1) bits of the last axis
        arrays[pre + 'scalar'] = np.stack(scalars)
        oc = env.outcome()
        games.append({'plies': len(acts), 'outcome': [oc[0], oc[1]], 'win_color': env.win_color,
                      'reward': env.reward()[0]})
    return arrays, games


# ---------------------------------------------------------------------------
# 6. GeisterNet (recurrent DRC ConvLSTM, geister.py:17-167): init, forward, RNN compute_loss
# ---------------------------------------------------------------------------

def geister_net_case():
    from handyrl.envs.geister import GeisterNet
    arrays = {}
    torch.manual_seed(11)
    net = GeisterNet()
    meta = {'state': {}}
    for k, v in net.state_dict().items():
        vv = v.double()
        meta['state'][k] = [list(v.shape), float(vv.sum()), float((vv * vv).sum())]
    # forward on a fixed observation batch with a non-zero hidden state (train mode)
    g = torch.Generator().manual_seed(12)
    N = 6
    obs = {'board': (torch.rand(N, 7, 6, 6, generator=g) < 0.4).float(),
           'scalar': (torch.rand(N, 18, generator=g) < 0.5).float()}
    hs = [torch.randn(N, 32, 6, 6, generator=g) * 0.1 for _ in range(3)]
    cs = [torch.randn(N, 32, 6, 6, generator=g) * 0.1 for _ in range(3)]
    arrays['fwd.board'] = _np(obs['board'])
    arrays['fwd.scalar'] = _np(obs['scalar'])
    for i in range(3):  # saved before the call: the reference DRC rebinds the list entries in place
        arrays['fwd.h%d' % i] = _np(hs[i])
        arrays['fwd.c%d' % i] = _np(cs[i])
    out = net(obs, (hs, cs))
    for i in range(3):
        arrays['fwd.out_h%d' % i] = _np(out['hidden'][0][i])
        arrays['fwd.out_c%d' % i] = _np(out['hidden'][1][i])
    for k in ('policy', 'value', 'return'):
        arrays['fwd.out_' + k] = _np(out[k])
    # compute_loss through the RNN branch on real Geister windows (train.py:155-174)
    eps = gen_episodes('Geister', 2, False, seed=13)
    B, T = 3, 6
    args = {'turn_based_training': True, 'observation': False, 'forward_steps': T, 'compress_steps': 4,
            'lambda': 0.7, 'gamma': 0.8, 'policy_target': 'UPGO', 'value_target': 'VTRACE',
            'entropy_regularization': 0.1, 'entropy_regularization_decay': 0.1}
    batch = ref_train.make_batch(select_windows(eps, B, T, 4, seed=14), args)
    model = ModelWrapper(net)
    hidden = model.init_hidden([B, batch['value'].size(2)])
    losses, dcnt = ref_train.compute_loss(batch, model, hidden, args)
    losses['total'].backward()
    for k, v in batch.items():
        if isinstance(v, dict):
            for kk, vv in v.items():
                arrays['batch.%s.%s' % (k, kk)] = _np(vv)
        else:
            arrays['batch.' + k] = _np(v)
    meta['loss'] = {'args': args, 'dcnt': dcnt, 'losses': {k: float(v.item()) for k, v in losses.items()},
                    'grad_sq': {n: float((p.grad.double() ** 2).sum()) for n, p in net.named_parameters()
                                if p.grad is not None}}
    return arrays, meta


# ---------------------------------------------------------------------------
# 7. GeeseNet (torus convs, hungry_geese.py:23-57) with kaggle_environments stubbed
# ---------------------------------------------------------------------------

def geese_net_case():
    import types
    if 'kaggle_environments' not in sys.modules:
        stub = types.ModuleType('kaggle_environments')

        def make(*_a, **_k):
            raise RuntimeError('kaggle_environments stub: the rules are not available')
        stub.make = make
        sys.modules['kaggle_environments'] = stub
    from handyrl.envs.kaggle.hungry_geese import GeeseNet
    sys.path.insert(0, os.path.dirname(os.path.dirname(OUT)))   # the repo: its synthetic batch generator
    from handyrl_amd.synthetic import geese_batch, geese_args

    arrays, meta = {}, {'state': {}}
    torch.manual_seed(21)
    net = GeeseNet()
    for k, v in net.state_dict().items():
        vv = v.double()
        meta['state'][k] = [list(v.shape), float(vv.sum()), float((vv * vv).sum())]

    # forward: train mode (batch statistics; updates the running statistics), then eval mode
    fwd = geese_batch(2, 5, torch.device('cpu'), seed=22)['observation'].reshape(10, 17, 7, 11)
    arrays['fwd.x'] = _np(fwd)
    net.train()
    out = net(fwd)
    arrays['fwd.train_policy'], arrays['fwd.train_value'] = _np(out['policy']), _np(out['value'])
    net.eval()
    with torch.no_grad():
        out = net(fwd)
    arrays['fwd.eval_policy'], arrays['fwd.eval_value'] = _np(out['policy']), _np(out['value'])
    for k, v in net.state_dict().items():
        if 'running' in k:
            arrays['fwd.after.' + k] = _np(v)

    # compute_loss (solo layout) and three learner steps from a fresh seeded net
    B, T = 8, 6
    args = geese_args(T, B)
    batch = geese_batch(B, T, torch.device('cpu'), seed=23)
    for k, v in batch.items():
        arrays['batch.' + k] = _np(v)
    torch.manual_seed(21)
    net = GeeseNet()
    model = ModelWrapper(net)
    model.train()
    losses, dcnt = ref_train.compute_loss(batch, model, None, args)
    losses['total'].backward()
    meta['loss'] = {'args': args, 'dcnt': dcnt, 'losses': {k: float(v.item()) for k, v in losses.items()}}
    for n, p in net.named_parameters():
        arrays['grad.' + n] = _np(p.grad)

    torch.manual_seed(21)
    net = GeeseNet()
    model = ModelWrapper(net)
    params = list(model.parameters())
    lr = 3e-8 * B * T
    opt = torch.optim.Adam(params, lr=lr, weight_decay=1e-5)
    model.train()
    steps = []
    for s in range(3):
        losses, dcnt = ref_train.compute_loss(batch, model, None, args)
        opt.zero_grad()
        losses['total'].backward()
        gn = nn.utils.clip_grad_norm_(params, 4.0)
        opt.step()
        steps.append({k: float(v.item()) for k, v in losses.items()})
        steps[-1]['grad_norm'] = float(gn)
        steps[-1]['dcnt'] = dcnt
    for k, v in net.state_dict().items():
        arrays['final.' + k] = _np(v)
    meta['learner'] = {'B': B, 'T': T, 'lr': lr, 'steps': steps}
    return arrays, meta


# ---------------------------------------------------------------------------
# 8. Trainer.train epochs: lr schedule and data-count EMA (train.py:312-401)
# ---------------------------------------------------------------------------

def trainer_case():
    from handyrl.envs.tictactoe import SimpleConv2dModel
    B, T = 16, 9
    eps = gen_episodes('TicTacToe', 32, False, seed=41, net_cls=SimpleConv2dModel)
    args = {'turn_based_training': True, 'observation': False, 'forward_steps': T, 'compress_steps': 4,
            'lambda': 0.7, 'gamma': 0.8, 'policy_target': 'UPGO', 'value_target': 'VTRACE',
            'entropy_regularization': 0.1, 'entropy_regularization_decay': 0.1, 'batch_size': B,
            'maximum_episodes': 1000, 'num_batchers': 1}
    batches = [ref_train.make_batch(select_windows(eps, B, T, 4, seed=60 + i), args) for i in range(5)]
    arrays = {}
    for i, b in enumerate(batches):
        for k, v in b.items():
            arrays['batch%d.%s' % (i, k)] = _np(v)
    torch.manual_seed(2025)
    net = SimpleConv2dModel()
    real_batcher = ref_train.Batcher
    ref_train.Batcher = lambda *a, **k: None       # no batcher processes: batches come from the list
    try:
        trainer = ref_train.Trainer(args, net)
    finally:
        ref_train.Batcher = real_batcher

    class ListBatcher:
        def __init__(self, items):
            self.items = list(items)

        def batch(self):
            b = self.items.pop(0)
            if not self.items:
                trainer.update_flag = True     # the epoch ends after this batch (train.py:372)
            return b
    epochs = []
    for lo, hi in ((0, 2), (2, 5)):
        trainer.update_flag = False
        trainer.batcher = ListBatcher(batches[lo:hi])
        trainer.train()
        epochs.append({'batches': [lo, hi], 'lr': trainer.optimizer.param_groups[0]['lr'],
                       'data_cnt_ema': trainer.data_cnt_ema, 'steps': trainer.steps})
    for k, v in trainer.model.state_dict().items():
        arrays['final.' + k] = _np(v)
    return arrays, {'args': args, 'epochs': epochs, 'seed': 2025}


# ---------------------------------------------------------------------------
# generation.py episodes (host-env batched generator parity)
# ---------------------------------------------------------------------------

GEN_CASES = (   # (name, env, observation, games, game seed, net seed)
    ('ttt_obs', 'TicTacToe', True, 6, 4000, 11),
    ('ttt', 'TicTacToe', False, 4, 4100, 11),
    ('pttt', 'ParallelTicTacToe', False, 6, 4200, 11),
    ('pttt_obs', 'ParallelTicTacToe', True, 6, 4300, 11),
    ('geister_obs', 'Geister', True, 1, 4400, 12),
)


def generation_cases():
    arrays, manifest = {}, []
    nets = {}
    for ci, (name, env_name, obs_flag, games, seed, net_seed) in enumerate(GEN_CASES):
        env = make_env({'env': env_name})
        torch.manual_seed(net_seed)
        net = env.net()()
        key = (env_name if env_name != 'ParallelTicTacToe' else 'TicTacToe', net_seed)
        if key not in nets:
            nets[key] = net
            if key[0] == 'TicTacToe':      # 29k parameters: stored; GeisterNet is rebuilt from its seed
                for k, v in net.state_dict().items():
                    arrays['net:%s:%d:%s' % (key[0], net_seed, k)] = _np(v)
        sums = {k: float(v.double().sum()) for k, v in net.state_dict().items()}
        model = ModelWrapper(net)
        gen = Generator(env, {'observation': obs_flag, 'gamma': 0.8, 'compress_steps': 4})
        players = env.players()
        P = len(players)
        case = {'id': ci, 'name': name, 'env': env_name, 'observation': obs_flag, 'net_seed': net_seed,
                'net_key': key[0], 'seeds': [], 'steps': [], 'obs_keys': None, 'players': players,
                'param_sums': sums}
        for k in range(games):
            random.seed(seed + k)
            ep = gen.generate({p: model for p in players}, {'player': players})
            assert ep is not None
            moments = sum([pickle.loads(bz2.decompress(b)) for b in ep['moment']], [])
            L = len(moments)
            m0 = moments[0]
            o0 = m0['observation'][m0['turn'][0]]
            A = len(m0['policy'][m0['turn'][0]])
            pre = '%d:%d:' % (ci, k)
            turn = np.zeros((L, P), dtype=bool)
            omask = np.zeros((L, P), dtype=bool)
            tmask = np.zeros((L, P), dtype=bool)
            pol = np.zeros((L, P, A), dtype=np.float32)
            amask = np.zeros((L, P, A), dtype=np.float32)
            act = np.full((L, P), -1, dtype=np.int64)
            val = np.zeros((L, P), dtype=np.float32)
            rew = np.full((L, P), np.nan, dtype=np.float64)
            ret = np.zeros((L, P), dtype=np.float64)
            if isinstance(o0, dict):
                case['obs_keys'] = list(o0.keys())
                obs = {kk: np.zeros((L, P) + np.shape(vv), dtype=np.float32) for kk, vv in o0.items()}
            else:
                obs = np.zeros((L, P) + np.shape(o0), dtype=np.float32)
            for t, m in enumerate(moments):
                for j, p in enumerate(players):
                    turn[t, j] = p in m['turn']
                    if m['observation'][p] is not None:
                        omask[t, j] = True
                        if isinstance(obs, dict):
                            for kk in obs:
                                obs[kk][t, j] = m['observation'][p][kk]
                        else:
                            obs[t, j] = m['observation'][p]
                    if m['value'][p] is not None:
                        val[t, j] = np.asarray(m['value'][p]).reshape(-1)[0]
                    if m['policy'][p] is not None:
                        tmask[t, j] = True
                        pol[t, j] = m['policy'][p]
                        amask[t, j] = m['action_mask'][p]
                        act[t, j] = m['action'][p]
                    if m['reward'][p] is not None:
                        rew[t, j] = m['reward'][p]
                    ret[t, j] = m['return'][p]
            for nm, a in (('turn', turn), ('omask', omask), ('tmask', tmask), ('policy', pol),
                          ('amask', amask), ('action', act), ('value', val), ('reward', rew), ('return', ret)):
                arrays[pre + nm] = a
            if isinstance(obs, dict):
                for kk, a in obs.items():
                    arrays[pre + 'obs.' + kk] = a
            else:
                arrays[pre + 'obs'] = obs
            arrays[pre + 'outcome'] = np.array([ep['outcome'][p] for p in players], dtype=np.float64)
            case['seeds'].append(seed + k)
            case['steps'].append(L)
        manifest.append(case)
    return arrays, manifest


def main():
    only = sys.argv[1:]
    if only == ['generation'] or not only:
        arr, man = generation_cases()
        np.savez_compressed(os.path.join(OUT, 'generation.npz'), **arr)
        with open(os.path.join(OUT, 'generation.json'), 'w') as f:
            json.dump(man, f, indent=1)
        print('generation: %d cases, %s plies' % (len(man), [c['steps'] for c in man]))
        if only:
            return
    if only == ['trainer']:
        arr, meta = trainer_case()
        np.savez_compressed(os.path.join(OUT, 'trainer.npz'), **arr)
        with open(os.path.join(OUT, 'trainer.json'), 'w') as f:
            json.dump(meta, f, indent=1)
        print('trainer: %d epochs' % len(meta['epochs']))
        return
    if only == ['geese']:
        arr, meta = geese_net_case()
        np.savez_compressed(os.path.join(OUT, 'geese_net.npz'), **arr)
        with open(os.path.join(OUT, 'geese_net.json'), 'w') as f:
            json.dump(meta, f, indent=1)
        print('geese net: %d tensors' % len(meta['state']))
        return
    arr, man = target_cases()
    np.savez_compressed(os.path.join(OUT, 'targets.npz'), **arr)
    with open(os.path.join(OUT, 'targets.json'), 'w') as f:
        json.dump(man, f, indent=0)
    print('targets: %d cases' % len(man))

    arr, man = loss_cases()
    np.savez_compressed(os.path.join(OUT, 'loss.npz'), **arr)
    with open(os.path.join(OUT, 'loss.json'), 'w') as f:
        json.dump(man, f, indent=1)
    print('loss: %d cases' % len(man))

    arr, man = make_batch_cases()
    np.savez_compressed(os.path.join(OUT, 'make_batch.npz'), **arr)
    with open(os.path.join(OUT, 'make_batch.json'), 'w') as f:
        json.dump(man, f)
    print('make_batch: %d cases' % len(man))

    arr, games = tictactoe_rules()
    np.savez_compressed(os.path.join(OUT, 'tictactoe_rules.npz'), **arr)
    with open(os.path.join(OUT, 'tictactoe_rules.json'), 'w') as f:
        json.dump(games, f)
    print('tictactoe rules: %d games' % len(games))

    arr, games = geister_rules()
    np.savez_compressed(os.path.join(OUT, 'geister_rules.npz'), **arr)
    with open(os.path.join(OUT, 'geister_rules.json'), 'w') as f:
        json.dump(games, f)
    print('geister rules: %d games, %d plies, win colours %s' % (
        len(games), sum(g['plies'] for g in games), sorted(g['win_color'] for g in games)))

    arr, meta = geister_net_case()
    np.savez_compressed(os.path.join(OUT, 'geister_net.npz'), **arr)
    with open(os.path.join(OUT, 'geister_net.json'), 'w') as f:
        json.dump(meta, f, indent=1)
    print('geister net: %d tensors' % len(meta['state']))

    arr, meta = geese_net_case()
    np.savez_compressed(os.path.join(OUT, 'geese_net.npz'), **arr)
    with open(os.path.join(OUT, 'geese_net.json'), 'w') as f:
        json.dump(meta, f, indent=1)
    print('geese net: %d tensors' % len(meta['state']))

    arr, meta = trainer_case()
    np.savez_compressed(os.path.join(OUT, 'trainer.npz'), **arr)
    with open(os.path.join(OUT, 'trainer.json'), 'w') as f:
        json.dump(meta, f, indent=1)
    print('trainer: %d epochs' % len(meta['epochs']))

    arr, meta = learner_case()
    np.savez_compressed(os.path.join(OUT, 'learner.npz'), **arr)
    with open(os.path.join(OUT, 'learner.json'), 'w') as f:
        json.dump(meta, f, indent=1)
    print('learner: %d steps' % len(meta['steps']))


if __name__ == '__main__':
    main()
