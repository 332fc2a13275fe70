"""Device-resident batched self-play and replay for the learner.

The reference plays one game per worker process, one batch-1 CPU inference
per player per ply (generation.py:20-88, model.py:43-53), ships each episode
as bz2(pickle) blocks over TCP/pipes (generation.py:79-86, worker.py), and a
batcher process rebuilds padded training windows on the CPU (train.py:33-133,
284-302).  Here thousands of games advance together on the GPU:

* ``TicTacToeBatch``  E concurrent games as tensors, rules of
  handyrl/envs/tictactoe.py:103-172 (black moves first, 8 winning lines,
  outcome +-1 / 0, 3-plane observation relative to the viewing player);
* ``DeviceGenerator`` one batched forward of the env network per ply for
  every live game, the reference's legal-action masking (-1e32,
  generation.py:49-52) and categorical sampling over the legal actions by
  Gumbel-max (the same distribution as ``random.choices(legal,
  weights=softmax(p[legal]))``, generation.py:53), episode returns as the
  reference's discounted sum (generation.py:73-77);
* ``DeviceReplay``    a ring buffer of episodes in HBM; ``sample`` draws
  windows with the reference Batcher's recency-weighted episode choice and
  uniform window start (train.py:284-293) and gathers them straight into the
  make_batch layout (train.py:109-133) the learner consumes -- no host copy,
  no pickling.

Training modes.  With turn_based_training=True and observation=False (the
stock configuration) only the player to move runs inference each ply and the
episode records one mover per ply.  With ``observation=True`` (every player
infers every ply, generation.py:35-46) or a simultaneous-move env
(``SIMULTANEOUS``, e.g. ``ParallelTicTacToeBatch``: every player moves every
ply, parallel_tictactoe.py:20-24) ``DeviceGenerator`` runs the per-player
ply instead: one forward over all P x E (player, game) views, per-player
recurrent state in HBM advanced for the players that inferred, the turn
players sampled, per-player records with the turn and observation masks;
``PlayerReplay`` gathers those into make_batch's per-player layout
(train.py:63-67), one random player per window for solo training
(turn_based_training=False, train.py:55-56).
"""

import contextlib

import numpy as np
import torch

from .util import map_r, bimap_r

__all__ = ['TicTacToeBatch', 'ParallelTicTacToeBatch', 'DeviceGenerator', 'DeviceReplay', 'PlayerReplay',
           'episodes_to_wire', 'player_episodes_to_wire', 'reference_uniforms']


class TicTacToeBatch:
    """E TicTacToe games on one device (handyrl/envs/tictactoe.py:72-172)."""

    A = 9
    P = 2
    MAX_PLIES = 9
    ALTERNATING = True   # the mover is ply % 2 in every live game
    OBS_SHAPE = (3, 3, 3)
    LINES = ((0, 1, 2), (3, 4, 5), (6, 7, 8), (0, 3, 6), (1, 4, 7), (2, 5, 8), (0, 4, 8), (2, 4, 6))

    def __init__(self, E, device):
        self.E, self.device = E, device
        self.lines = torch.tensor(self.LINES, device=device)
        self.reset()

    def reset(self):
        """State tensors are allocated once and then reset and advanced in place, so a HIP graph captured
        over a ply (DeviceGenerator) keeps addressing them."""
        E, dev = self.E, self.device
        if not hasattr(self, 'board'):
            self.board = torch.zeros(E, 9, dtype=torch.int8, device=dev)     # +1 black, -1 white
            self.color = torch.ones(E, dtype=torch.int8, device=dev)          # side to move
            self.nmoves = torch.zeros(E, dtype=torch.int32, device=dev)
            self.winner = torch.zeros(E, dtype=torch.int8, device=dev)
        self.board.zero_()
        self.color.fill_(1)
        self.nmoves.zero_()
        self.winner.zero_()

    def turn(self):
        """Index of the player to move: 0 (black) on even plies."""
        return (self.nmoves % 2).long()

    def plies(self):
        return self.nmoves

    def terminal(self):
        return (self.winner != 0) | (self.nmoves >= 9)

    def legal(self):
        return self.board == 0

    def observation(self, player):
        """(E,3,3,3): [turn-view indicator, own stones, opponent stones] for `player` (E,) (tictactoe.py:157-168)."""
        turn_view = player == self.turn()
        me = torch.where(turn_view, self.color, -self.color).view(-1, 1)
        b = self.board
        planes = torch.stack([turn_view.view(-1, 1).expand(-1, 9), b == me, b == -me], dim=1)
        return planes.float().view(-1, 3, 3, 3)

    def step(self, action, active):
        """Play `action` (E,) for the side to move in every `active` game (tictactoe.py:103-118)."""
        rows = torch.arange(self.E, device=self.device)
        act = torch.where(active, action, torch.zeros_like(action))
        new = torch.where(active, self.color, self.board[rows, act])
        self.board[rows, act] = new
        sums = self.board.long()[:, self.lines].sum(-1)                   # (E, 8)
        won = active & (sums == 3 * self.color.long().view(-1, 1)).any(-1)
        self.winner.copy_(torch.where(won, self.color, self.winner))
        self.color.copy_(torch.where(active, -self.color, self.color))
        self.nmoves.add_(active.int())

    def outcome(self):
        """(E, 2) float: +1/-1 for the winner/loser, 0/0 for a draw (tictactoe.py:140-147)."""
        w = self.winner.float()
        return torch.stack([w, -w], dim=1)

    def turns_mask(self):
        """(E, P) bool: the players to move (turns(), environment.py:107-113): the side to move."""
        return torch.nn.functional.one_hot(self.turn(), self.P).bool()


class ParallelTicTacToeBatch(TicTacToeBatch):
    """E Parallel Tic-Tac-Toe games (handyrl/envs/parallel_tictactoe.py:13-61): both players choose a move every
    ply (turns() = both) and one of them, picked uniformly, is played with its own colour.  The reference's turn()
    returns an exception object, so observation(p) is the non-turn view for both p, and its colour never changes
    from black: both players see [zeros, white stones, black stones] (tictactoe.py:157-168)."""

    ALTERNATING = False
    SIMULTANEOUS = True

    def turns_mask(self):
        return torch.ones(self.E, self.P, dtype=torch.bool, device=self.device)

    def turn(self):
        return torch.zeros(self.E, dtype=torch.long, device=self.device)

    def observation(self, player):
        b = self.board
        planes = torch.stack([torch.zeros_like(b, dtype=torch.bool), b == -1, b == 1], dim=1)
        return planes.float().view(-1, 3, 3, 3)

    def step_players(self, actions, turns, active, u):
        """The played player: floor(u * P) of the E uniforms u (random.choice over the action dict's P keys,
        parallel_tictactoe.py:21); its action with its colour, player 0 black (parallel_tictactoe.py:25-35)."""
        rows = torch.arange(self.E, device=self.device)
        sel = torch.clamp((u * self.P).long(), max=self.P - 1)
        act = torch.where(active, actions[rows, sel], torch.zeros_like(sel))
        colour = torch.where(sel == 0, 1, -1).to(self.board.dtype)
        self.board[rows, act] = torch.where(active, colour, self.board[rows, act])
        sums = self.board.long()[:, self.lines].sum(-1)                   # (E, 8)
        won = active & (sums == 3 * colour.long().view(-1, 1)).any(-1)
        self.winner.copy_(torch.where(won, colour, self.winner))
        self.nmoves.add_(active.int())


def _leaves(x):
    """The tensors of a nested list / tuple / dict, in order."""
    out = []
    map_r(x, out.append)
    return out


def _alloc(spec, lead, device, dtype=torch.float32):
    """Zero tensors (*lead, *shape) for an observation spec: a shape tuple or {name: shape}."""
    if isinstance(spec, dict):
        return {k: torch.zeros(*lead, *v, device=device, dtype=dtype) for k, v in spec.items()}
    return torch.zeros(*lead, *spec, device=device, dtype=dtype)


def _stack_views(views, batch_first=False):
    """P views (each a tensor (E, ...) or {name: (E, ...)}) -> (P * E, ...) player-major, or (E, P, ...)."""
    def stack(xs):
        return torch.stack(xs, 1) if batch_first else torch.cat(xs, 0)
    if isinstance(views[0], dict):
        return {k: stack([v[k] for v in views]) for k in views[0]}
    return stack(views)


def reference_uniforms(seeds, Tm, P, simultaneous=False):
    """The random-stream values seeded reference games draw (generation.py:53, parallel_tictactoe.py:21): for
    game k, ``random.seed(seeds[k])`` then per ply each turn player's ``random.choices`` takes one ``random()``
    (players in order: the mover, ply % P, or every player of a simultaneous env) and a simultaneous env's step
    one ``random.choice`` over the P players.  Returns u (E, Tm, P) float64 and sel (E, Tm) int64 (None for
    alternating envs), for ``DeviceGenerator.generate(reference=...)``.  Draws past a game's end are unused."""
    import random as _random
    E = len(seeds)
    u = np.zeros((E, Tm, P), dtype=np.float64)
    sel = np.zeros((E, Tm), dtype=np.int64) if simultaneous else None
    for e, seed in enumerate(seeds):
        r = _random.Random(seed)
        for t in range(Tm):
            for p in (range(P) if simultaneous else (t % P,)):
                u[e, t, p] = r.random()
            if simultaneous:
                sel[e, t] = r.choice(list(range(P)))
    return u, sel


def sample_record_torch(st, logits, legal, value, active, player, reward):
    """The ply's sampling and recording tail as torch ops (generation.py:43-62): illegal logits masked by
    -1e32, Gumbel-max over the ply's uniforms st['U'][t] (the distribution of random.choices over the softmax
    of the legal logits), and slot t of the policy / action mask / action / value / turn / reward records
    (reset values for finished games).  Returns the sampled action per game."""
    E, t = logits.shape[0], st['t']
    m = torch.where(legal, 0.0, 1e32)                                  # generation.py:50-51
    p = logits - m
    u = st['U'].index_select(0, t).view(E, -1)
    a = torch.argmax(p - torch.log(-torch.log(u)), dim=-1)              # Gumbel-max = softmax over legal

    def record(buf, x, fill=0):
        live = active.view(-1, *([1] * (x.dim() - 1)))
        buf.index_copy_(1, t, torch.where(live, x, fill).to(buf.dtype).unsqueeze(1))
    record(st['policy'], p)
    record(st['amask'], m, 1e32)
    record(st['action'], a)
    record(st['value'], value.reshape(-1))
    record(st['turn'], player)
    if reward is not None:
        record(st['reward'], reward)
    return a


def sample_record_hip(st, logits, legal, value, active, player, reward):
    """sample_record_torch as ONE launch (csrc/hrl_selfplay.hip, one wave per game): the same fp32 operations,
    torch.argmax's tie order, the same records."""
    from . import _native
    E, A = logits.shape
    Tm = st['action'].shape[1]
    P = st['reward'].shape[2]
    logits = logits.float()
    if logits.stride(1) != 1:
        logits = logits.contiguous()
    value = value.reshape(E).float().contiguous()
    legal, active = legal.contiguous(), active.contiguous()
    player = player.to(torch.long).contiguous()
    assert legal.shape == (E, A) and legal.dtype == torch.bool and active.shape == (E,) and player.shape == (E,)
    assert st['policy'].shape == (E, Tm, A) and st['U'].shape == (Tm, E, A)
    if reward is not None:
        reward = reward.to(torch.float64).contiguous()
        assert reward.shape == (E, P)
    a = torch.empty(E, dtype=torch.long, device=logits.device)
    _native.check(_native.load().hrl_selfplay_sample_record(
        _native.ptr(logits), logits.stride(0), _native.ptr(legal), _native.ptr(st['U']), _native.ptr(st['t']),
        _native.ptr(value), _native.ptr(active), _native.ptr(player), _native.ptr(reward), E, A, Tm, P,
        _native.ptr(a), _native.ptr(st['policy']), _native.ptr(st['amask']), _native.ptr(st['action']),
        _native.ptr(st['value']), _native.ptr(st['turn']), None if reward is None else _native.ptr(st['reward']),
        _native.stream_of(logits.device)), 'hrl_selfplay_sample_record')
    return a


class DeviceGenerator:
    """Batched self-play of E games with one env-network forward per ply (generation.py:20-88).

    Recurrent nets (``init_hidden``, e.g. GeisterNet) keep one hidden state
    per game and player in HBM, starting from ``init_hidden`` zeros; each ply
    only the mover's state advances (generation.py:23-25, 38-41).  Rewards
    (``env.reward()``, e.g. Geister's -0.01 per ply) are recorded for both
    players every ply and turned into discounted returns in fp64 exactly as
    the reference's Python-float loop (generation.py:73-77).

    Every buffer of a call (episode tensors, hidden state, the ply's uniforms,
    the ply index as a device scalar) is allocated once and reset in place, and
    the ply body addresses the current ply through that device scalar.  So on
    a GPU the ply is captured ONCE per mover parity as a HIP graph (``graph``;
    default: on for CUDA envs whose mover is ply % P) and each ply is one
    graph replay instead of ≈100 small launches; the discounted-return loop is
    a third graph.  Eager and graph mode run the same ply function on the same
    uniforms (one (Tm, E, A) draw per call), so they give the same episodes.

    ``observation=True`` or a ``SIMULTANEOUS`` env selects the per-player ply
    (module doc; ``_ply_players``): the episode's records gain a player axis
    (E, Tm, P, ...) with ``tmask`` / ``omask``; its ply is one graph for every
    ply.  ``generate(reference=(u, sel))`` samples by the reference's inverse
    CDF instead of Gumbel-max: u (E, Tm, P) are the ``random()`` values each
    turn player's ``random.choices`` draws and sel (E, Tm) the simultaneous
    env's played-player uniforms (``reference_uniforms``), so seeded reference
    games replay move for move.
    """

    def __init__(self, env_batch, net, gamma=0.8, check_every=16, graph=None, observation=False, per_player=None):
        self.env = env_batch
        self.net = net
        self.gamma = gamma
        self.check_every = check_every
        self.graph = graph
        self.observation = bool(observation)
        # per_player=True also for a mover-only alternating game whose batches need per-player records (solo)
        self.per_player = (self.observation or getattr(env_batch, 'SIMULTANEOUS', False) if per_player is None
                           else bool(per_player) or self.observation or getattr(env_batch, 'SIMULTANEOUS', False))
        self._st = None

    def _use_graph(self):
        dev = torch.device(self.env.device)
        if self.graph is None:
            return dev.type == 'cuda' and (self.per_player or getattr(self.env, 'ALTERNATING', False))
        return bool(self.graph) and dev.type == 'cuda'

    def _state(self):
        """The call's buffers, allocated once per (generator, net)."""
        # a captured ply reads the net's parameters and buffers where they live: recapture if any moved
        key = tuple(t.data_ptr() for t in list(self.net.parameters()) + list(self.net.buffers()))
        if self._st is not None and self._st['net'] is self.net and self._st['key'] == key:
            return self._st
        env, E, dev = self.env, self.env.E, self.env.device
        Tm, A, P = env.MAX_PLIES, env.A, env.P
        st = {'net': self.net, 'key': key, 'graphs': None,
              'obs': _alloc(env.OBS_SHAPE, (E, Tm), dev),
              'policy': torch.zeros(E, Tm, A, device=dev),
              'amask': torch.full((E, Tm, A), 1e32, device=dev),
              'action': torch.zeros(E, Tm, dtype=torch.long, device=dev),
              'value': torch.zeros(E, Tm, device=dev),
              'turn': torch.zeros(E, Tm, dtype=torch.long, device=dev),
              'reward': torch.zeros(E, Tm, P, device=dev, dtype=torch.float64),  # Python floats in the reference
              'ret': torch.zeros(E, Tm, P, device=dev),
              'U': torch.empty(Tm, E, A, device=dev),
              't': torch.zeros(1, dtype=torch.long, device=dev),
              'rows': torch.arange(E, device=dev),
              'hidden': None, 'obs_dev': torch.device(dev).type}
        if self.per_player:
            # records with a player axis; the uniforms (Tm, E, P, A) for Gumbel-max, (E, Tm, P) / (E, Tm) for the
            # reference sampler; the state (P, E, ...): the (player, game) rows of one forward are its view
            st.update(obs=_alloc(env.OBS_SHAPE, (E, Tm, P), dev),
                      policy=torch.zeros(E, Tm, P, A, device=dev),
                      amask=torch.full((E, Tm, P, A), 1e32, device=dev),
                      action=torch.zeros(E, Tm, P, dtype=torch.long, device=dev),
                      value=torch.zeros(E, Tm, P, device=dev),
                      tmask=torch.zeros(E, Tm, P, dtype=torch.bool, device=dev),
                      omask=torch.zeros(E, Tm, P, dtype=torch.bool, device=dev),
                      U=torch.empty(Tm, E, P, A, device=dev),
                      Uref=torch.zeros(E, Tm, P, dtype=torch.float64, device=dev),
                      Usel=torch.empty(Tm, E, device=dev),
                      ref_mode=False, rank=False,
                      players=torch.arange(P, device=dev).view(P, 1).expand(P, E).contiguous(), pmajor=True)
            st['flat_state'] = False
            if (self.observation and hasattr(self.net, 'inference_hidden') and hasattr(self.net, 'inference_session')
                    and torch.device(dev).type == 'cuda'):
                # every player infers every ply: the net's own stacked layout over the P*E rows, advanced in place
                # inside its inference session (GeisterNet), leaves (P*E, ...) player-major
                st['hidden'] = map_r(self.net.inference_hidden(P * E, 1, dev), lambda h: h[0])
                st['flat_state'] = True
            elif hasattr(self.net, 'init_hidden'):
                st['hidden'] = map_r(self.net.init_hidden([P, E]), lambda h: h.to(dev).contiguous())
            self._st = st
            return st
        st['pmajor'] = False   # state leaves (E, P, ...) as init_hidden gives them
        if hasattr(self.net, 'inference_hidden') and torch.device(dev).type == 'cuda':
            st['hidden'] = self.net.inference_hidden(E, P, dev)   # leaves (P, E, ...), the net's own layout
            st['pmajor'] = True
        elif hasattr(self.net, 'init_hidden'):
            st['hidden'] = map_r(self.net.init_hidden([E, P]), lambda h: h.to(dev).contiguous())
        self._st = st
        return st

    def _reset(self, st, generator, draw=True):
        self.env.reset()
        map_r(st['obs'], lambda b: b.zero_())
        for k in ('policy', 'action', 'value', 'turn', 'reward', 'ret') + (('tmask', 'omask') if self.per_player
                                                                           else ()):
            st[k].zero_()
        st['amask'].fill_(1e32)
        if st['hidden'] is not None:
            map_r(st['hidden'], lambda h: h.zero_())
        if draw:
            torch.rand(st['U'].shape, out=st['U'], generator=generator, device=st['U'].device)
            st['U'].clamp_(1e-20, 1.0)
            if self.per_player:
                torch.rand(st['Usel'].shape, out=st['Usel'], generator=generator, device=st['Usel'].device)
        st['t'].zero_()

    def _ply_players(self, st):
        """The per-player ply (generation.py:35-62 with observation, or every player a turn player): every
        (player, game) view in one forward -- the players that infer are the turn players, or all with
        ``observation`` --, their values / observations recorded and their state advanced, the turn players'
        policies masked and sampled, then the env steps on the turn players' actions."""
        env, E, P, A = self.env, self.env.E, self.env.P, self.env.A
        t = st['t']
        hidden = st['hidden']
        # a snapshot: an env's active() may be state its step updates in place (GeisterBatch.live), and the
        # reward after the step is recorded for the games that were live before it
        active = (env.active() if hasattr(env, 'active') else ~env.terminal()).clone()
        live = active.view(E, 1)
        turns = (env.turns_mask() if hasattr(env, 'turns_mask') else
                 torch.nn.functional.one_hot(env.turn().long(), P).bool()) & live          # (E, P)
        infer = live.expand(E, P) if self.observation else turns
        views = [env.observation(st['players'][p]) for p in range(P)]
        o = _stack_views(views)                                                           # (P * E, ...)
        h_in = (None if hidden is None else hidden if st['flat_state'] else
                map_r(hidden, lambda h: h.view(P * E, *h.shape[2:])))
        out = self.net(o, h_in)
        logits = out['policy'].float().view(P, E, A).transpose(0, 1)                   # (E, P, A)
        value = out['value'].float().reshape(P, E).t()                                  # (E, P)
        legal = (env.legal_players() if hasattr(env, 'legal_players') else
                 env.legal().view(E, 1, A).expand(E, P, A))
        m = torch.where(legal, 0.0, 1e32)                                                 # generation.py:50-51
        p = logits - m
        # Gumbel-max over the legal logits (softmax sampling), or the reference's inverse CDF of random.choices:
        # bisect(cumsum(softmax(p[legal])), u * total), fp64 here (the reference's fp32 sums decide otherwise only
        # when u falls within their rounding of a boundary)
        if not st['ref_mode']:
            g = st['U'].index_select(0, t).view(E, P, A)
            a = torch.argmax(p - torch.log(-torch.log(g)), dim=-1)
        else:
            # the reference's legal_actions order: ascending labels, or the env's own (legal_rank: Geister's pieces)
            base = (env.legal_rank().view(E, 1, A) if st['rank'] else
                    torch.arange(A, device=p.device).view(1, 1, A)).expand(E, P, A)
            order = torch.argsort(torch.where(legal, base, 1 << 30), dim=-1, stable=True)    # legal ones first
            lo = torch.gather(legal, -1, order)
            pd = torch.where(lo, torch.gather(p, -1, order).double(), float('-inf'))
            w = torch.exp(pd - pd.max(-1, keepdim=True).values)
            cum = torch.cumsum(w / w.sum(-1, keepdim=True), -1)
            x = st['Uref'].index_select(1, t).view(E, P, 1) * cum[..., -1:]
            k = ((cum <= x) & lo).sum(-1, keepdim=True)                                  # bisect_right over legal
            k = torch.minimum(k, lo.sum(-1, keepdim=True) - 1).clamp(min=0)
            a = torch.gather(order, -1, k).squeeze(-1)                                   # legal entries lead

        def record(buf, x, mask, fill=0):
            keep = mask.view(*mask.shape, *([1] * (x.dim() - mask.dim())))
            buf.index_copy_(1, t, torch.where(keep, x, fill).to(buf.dtype).unsqueeze(1))
        views_e = _stack_views(views, batch_first=True)                                   # (E, P, ...)
        bimap_r(st['obs'], views_e, lambda b, v: record(b, v, infer))
        record(st['value'], value, infer)
        record(st['policy'], p, turns)
        record(st['amask'], m, turns, 1e32)
        record(st['action'], a, turns)
        record(st['tmask'], turns, turns)
        record(st['omask'], infer, infer)
        if hidden is not None and st['flat_state']:
            # the session advanced every (player, game) row in place -- all of them inferred (observation); a
            # finished game's rows moved too, but nothing reads them again.  Without the in-place form: a copy
            dst, src = _leaves(hidden), _leaves(out['hidden'])
            if not all(d.data_ptr() == x.data_ptr() and d.stride() == x.stride() for d, x in zip(dst, src)):
                for d, x in zip(dst, src):
                    d.copy_(x)
        elif hidden is not None:                                   # only the players that inferred advance
            keep = infer.t().contiguous()                          # (P, E)

            def advance(h, nh):
                nh = nh.view(h.shape)
                h.copy_(torch.where(keep.view(P, E, *([1] * (h.dim() - 2))), nh, h))
            bimap_r(hidden, out['hidden'], advance)
        if getattr(env, 'SIMULTANEOUS', False):
            env.step_players(a, turns, active, st['Usel'].index_select(0, t).view(E))
        else:
            rows = torch.arange(E, device=a.device)
            env.step(a[rows, env.turn().long()], active)
        if hasattr(env, 'reward'):
            r = env.reward().to(st['reward'].dtype)
            st['reward'].index_copy_(1, t, torch.where(live, r, 0).unsqueeze(1))
        t.add_(1)

    def _ply(self, st, mover):
        """One ply for every game at ply index st['t'] (a device scalar, advanced here); ``mover``: the
        player index every live game moves with (ALTERNATING envs), or None."""
        if self.per_player:
            return self._ply_players(st)
        env, E = self.env, self.env.E
        t = st['t']
        hidden = st['hidden']
        active = env.active() if hasattr(env, 'active') else ~env.terminal()
        player = env.turn()
        # envs with a GPU observation kernel record the view into slot t in the same launch
        obs_recorded = st['obs_dev'] == 'cuda' and hasattr(env, 'observation_record')
        o = env.observation_record(player, st['obs'], t, active) if obs_recorded else env.observation(player)
        # envs whose mover is ply % P in every live game (TicTacToe, Geister): the mover's state is a view
        if hidden is None:
            h_in = None
        elif mover is not None:
            h_in = map_r(hidden, (lambda h: h[mover]) if st['pmajor'] else (lambda h: h[:, mover]))
        elif st['pmajor']:
            h_in = map_r(hidden, lambda h: h[player, st['rows']])
        else:
            h_in = map_r(hidden, lambda h: h[st['rows'], player])
        out = self.net(o, h_in)
        # the reference reads the reward after env.step (generation.py:59-65); an env whose reward does not
        # depend on the state (REWARD_STATELESS, e.g. Geister's -0.01 per ply) has it recorded by the
        # sampling launch, any other env's after its step below
        has_reward = hasattr(env, 'reward')
        early = has_reward and getattr(env, 'REWARD_STATELESS', False)
        reward = env.reward() if early else None
        # slot t of every record is written once per call, so a finished game keeps the reset value
        def record(buf, x, fill=0):
            live = active.view(-1, *([1] * (x.dim() - 1)))
            buf.index_copy_(1, t, torch.where(live, x, fill).to(buf.dtype).unsqueeze(1))
        if not obs_recorded:
            bimap_r(st['obs'], o, record)
        sample = sample_record_hip if st['obs_dev'] == 'cuda' else sample_record_torch
        a = sample(st, out['policy'], env.legal(), out['value'], active, player, reward)
        if hidden is not None and mover is not None and st['obs_dev'] == 'cuda':
            dst = [h[mover] if st['pmajor'] else h[:, mover] for h in _leaves(hidden)]
            src = _leaves(out['hidden'])
            # a net that advanced its stacked state in place (GeisterNet in an in-place session) left nothing to
            # copy: finished games' states moved too, but nothing reads them again (their records are reset
            # values); otherwise one HIP launch for every state tensor instead of a where + copy per tensor
            if not all(d.data_ptr() == x.data_ptr() and d.stride() == x.stride() for d, x in zip(dst, src)):
                from .nn import masked_rows_copy_
                masked_rows_copy_(dst, src, active.contiguous())
        elif hidden is not None:
            def advance(h, nh):
                live = active.view(-1, *([1] * (nh.dim() - 1)))
                if st['pmajor']:
                    h[player, st['rows']] = torch.where(live, nh, h[player, st['rows']])
                elif mover is not None:
                    h[:, mover].copy_(torch.where(live, nh, h[:, mover]))
                else:
                    h[st['rows'], player] = torch.where(live, nh, h[st['rows'], player])
            bimap_r(hidden, out['hidden'], advance)
        env.step(a, active)
        if has_reward and not early:
            r = env.reward().to(st['reward'].dtype)
            st['reward'].index_copy_(1, t, torch.where(active.view(-1, 1), r, 0).unsqueeze(1))
        t.add_(1)

    def _returns(self, st):
        """Discounted returns per player, fp64 like the reference's Python floats (generation.py:73-77)."""
        reward, ret = st['reward'], st['ret']
        acc = torch.zeros_like(reward[:, 0])
        for t in range(reward.shape[1] - 1, -1, -1):
            acc = reward[:, t] + self.gamma * acc
            ret[:, t].copy_(acc)

    def _capture(self, st, keys):
        """Graphs of the ply (one per mover key) and of the return loop; warm-up plies run first on a side
        stream (library workspaces), then the state is reset."""
        dev = torch.device(self.env.device)
        side = torch.cuda.Stream(dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            for k in keys:
                self._ply(st, k)
            self._returns(st)
        torch.cuda.current_stream(dev).wait_stream(side)
        graphs, pool = {}, None
        for k in list(keys) + ['returns']:
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, pool=pool):
                if k == 'returns':
                    self._returns(st)
                else:
                    self._ply(st, k)
            pool = g.pool()
            graphs[k] = g
        st['graphs'] = graphs
        self._reset(st, None, draw=False)   # the call's uniforms stay as drawn

    @torch.no_grad()
    def generate(self, generator=None, reference=None):
        """One batch of E games; ``reference`` (per-player mode): (u, sel) from ``reference_uniforms``."""
        alternating = getattr(self.env, 'ALTERNATING', False) and not self.per_player
        st = self._state()
        if reference is not None and not self.per_player:
            raise ValueError('the reference sampler is the per-player ply\'s (observation or simultaneous envs)')
        was_training = self.net.training
        self.net.eval()
        # per-call weight preparation (GeisterNet); its own stacked state is advanced in place by the net (the
        # per-player ply too when every player infers; otherwise it runs the net's ordinary forward)
        session = (getattr(self.net, 'inference_session', None)
                   if (not self.per_player or st.get('flat_state')) else None)
        with session(inplace_state=st['pmajor']) if session is not None else contextlib.nullcontext():
            out = self._generate(st, generator, alternating, reference)
        self.net.train(was_training)
        return out

    def _generate(self, st, generator, alternating, reference=None):
        env = self.env
        Tm, P = env.MAX_PLIES, env.P
        if self.per_player:
            # the sampler is part of the captured ply: a change of sampler recaptures it; an env whose
            # legal_actions order is not ascending keeps what gives it (Geister: piece indices)
            ref_mode = reference is not None
            if ref_mode != st['ref_mode']:
                st['ref_mode'], st['graphs'] = ref_mode, None
            st['rank'] = ref_mode and hasattr(env, 'legal_rank')
            if st['rank'] and getattr(env, 'pidx', None) is None:
                env.piece_order(True)
                st['graphs'] = None
        self._reset(st, generator)
        if self.per_player:
            if reference is not None:
                u, sel = reference
                st['Uref'].copy_(torch.as_tensor(u, dtype=torch.float64))
                if sel is not None:   # the played player p is floor(Usel * P): the middle of its interval
                    st['Usel'].copy_(((torch.as_tensor(sel, dtype=torch.float64) + 0.5) / P).t().float())
        graphs = None
        if self._use_graph():
            if st['graphs'] is None:
                self._capture(st, list(range(P)) if alternating else [None])
            graphs = st['graphs']
        for t in range(Tm):
            if t and self.check_every and t % self.check_every == 0 and bool(env.terminal().all()):
                break
            mover = t % P if alternating else None
            if graphs is not None:
                graphs[mover].replay()
            else:
                self._ply(st, mover)
        if hasattr(env, 'reward'):
            if graphs is not None:
                graphs['returns'].replay()
            else:
                self._returns(st)
        out = {'observation': map_r(st['obs'], lambda b: b.clone())}
        for key, k in (('policy', 'policy'), ('action_mask', 'amask'), ('action', 'action'), ('value', 'value'),
                       ('turn', 'turn'), ('return', 'ret')) + ((('tmask', 'tmask'), ('omask', 'omask'))
                                                            if self.per_player else ()):
            out[key] = st[k].clone()
        out.update(length=env.plies().long(), outcome=env.outcome(), reward=st['reward'].float())
        return out


class DeviceReplay:
    """Ring buffer of episodes in HBM; windows gathered into the make_batch layout.

    ``obs_shape`` is a shape or {name: shape}; ``obs_dtype`` lets binary
    observation planes (TicTacToe, Geister) live in HBM as uint8, a quarter
    of the bytes, widened to fp32 by the gather.
    """

    def __init__(self, capacity, max_plies, obs_shape, A, P, device, maximum_episodes=None,
                 obs_dtype=torch.float32):
        self.N, self.Tm, self.P, self.device = capacity, max_plies, P, device
        self.maximum_episodes = maximum_episodes or capacity
        f = dict(device=device)
        self.obs = _alloc(obs_shape, (capacity, max_plies), device, obs_dtype)
        self.policy = torch.zeros(capacity, max_plies, A, **f)
        self.amask = torch.full((capacity, max_plies, A), 1e32, **f)
        self.action = torch.zeros(capacity, max_plies, dtype=torch.long, **f)
        self.value = torch.zeros(capacity, max_plies, **f)
        self.turn = torch.zeros(capacity, max_plies, dtype=torch.long, **f)
        self.reward = torch.zeros(capacity, max_plies, P, **f)
        self.ret = torch.zeros(capacity, max_plies, P, **f)
        self.length = torch.ones(capacity, dtype=torch.long, **f)
        self.outcome = torch.zeros(capacity, P, **f)
        self.ptr = 0      # next slot
        self.count = 0    # stored episodes (<= capacity)

    def add(self, ep):
        E = ep['length'].shape[0]
        slots = (self.ptr + torch.arange(E, device=self.device)) % self.N
        bimap_r(self.obs, ep['observation'], lambda dst, src: dst.index_copy_(0, slots, src.to(dst.dtype)))
        for dst, key in ((self.policy, 'policy'), (self.amask, 'action_mask'),
                         (self.action, 'action'), (self.value, 'value'), (self.turn, 'turn'),
                         (self.reward, 'reward'), (self.ret, 'return'), (self.length, 'length'),
                         (self.outcome, 'outcome')):
            dst.index_copy_(0, slots, ep[key])
        self.ptr = (self.ptr + E) % self.N
        self.count = min(self.count + E, self.N)

    def _age_order(self):
        """Slot of the i-th oldest stored episode (i = 0 oldest)."""
        start = (self.ptr - self.count) % self.N
        return (start + torch.arange(self.count, device=self.device)) % self.N

    def sample_windows(self, B, T, generator=None):
        """(slot, start) of B windows, as Batcher.select_episode draws them (train.py:284-293).

        Episode i of the n newest (i = n-1 newest) is accepted with probability
        1 - (n-1-i)/maximum_episodes; drawing from that weighting directly is
        the distribution of the reference's rejection loop.
        """
        n = min(self.count, self.maximum_episodes)
        i = torch.arange(n, device=self.device, dtype=torch.float64)
        w = 1.0 - (n - 1 - i) / self.maximum_episodes
        pick = torch.multinomial(w.float(), B, replacement=True, generator=generator)
        slots = self._age_order()[self.count - n:][pick]
        steps = self.length[slots]
        cand = 1 + torch.clamp(steps - T, min=0)
        u = torch.rand(B, device=self.device, generator=generator)
        start = torch.minimum((u * cand).long(), cand - 1)
        return slots, start

    def gather(self, slots, start, T):
        """make_batch-layout batch of the windows [start, start+T) of episodes `slots` (train.py:33-133)."""
        B, P, dev = slots.shape[0], self.P, self.device
        t = start.view(-1, 1) + torch.arange(T, device=dev).view(1, -1)      # (B, T)
        length = self.length[slots].view(-1, 1)
        valid = t < length
        tc = torch.minimum(t, length - 1)
        e = slots.view(-1, 1)
        vf = valid.float()
        obs = map_r(self.obs, lambda o: (o[e, tc].float() * vf.view(B, T, *([1] * (o.dim() - 2)))).unsqueeze(2))
        pol = self.policy[e, tc] * vf.unsqueeze(-1)
        amask = torch.where(valid.unsqueeze(-1), self.amask[e, tc], torch.full_like(pol, 1e32))
        act = self.action[e, tc] * valid.long()
        onehot = torch.nn.functional.one_hot(self.turn[e, tc], P).float() * vf.unsqueeze(-1)   # (B,T,P)
        oc = self.outcome[slots].view(B, 1, P, 1)
        val = (onehot * self.value[e, tc].unsqueeze(-1)).unsqueeze(-1)
        val = torch.where(valid.view(B, T, 1, 1), val, oc.expand(B, T, P, 1))
        rew = self.reward[e, tc] * vf.unsqueeze(-1)
        ret = self.ret[e, tc] * vf.unsqueeze(-1)
        progress = torch.where(valid, t.float() / length.float(), torch.ones_like(vf))
        return {
            'observation': obs,
            'policy': pol.unsqueeze(2).contiguous(),
            'value': val.contiguous(),
            'action': act.view(B, T, 1, 1).contiguous(),
            'outcome': oc.contiguous(),
            'reward': rew.unsqueeze(-1).contiguous(),
            'return': ret.unsqueeze(-1).contiguous(),
            'episode_mask': vf.view(B, T, 1, 1).contiguous(),
            'turn_mask': onehot.unsqueeze(-1).contiguous(),
            'observation_mask': onehot.unsqueeze(-1).clone(),
            'action_mask': amask.unsqueeze(2).contiguous(),
            'progress': progress.unsqueeze(-1).contiguous(),
        }

    def sample(self, B, T, generator=None):
        slots, start = self.sample_windows(B, T, generator)
        return self.gather(slots, start, T)


class PlayerReplay(DeviceReplay):
    """DeviceReplay for the per-player episodes (``DeviceGenerator`` with ``observation`` or a simultaneous env):
    records (N, Tm, P, ...) with the turn and observation masks; ``gather`` forms make_batch's per-player layout
    (train.py:63-67, 76-83): every player, or one player per window (``players``, solo training, train.py:55-56),
    zeros / 1e32 / the outcome where a player did not infer or move and past the episode's end.  ``solo``
    (turn_based_training=False) samples one player per window; ``mover`` (turn_based_training without
    observation, e.g. a simultaneous env under the stock configuration) takes observation, policy, action and
    action mask from each ply's first turn player and the rest per player, as make_batch's first branch does
    (train.py:62-66)."""

    def __init__(self, capacity, max_plies, obs_shape, A, P, device, maximum_episodes=None,
                 obs_dtype=torch.float32, solo=False, mover=False):
        self.solo, self.mover = bool(solo), bool(mover)
        self.N, self.Tm, self.P, self.device = capacity, max_plies, P, device
        self.maximum_episodes = maximum_episodes or capacity
        f = dict(device=device)
        self.obs = _alloc(obs_shape, (capacity, max_plies, P), device, obs_dtype)
        self.policy = torch.zeros(capacity, max_plies, P, A, **f)
        self.amask = torch.full((capacity, max_plies, P, A), 1e32, **f)
        self.action = torch.zeros(capacity, max_plies, P, dtype=torch.long, **f)
        self.value = torch.zeros(capacity, max_plies, P, **f)
        self.tmask = torch.zeros(capacity, max_plies, P, dtype=torch.bool, **f)
        self.omask = torch.zeros(capacity, max_plies, P, dtype=torch.bool, **f)
        self.reward = torch.zeros(capacity, max_plies, P, **f)
        self.ret = torch.zeros(capacity, max_plies, P, **f)
        self.length = torch.ones(capacity, dtype=torch.long, **f)
        self.outcome = torch.zeros(capacity, P, **f)
        self.ptr = 0
        self.count = 0

    def add(self, ep):
        E = ep['length'].shape[0]
        slots = (self.ptr + torch.arange(E, device=self.device)) % self.N
        bimap_r(self.obs, ep['observation'], lambda dst, src: dst.index_copy_(0, slots, src.to(dst.dtype)))
        for dst, key in ((self.policy, 'policy'), (self.amask, 'action_mask'), (self.action, 'action'),
                         (self.value, 'value'), (self.tmask, 'tmask'), (self.omask, 'omask'),
                         (self.reward, 'reward'), (self.ret, 'return'), (self.length, 'length'),
                         (self.outcome, 'outcome')):
            dst.index_copy_(0, slots, ep[key].to(dst.dtype))
        self.ptr = (self.ptr + E) % self.N
        self.count = min(self.count + E, self.N)

    def gather(self, slots, start, T, players=None, mover=None):
        """make_batch of the windows [start, start+T) of episodes ``slots`` over every player, or over one
        player per window (``players`` (B,) long); ``mover`` (default: the replay's): observation, policy, action
        and action mask of each ply's first turn player."""
        mover = self.mover if mover is None else mover
        B, dev = slots.shape[0], self.device
        t = start.view(-1, 1) + torch.arange(T, device=dev).view(1, -1)      # (B, T)
        length = self.length[slots].view(-1, 1)
        valid = t < length
        tc = torch.minimum(t, length - 1)
        e = slots.view(-1, 1)
        pidx = (torch.arange(self.P, device=dev).view(1, 1, -1).expand(B, T, self.P) if players is None
                else players.view(B, 1, 1).expand(B, T, 1))
        # make_batch's first branch: m['turn'][0], the lowest-index turn player of the ply
        midx = torch.argmax(self.tmask[e, tc].long(), dim=-1, keepdim=True) if mover else pidx

        def take(x, ix=pidx):   # (N, Tm, P, ...) -> (B, T, Pn, ...)
            y = x[e, tc]
            Pn = ix.shape[2]
            idx = ix.reshape(B, T, Pn, *([1] * (y.dim() - 3))).expand(B, T, Pn, *y.shape[3:])
            return torch.gather(y, 2, idx)
        Pn = pidx.shape[2]
        vf = valid.float()
        vp = vf.view(B, T, 1)
        obs = map_r(self.obs, lambda o: take(o, midx).float() * vp.view(B, T, 1, *([1] * (o.dim() - 3))))
        pol = take(self.policy, midx) * vp.unsqueeze(-1)
        amask = torch.where(valid.view(B, T, 1, 1), take(self.amask, midx), torch.full_like(pol, 1e32))
        act = take(self.action, midx) * valid.long().view(B, T, 1)
        oc = torch.gather(self.outcome[slots], 1, pidx[:, 0]).view(B, 1, Pn, 1)
        val = torch.where(valid.view(B, T, 1, 1), take(self.value).unsqueeze(-1), oc.expand(B, T, Pn, 1))
        rew = take(self.reward) * vp
        ret = take(self.ret) * vp
        tm = take(self.tmask).float() * vp
        om = take(self.omask).float() * vp
        progress = torch.where(valid, t.float() / length.float(), torch.ones_like(vf))
        return {
            'observation': obs,
            'policy': pol.contiguous(),
            'value': val.contiguous(),
            'action': act.unsqueeze(-1).contiguous(),
            'outcome': oc.contiguous(),
            'reward': rew.unsqueeze(-1).contiguous(),
            'return': ret.unsqueeze(-1).contiguous(),
            'episode_mask': vf.view(B, T, 1, 1).contiguous(),
            'turn_mask': tm.unsqueeze(-1).contiguous(),
            'observation_mask': om.unsqueeze(-1).contiguous(),
            'action_mask': amask.contiguous(),
            'progress': progress.unsqueeze(-1).contiguous(),
        }

    def sample(self, B, T, generator=None):
        """B windows; solo replays: one uniformly chosen player per window (train.py:55-56)."""
        slots, start = self.sample_windows(B, T, generator)
        players = torch.randint(self.P, (B,), device=self.device, generator=generator) if self.solo else None
        return self.gather(slots, start, T, players)


def player_episodes_to_wire(ep, compress_steps=4):
    """Per-player device episodes -> the reference episode format (generation.py:29-86): a player's observation
    and value where it inferred, its policy / action mask / action where it moved, None elsewhere."""
    import bz2
    import pickle
    cpu = map_r(ep, lambda v: v.cpu().numpy())
    P = cpu['tmask'].shape[2]
    has_reward = bool((cpu['reward'] != 0).any())
    out = []
    for e in range(cpu['length'].shape[0]):
        L = int(cpu['length'][e])
        moments = []
        for t in range(L):
            m = {k: {p: None for p in range(P)} for k in ('observation', 'policy', 'action_mask', 'action',
                                                          'value', 'reward', 'return')}
            for p in range(P):
                if cpu['omask'][e, t, p]:
                    m['observation'][p] = map_r(cpu['observation'], lambda o: o[e, t, p].astype(np.float32))
                    m['value'][p] = np.array([cpu['value'][e, t, p]], dtype=np.float32)
                if cpu['tmask'][e, t, p]:
                    m['policy'][p] = cpu['policy'][e, t, p].astype(np.float32)
                    m['action_mask'][p] = cpu['action_mask'][e, t, p].astype(np.float32)
                    m['action'][p] = int(cpu['action'][e, t, p])
                if has_reward:
                    m['reward'][p] = float(cpu['reward'][e, t, p])
                m['return'][p] = float(cpu['return'][e, t, p])
            m['turn'] = [p for p in range(P) if cpu['tmask'][e, t, p]]
            moments.append(m)
        out.append({'args': {}, 'steps': L, 'outcome': {p: float(cpu['outcome'][e, p]) for p in range(P)},
                    'moment': [bz2.compress(pickle.dumps(moments[i:i + compress_steps]))
                               for i in range(0, L, compress_steps)]})
    return out


def episodes_to_wire(ep, compress_steps=4):
    """Device episodes -> the reference episode format (generation.py:79-86), for parity checks."""
    import bz2
    import pickle
    cpu = map_r(ep, lambda v: v.cpu().numpy())
    has_reward = bool((cpu['reward'] != 0).any())
    out = []
    for e in range(cpu['length'].shape[0]):
        L = int(cpu['length'][e])
        moments = []
        for t in range(L):
            p = int(cpu['turn'][e, t])
            m = {k: {0: None, 1: None} for k in ('observation', 'policy', 'action_mask', 'action', 'value',
                                                    'reward', 'return')}
            m['observation'][p] = map_r(cpu['observation'], lambda o: o[e, t].astype(np.float32))
            m['policy'][p] = cpu['policy'][e, t].astype(np.float32)
            m['action_mask'][p] = cpu['action_mask'][e, t].astype(np.float32)
            m['action'][p] = int(cpu['action'][e, t])
            m['value'][p] = np.array([cpu['value'][e, t]], dtype=np.float32)
            for q in (0, 1):
                if has_reward:
                    m['reward'][q] = float(cpu['reward'][e, t, q])
                m['return'][q] = float(cpu['return'][e, t, q])
            m['turn'] = [p]
            moments.append(m)
        out.append({'args': {}, 'steps': L, 'outcome': {0: float(cpu['outcome'][e, 0]), 1: float(cpu['outcome'][e, 1])},
                    'moment': [bz2.compress(pickle.dumps(moments[i:i + compress_steps]))
                               for i in range(0, L, compress_steps)]})
    return out
