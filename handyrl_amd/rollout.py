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

Scope: turn-based two-player training without opponent observation
(turn_based_training=True, observation=False), the TicTacToe configuration.
"""

import contextlib

import numpy as np
import torch

from .util import map_r, bimap_r

__all__ = ['TicTacToeBatch', 'DeviceGenerator', 'DeviceReplay', 'episodes_to_wire']


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
    """

    def __init__(self, env_batch, net, gamma=0.8, check_every=16, graph=None):
        self.env = env_batch
        self.net = net
        self.gamma = gamma
        self.check_every = check_every
        self.graph = graph
        self._st = None

    def _use_graph(self):
        dev = torch.device(self.env.device)
        if self.graph is None:
            return dev.type == 'cuda' and getattr(self.env, 'ALTERNATING', False)
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
        for k in ('policy', 'action', 'value', 'turn', 'reward', 'ret'):
            st[k].zero_()
        st['amask'].fill_(1e32)
        if st['hidden'] is not None:
            map_r(st['hidden'], lambda h: h.zero_())
        if draw:
            torch.rand(st['U'].shape, out=st['U'], generator=generator, device=st['U'].device)
            st['U'].clamp_(1e-20, 1.0)
        st['t'].zero_()

    def _ply(self, st, mover):
        """One ply for every game at ply index st['t'] (a device scalar, advanced here); ``mover``: the
        player index every live game moves with (ALTERNATING envs), or None."""
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
    def generate(self, generator=None):
        alternating = getattr(self.env, 'ALTERNATING', False)
        st = self._state()
        was_training = self.net.training
        self.net.eval()
        # per-call weight preparation (GeisterNet); its own stacked state is advanced in place by the net
        session = getattr(self.net, 'inference_session', None)
        with session(inplace_state=st['pmajor']) if session is not None else contextlib.nullcontext():
            out = self._generate(st, generator, alternating)
        self.net.train(was_training)
        return out

    def _generate(self, st, generator, alternating):
        env = self.env
        Tm, P = env.MAX_PLIES, env.P
        self._reset(st, generator)
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
                       ('turn', 'turn'), ('return', 'ret')):
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
