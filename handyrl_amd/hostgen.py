"""Host-env batched self-play and a moment replay: ANY plugin env trains (north star: existing envs drop in).

The reference's worker plays one game per process through the Environment
plugin API with one batch-1 inference per observing player per ply
(generation.py:20-88, model.py:43-53).  ``HostBatchGenerator`` keeps the
same per-game semantics for every ``BaseEnvironment`` -- ``turns()`` (several
movers for simultaneous games), ``observation(p)`` for the turn players and,
with ``args['observation']``, for every player; a recurrent state per game and
player advanced for every player that observed; ``legal_actions``; masking by
1e32; ``step(actions)``; ``reward()`` read after the step; discounted returns
in Python floats -- but plays E games at once on the host and runs ONE
batched forward of the network on the GPU per ply for all of their requests:

* the games are split in ``groups`` (default 2) that take turns: while the GPU
  runs one group's forward, the host steps the other group's envs, and the
  forward's outputs come back through pinned buffers behind an event, so the
  host never waits for a forward it does not need yet;
* finished games restart at once (a slot never idles while a long game runs),
  until ``generate(n)`` has its n episodes;
* ``sampler='gumbel'`` (default) samples every turn player of a ply at once by
  Gumbel-max over the masked logits (numpy, seeded): the distribution of the
  reference's ``random.choices(legal, weights=softmax(p[legal]))``;
  ``sampler='reference'`` calls exactly that per turn player, with every game
  owning a Python ``random`` state that is swapped in around its sampling and
  its ``env.step`` (ParallelTicTacToe's step draws from ``random``), so game k
  reproduces the reference's ``random.seed(seed_k); Generator.generate``
  move for move (tests/test_hostgen.py against reference-generated episodes).

An episode is the reference's episode (generation.py:79-88) with the moment
list not yet compressed: {'args', 'steps', 'outcome', 'moments'}; ``to_wire``
compresses it into bz2(pickle) blocks for the reference's make_batch.

``MomentReplay`` stores episodes in HBM as a ring of moments (any episode
length, every (moment, player) slot of the reference's moment dicts) and
gathers B windows straight into the make_batch layout (train.py:33-133) for
all four training modes -- turn-based or solo, with or without opponent
observation -- with the reference Batcher's recency-weighted episode choice
and uniform window start (train.py:284-293).
"""

import bz2
import contextlib
import pickle
import random
import time

import numpy as np
import torch

from .util import map_r, bimap_r

__all__ = ['HostBatchGenerator', 'MomentReplay', 'to_wire', 'softmax']


def softmax(x):
    """handyrl/util.py:61-63 (float32 in, float32 out)."""
    x = np.exp(x - np.max(x, axis=-1))
    return x / x.sum(axis=-1)


def _stack(template, items):
    """Stack nested observations leaf by leaf along a new axis 0 (numpy)."""
    if isinstance(template, dict):
        return {k: _stack(v, [it[k] for it in items]) for k, v in template.items()}
    if isinstance(template, (list, tuple)):
        return type(template)(_stack(v, [it[i] for it in items]) for i, v in enumerate(template))
    return np.stack([np.asarray(it) for it in items])


def to_wire(ep, compress_steps=4):
    """The reference's episode record (generation.py:79-86): moments in bz2(pickle) blocks."""
    ms = ep['moments']
    return {'args': ep.get('args', {}), 'steps': ep['steps'], 'outcome': ep['outcome'],
            'moment': [bz2.compress(pickle.dumps(ms[i:i + compress_steps])) for i in range(0, len(ms), compress_steps)]}


class _Slot:
    __slots__ = ('env', 'moments', 'rng', 'players', 'turns', 'requests', 'game')

    def __init__(self, env):
        self.env = env
        self.moments = None
        self.rng = None
        self.players = None
        self.turns = None
        self.requests = []
        self.game = -1


class _Group:
    """Slots that share one forward per ply; ``pending`` holds the launched forward's host buffers."""

    def __init__(self, slots):
        self.slots = slots
        self.pending = None
        self.staging = None


class HostBatchGenerator:
    """E plugin-env games on the host, one batched network forward per ply (generation.py:20-88).

    ``env_factory()`` returns a fresh ``BaseEnvironment`` (e.g. ``lambda: make_env(env_args)``); ``net`` is the
    env's network (any device); ``args`` needs 'observation' and 'gamma'.  ``seed`` seeds the Gumbel sampler;
    in reference mode game k uses ``game_seeds[k]`` (default seed + k) as its ``random.seed``.
    """

    def __init__(self, env_factory, net, args, E=64, sampler='gumbel', seed=0, game_seeds=None, groups=None,
                 max_forward=None):
        if sampler not in ('gumbel', 'reference'):
            raise ValueError('sampler must be gumbel or reference, not %r' % (sampler,))
        self.env_factory = env_factory
        self.net = net
        self.args = args
        self.E = int(E)
        self.sampler = sampler
        self.seed = seed
        self.game_seeds = game_seeds
        self.np_rng = np.random.default_rng(seed)
        self.slots = [_Slot(env_factory()) for _ in range(self.E)]
        self.players = list(self.slots[0].env.players())
        self.pidx = {p: i for i, p in enumerate(self.players)}
        self.device = next(iter(net.parameters())).device
        ng = groups or (2 if self.device.type == 'cuda' and self.E >= 2 else 1)
        ng = max(1, min(ng, self.E))
        self.groups = [_Group(list(range(g, self.E, ng))) for g in range(ng)]
        self.max_forward = max_forward
        # a net with its own numpy inference (model.py:45-46) is called per request, batch 1
        self.own_inference = hasattr(net, 'inference')
        self.hidden = None
        self.own_hidden = None
        self._hidden_ready = False
        self.games_started = 0
        self.failed = 0
        # seconds per phase of the last generate(): 'requests' (env observations, the plugin's own cost), 'launch'
        # (stacking into pinned buffers, H2D, the forward's launch), 'wait' (host blocked on a forward), 'advance'
        # (masks, sampling, env.step / reward, moment records)
        self.timing = {}

    # -- recurrent state: one per (game slot, player), on the net's device -------------------------------
    def _init_hidden(self):
        self._hidden_ready = True
        if self.own_inference:
            self.own_hidden = [[None] * len(self.players) for _ in range(self.E)]
            return
        if not hasattr(self.net, 'init_hidden'):
            return
        h = self.net.init_hidden([self.E, len(self.players)])
        if h is None:
            return
        self.hidden = map_r(h, lambda x: torch.as_tensor(x).to(self.device).contiguous())
        self.hidden_init = map_r(self.hidden, lambda x: x.clone())   # a game's states start from these

    def _reset_hidden(self, s):
        """generation.py:23-25: every player's state starts from init_hidden()."""
        if self.own_hidden is not None:
            init = getattr(self.net, 'init_hidden', None)
            self.own_hidden[s] = [init() if init is not None else None for _ in self.players]
        if self.hidden is not None:
            bimap_r(self.hidden, self.hidden_init, lambda h, h0: h[s].copy_(h0[s]))

    # -- game lifecycle -------------------------------------------------------------------------------
    def _start(self, slot_index, n_target):
        """Start the next game in a slot; False when no game is left to start."""
        slot = self.slots[slot_index]
        while self.games_started < n_target:
            k = self.games_started
            self.games_started += 1
            slot.game = k
            if self.sampler == 'reference':
                seed = self.game_seeds[k] if self.game_seeds is not None else self.seed + k
                slot.rng = random.Random(seed).getstate()
                random.setstate(slot.rng)
            err = slot.env.reset()
            if self.sampler == 'reference':
                slot.rng = random.getstate()
            self._reset_hidden(slot_index)
            slot.moments = []
            if err or slot.env.terminal():   # generation.py:27-29, 70-71: None episode
                self.failed += 1
                continue
            return True
        slot.moments = None
        return False

    def _requests(self, s):
        """The slot's inference requests for this ply (generation.py:35-40)."""
        slot = self.slots[s]
        env = slot.env
        slot.turns = env.turns()
        observe = self.args['observation']
        slot.requests = [(p, env.observation(p)) for p in self.players if p in slot.turns or observe]
        return slot.requests

    def _finish(self, s, out):
        slot = self.slots[s]
        moments = slot.moments
        gamma = self.args['gamma']
        for p in self.players:                      # generation.py:73-77
            ret = 0
            for i in range(len(moments) - 1, -1, -1):
                m = moments[i]
                ret = (m['reward'][p] or 0) + gamma * ret
                m['return'][p] = ret
        out[slot.game] = {'args': {'player': self.players}, 'steps': len(moments),
                          'outcome': slot.env.outcome(), 'moments': moments}

    # -- the forward ----------------------------------------------------------------------------------
    def _staging(self, group, obs0, n):
        """The group's pinned host buffers (observation leaves, row indices, outputs), reused every ply: a
        buffer is rewritten only after the group's previous forward has been waited for."""
        st = group.staging
        if st is None or st['rows'] < n:
            rows = max(n, len(group.slots) * len(self.players))
            st = group.staging = {
                'rows': rows,
                'obs': map_r(obs0, lambda a: torch.empty((rows,) + np.shape(a), dtype=torch.float32,
                                                        pin_memory=True)),
                'idx': torch.empty(2, rows, dtype=torch.long, pin_memory=True),
                'out': {}}
        return st

    def _launch(self, group):
        """Gather the group's requests and launch their forward; the outputs land in host buffers."""
        rows, obs = [], []
        t0 = time.perf_counter()
        for s in group.slots:
            if self.slots[s].moments is None:
                continue
            for p, o in self._requests(s):
                rows.append((s, self.pidx[p]))
                obs.append(o)
        t1 = time.perf_counter()
        self.timing['requests'] = self.timing.get('requests', 0.0) + (t1 - t0)
        try:
            self._launch_rows(group, rows, obs)
        finally:
            self.timing['launch'] = self.timing.get('launch', 0.0) + (time.perf_counter() - t1)

    def _launch_rows(self, group, rows, obs):
        if not rows:
            group.pending = None
            return
        if self.own_inference:              # model.py:45-46: the net's own numpy inference, batch 1
            outs = []
            for (s, pi), o in zip(rows, obs):
                o_ = self.net.inference(o, self.own_hidden[s][pi])
                self.own_hidden[s][pi] = o_.get('hidden', None)
                outs.append(o_)
            group.pending = ('own', rows, outs)
            return
        n = len(rows)
        cuda = self.device.type == 'cuda'
        if cuda:
            st = self._staging(group, obs[0], n)
            bimap_r(st['obs'], _stack(obs[0], obs), lambda dst, src: dst[:n].numpy().__setitem__(Ellipsis, src))
            idx = st['idx'][:, :n]
            idx.numpy()[...] = np.asarray(rows, dtype=np.int64).T
            x = map_r(st['obs'], lambda a: a[:n].to(self.device, non_blocking=True))
            idx = idx.to(self.device, non_blocking=True)
            gi, pi = idx[0], idx[1]
        else:
            x = map_r(_stack(obs[0], obs), lambda a: torch.from_numpy(np.ascontiguousarray(a, dtype=np.float32)))
            gi = torch.tensor([r[0] for r in rows])
            pi = torch.tensor([r[1] for r in rows])
        h = None
        if self.hidden is not None:
            h = map_r(self.hidden, lambda t: t[gi, pi])
        out = self.net(x, h)
        if self.hidden is not None:
            nh = out.get('hidden')
            if nh is None:
                raise ValueError('a net with init_hidden must return its new state as outputs["hidden"]')
            bimap_r(self.hidden, nh, lambda dst, src: dst.index_put_((gi, pi), src))
        vals = [out['policy'].float()]
        if out.get('value') is not None:
            vals.append(out['value'].float().reshape(n, -1))
        if cuda:
            host = []
            for k, v in enumerate(vals):
                buf = st['out'].get(k)
                if buf is None or buf.shape[0] < st['rows'] or buf.shape[1:] != v.shape[1:]:
                    buf = st['out'][k] = torch.empty((st['rows'],) + tuple(v.shape[1:]), pin_memory=True)
                buf[:n].copy_(v, non_blocking=True)
                host.append(buf[:n])
            ev = torch.cuda.Event()
            ev.record()
        else:
            host, ev = [v.detach() for v in vals], None
        group.pending = ('batch', rows, host, ev)

    def _outputs(self, group):
        """(rows, policy (N, A) float32, value (N, K) or None) of the group's launched forward."""
        kind = group.pending[0]
        if kind == 'own':
            _, rows, outs = group.pending
            pol = np.stack([np.asarray(o['policy'], dtype=np.float32) for o in outs])
            val = None
            if outs and outs[0].get('value') is not None:
                val = np.stack([np.asarray(o['value'], dtype=np.float32).reshape(-1) for o in outs])
            return rows, pol, val
        _, rows, host, ev = group.pending
        if ev is not None:
            t0 = time.perf_counter()
            ev.synchronize()
            self.timing['wait'] = self.timing.get('wait', 0.0) + (time.perf_counter() - t0)
        pol = host[0].numpy()
        val = host[1].numpy() if len(host) > 1 else None
        return rows, pol, val

    # -- one ply of a group on the host ----------------------------------------------------------------
    def _advance(self, group, n_target, out):
        rows, pol, val = self._outputs(group)
        group.pending = None
        # per slot: its rows in request (= players) order
        by_slot = {}
        for i, (s, pi) in enumerate(rows):
            by_slot.setdefault(s, []).append(i)
        moment_keys = ('observation', 'policy', 'action_mask', 'action', 'value', 'reward', 'return')
        reference = self.sampler == 'reference'
        plan = []
        turn_rows = []
        for s, idx in by_slot.items():
            slot = self.slots[s]
            env = slot.env
            moment = {key: {p: None for p in self.players} for key in moment_keys}
            for i, (p, o) in zip(idx, slot.requests):
                moment['observation'][p] = o
                moment['value'][p] = None if val is None else val[i].copy()
                if p in slot.turns:
                    legal = env.legal_actions(p)
                    p_ = pol[i]
                    amask = np.ones_like(p_) * 1e32
                    amask[legal] = 0
                    masked = p_ - amask
                    moment['policy'][p] = masked
                    moment['action_mask'][p] = amask
                    turn_rows.append((s, p, legal, masked))
            plan.append((s, moment))
        if not reference and turn_rows:
            # Gumbel-max over every turn player of the ply at once: argmax(p - log(-log u)) is a draw from
            # softmax over the legal actions (illegal ones sit at -1e32)
            logits = np.stack([r[3] for r in turn_rows])
            u = self.np_rng.random(logits.shape)
            np.clip(u, 1e-20, 1.0, out=u)
            acts = np.argmax(logits - np.log(-np.log(u)), axis=-1)
            chosen = {(r[0], r[1]): int(a) for r, a in zip(turn_rows, acts)}
        for s, moment in plan:
            slot = self.slots[s]
            env = slot.env
            if reference:
                random.setstate(slot.rng)
            for p in self.players:
                if moment['policy'][p] is None:
                    continue
                if reference:   # generation.py:49-53
                    legal = env.legal_actions(p)
                    pm = moment['policy'][p]
                    moment['action'][p] = random.choices(legal, weights=softmax(pm[legal]))[0]
                else:
                    moment['action'][p] = chosen[(s, p)]
            err = env.step(moment['action'])
            if reference:
                slot.rng = random.getstate()
            if err:                                  # generation.py:59-61: the game is dropped
                self.failed += 1
                self._start(s, n_target)
                continue
            reward = env.reward()                    # generation.py:63-65: after the step
            for p in self.players:
                moment['reward'][p] = reward.get(p, None)
            moment['turn'] = slot.turns
            slot.moments.append(moment)
            if env.terminal():
                self._finish(s, out)
                self._start(s, n_target)

    @torch.no_grad()
    def generate(self, n):
        """Play n games (the E slots restart finished games); returns the n episodes in game order
        (fewer if some failed: generation.py's None episodes are dropped)."""
        if not self._hidden_ready:
            self._init_hidden()
        was_training = self.net.training
        self.net.eval()                              # model.py:48
        saved = random.getstate() if self.sampler == 'reference' else None
        self.games_started, self.failed = 0, 0
        self.timing = {}
        out = {}
        # a net with per-call inference preparation (GeisterNet: stacked DRC weights, packed conv fragments,
        # BatchNorm coefficients) prepares once for the whole call instead of once per forward
        session = getattr(self.net, 'inference_session', None)
        ctx = session() if session is not None and self.device.type == 'cuda' else contextlib.nullcontext()
        try:
            with ctx:   # entered and exited as a pair; an exception in the body reaches __exit__ and propagates
                self._run(n, out)
        finally:
            if saved is not None:
                random.setstate(saved)
            self.net.train(was_training)
        return [out[k] for k in sorted(out)]

    def _run(self, n, out):
        """generate()'s body inside the net's inference session: start every slot, then advance and relaunch the
        slot groups until none has a forward pending."""
        for s in range(self.E):
            self._start(s, n)
        for g in self.groups:
            self._launch(g)
        while any(g.pending is not None for g in self.groups):
            for g in self.groups:
                if g.pending is None:
                    continue
                t0 = time.perf_counter()
                w0 = self.timing.get('wait', 0.0)
                self._advance(g, n, out)
                self.timing['advance'] = self.timing.get('advance', 0.0) + (
                    time.perf_counter() - t0 - (self.timing.get('wait', 0.0) - w0))
                self._launch(g)


class MomentReplay:
    """Episodes in HBM as a ring of moments; windows gathered into the make_batch layout.

    Every (moment, player) slot of the reference's moment dicts is kept: observation (zeros when None),
    policy (zeros), action mask (1e32), action (0), value (0), reward (0), return, and the turn / observation
    flags (``policy is not None`` / ``value is not None``, train.py:86-87), plus the moment's first turn
    player (``m['turn'][0]``, the slot turn-based training without observation reads, train.py:64-68).
    ``sample`` draws windows as Batcher.select_episode (train.py:284-293) and gathers them for
    ``args['turn_based_training']`` / ``args['observation']`` as make_batch lays them out (train.py:57-133).
    Storage grows by doubling as episodes arrive, up to ``maximum_episodes`` episodes.
    """

    def __init__(self, args, device, maximum_episodes=None, capacity=1 << 14):
        self.args = args
        self.device = torch.device(device)
        self.maximum_episodes = int(maximum_episodes or args['maximum_episodes'])
        self.cap = int(capacity)                  # moments
        self.head = 0                             # absolute index of the next moment
        self.ep_cap = self.maximum_episodes
        self.ep_start = np.zeros(self.ep_cap, dtype=np.int64)
        self.ep_len = np.zeros(self.ep_cap, dtype=np.int64)
        self.ep_ptr = 0                           # next episode slot
        self.count = 0                            # stored episodes
        self.store = None
        self.players = None
        self._dev = None

    # -- layout ----------------------------------------------------------------------------------------
    def _alloc(self, template, A, P, n):
        dev = self.device
        st = {'obs': map_r(template, lambda a: torch.zeros(n, P, *np.shape(a), dtype=torch.float32, device=dev)),
              'policy': torch.zeros(n, P, A, device=dev),
              'amask': torch.full((n, P, A), 1e32, device=dev),
              'action': torch.zeros(n, P, dtype=torch.long, device=dev),
              'value': torch.zeros(n, P, device=dev),
              'reward': torch.zeros(n, P, device=dev),
              'ret': torch.zeros(n, P, device=dev),
              'tmask': torch.zeros(n, P, device=dev),
              'omask': torch.zeros(n, P, device=dev),
              'first': torch.zeros(n, dtype=torch.long, device=dev)}
        return st

    def _grow(self, need):
        """Double the moment ring until `need` moments fit; live moments keep their absolute index."""
        new_cap = self.cap
        while new_cap < need:
            new_cap *= 2
        lo = self.head - self._live_moments()
        new = self._alloc(self.template, self.A, self.P, new_cap)
        if self.head > lo:
            absi = torch.arange(lo, self.head, device=self.device)
            src, dst = absi % self.cap, absi % new_cap
            bimap_r(new, self.store, lambda d, s: d.index_copy_(0, dst, s.index_select(0, src)))
        self.store, self.cap = new, new_cap

    def _live_moments(self):
        if self.count == 0:
            return 0
        oldest = (self.ep_ptr - self.count) % self.ep_cap
        return self.head - int(self.ep_start[oldest])

    def __len__(self):
        return self.count

    # -- adding episodes -------------------------------------------------------------------------------
    def add(self, episodes):
        """Store HostBatchGenerator episodes (moment dicts, generation.py:31-77)."""
        episodes = [ep for ep in episodes if ep is not None and ep['steps'] > 0]
        if not episodes:
            return
        if self.store is None:
            m0 = episodes[0]['moments'][0]
            self.players = list(m0['observation'].keys())
            first = m0['turn'][0]
            self.template = m0['observation'][first]
            self.A = int(np.shape(m0['policy'][first])[-1])
            self.P = len(self.players)
            self.store = self._alloc(self.template, self.A, self.P, self.cap)
        P, A = self.P, self.A
        pidx = {p: i for i, p in enumerate(self.players)}
        n = sum(ep['steps'] for ep in episodes)
        # host staging of the new moments, the reference's None replacements applied (train.py:50-87)
        obs = map_r(self.template, lambda a: np.zeros((n, P) + np.shape(a), dtype=np.float32))
        pol = np.zeros((n, P, A), dtype=np.float32)
        amask = np.full((n, P, A), 1e32, dtype=np.float32)
        act = np.zeros((n, P), dtype=np.int64)
        val = np.zeros((n, P), dtype=np.float32)
        rew = np.zeros((n, P), dtype=np.float32)
        ret = np.zeros((n, P), dtype=np.float32)
        tmask = np.zeros((n, P), dtype=np.float32)
        omask = np.zeros((n, P), dtype=np.float32)
        first = np.zeros(n, dtype=np.int64)
        row = 0
        outcomes = np.zeros((len(episodes), P), dtype=np.float32)
        for e, ep in enumerate(episodes):
            for p in self.players:
                outcomes[e, pidx[p]] = ep['outcome'][p]
            for m in ep['moments']:
                first[row] = pidx[m['turn'][0]]
                for p, j in pidx.items():
                    o = m['observation'][p]
                    if o is not None:
                        bimap_r(obs, o, lambda dst, src: dst[row, j].__setitem__(Ellipsis, src))
                    if m['policy'][p] is not None:
                        pol[row, j] = m['policy'][p]
                        tmask[row, j] = 1
                    if m['action_mask'][p] is not None:
                        amask[row, j] = m['action_mask'][p]
                    if m['action'][p] is not None:
                        act[row, j] = m['action'][p]
                    if m['value'][p] is not None:
                        v = np.asarray(m['value'][p], dtype=np.float32).reshape(-1)
                        if v.size != 1:
                            # make_batch pads values with the (P, 1) outcome (train.py:94-96), so the reference
                            # learner takes one value per player; a wider head would be silently truncated here
                            raise ValueError('MomentReplay: a moment value has %d elements; the learner takes one '
                                             'value per player' % v.size)
                        val[row, j] = v[0]
                        omask[row, j] = 1
                    if m['reward'][p] is not None:
                        rew[row, j] = m['reward'][p]
                    ret[row, j] = m['return'][p]
                row += 1
        staged = {'obs': obs, 'policy': pol, 'amask': amask, 'action': act, 'value': val, 'reward': rew,
                  'ret': ret, 'tmask': tmask, 'omask': omask, 'first': first}
        # make room: grow while fewer than maximum_episodes are stored, else evict the oldest
        if self._live_moments() + n > self.cap and self.count + len(episodes) <= self.maximum_episodes:
            self._grow(self._live_moments() + n)
        if n > self.cap:
            self._grow(n)
        absi = torch.arange(self.head, self.head + n, device=self.device) % self.cap
        bimap_r(self.store, staged, lambda d, s: d.index_copy_(0, absi, torch.from_numpy(s).to(self.device)))
        start = self.head
        for e, ep in enumerate(episodes):
            if self.count == self.ep_cap:
                self.count -= 1                   # the ring's oldest episode is overwritten
            self.ep_start[self.ep_ptr] = start
            self.ep_len[self.ep_ptr] = ep['steps']
            self._outcome_host()[self.ep_ptr] = outcomes[e]
            start += ep['steps']
            self.ep_ptr = (self.ep_ptr + 1) % self.ep_cap
            self.count += 1
        self.head += n
        # episodes whose moments were overwritten are gone
        while self.count and int(self.ep_start[(self.ep_ptr - self.count) % self.ep_cap]) < self.head - self.cap:
            self.count -= 1
        self._dev = None

    def _outcome_host(self):
        if not hasattr(self, '_oc'):
            self._oc = np.zeros((self.ep_cap, self.P), dtype=np.float32)
        return self._oc

    def _device_tables(self):
        if self._dev is None:
            order = (self.ep_ptr - self.count + np.arange(self.count)) % self.ep_cap      # oldest first
            self._dev = (torch.from_numpy(self.ep_start[order]).to(self.device),
                         torch.from_numpy(self.ep_len[order]).to(self.device),
                         torch.from_numpy(self._outcome_host()[order]).to(self.device))
        return self._dev

    # -- windows ---------------------------------------------------------------------------------------
    def sample_windows(self, B, T, generator=None):
        """(episode index in age order, window start) of B windows (train.py:284-293): episode i of the n
        newest accepted with probability 1 - (n-1-i)/maximum_episodes, start uniform over the
        1 + max(0, steps - T) candidates."""
        if self.count == 0:
            raise ValueError('MomentReplay.sample: no episodes stored')
        _, length, _ = self._device_tables()
        n = min(self.count, self.maximum_episodes)
        i = torch.arange(n, device=self.device, dtype=torch.float64)
        w = 1.0 - (n - 1 - i) / self.maximum_episodes
        pick = torch.multinomial(w.float(), B, replacement=True, generator=generator) + (self.count - n)
        steps = length[pick]
        cand = 1 + torch.clamp(steps - T, min=0)
        u = torch.rand(B, device=self.device, generator=generator)
        start = torch.minimum((u * cand).long(), cand - 1)
        return pick, start

    def gather(self, pick, start, T, solo_player=None):
        """make_batch layout of the windows [start, start+T) of episodes `pick` (age order).  Solo training
        (turn_based_training False) trains `solo_player` (B,) per window (train.py:57-58)."""
        st, args = self.store, self.args
        ep_start, ep_len, ep_oc = self._device_tables()
        B, dev = pick.shape[0], self.device
        t = start.view(-1, 1) + torch.arange(T, device=dev).view(1, -1)           # (B, T)
        length = ep_len[pick].view(-1, 1)
        valid = t < length
        m = (ep_start[pick].view(-1, 1) + torch.minimum(t, length - 1)) % self.cap
        vf = valid.float()
        oc = ep_oc[pick]                                                           # (B, P)
        if not args['turn_based_training']:
            players = solo_player.view(B, 1)                                         # (B, 1)
            oc = oc.gather(1, players)
        else:
            players = torch.arange(self.P, device=dev).view(1, -1).expand(B, -1)   # (B, P)
        Pv = players.shape[1]
        mm = m.unsqueeze(-1).expand(B, T, Pv)
        pp = players.view(B, 1, Pv).expand(B, T, Pv)
        if args['turn_based_training'] and not args['observation']:
            ps = st['first'][m].unsqueeze(-1)                                      # (B, T, 1)
            ms = m.unsqueeze(-1)
        else:
            ps, ms = pp, mm

        def pad(x, fill):
            live = valid.view(B, T, *([1] * (x.dim() - 2)))
            return torch.where(live, x, torch.full_like(x, fill))
        obs = map_r(st['obs'], lambda o: pad(o[ms, ps], 0))
        pol = pad(st['policy'][ms, ps], 0)
        amask = pad(st['amask'][ms, ps], 1e32)
        act = pad(st['action'][ms, ps], 0).unsqueeze(-1)

        def per_player(key):
            return pad(st[key][mm, pp], 0).unsqueeze(-1)                           # (B, T, Pv, 1)
        val = torch.where(valid.view(B, T, 1, 1), st['value'][mm, pp].unsqueeze(-1),
                          oc.view(B, 1, Pv, 1).expand(B, T, Pv, 1))
        progress = torch.where(valid, t.float() / length.float(), torch.ones_like(vf))
        return {
            'observation': obs,
            'policy': pol.contiguous(),
            'value': val.contiguous(),
            'action': act.contiguous(),
            'outcome': oc.view(B, 1, Pv, 1).contiguous(),
            'reward': per_player('reward').contiguous(),
            'return': per_player('ret').contiguous(),
            'episode_mask': vf.view(B, T, 1, 1).contiguous(),
            'turn_mask': per_player('tmask').contiguous(),
            'observation_mask': per_player('omask').contiguous(),
            'action_mask': amask.contiguous(),
            'progress': progress.unsqueeze(-1).contiguous(),
        }

    def sample(self, B, T, generator=None):
        pick, start = self.sample_windows(B, T, generator)
        solo = None
        if not self.args['turn_based_training']:
            solo = torch.randint(self.P, (B,), device=self.device, generator=generator)
        return self.gather(pick, start, T, solo)
