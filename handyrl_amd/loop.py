"""Device-resident self-play training loop (generation -> replay -> learner) and evaluation.

The reference runs this loop across processes: workers generate episodes
(generation.py:20-88), the learner's server feeds them to the trainer's
episode deque (train.py:480-503), batchers cut windows (train.py:261-309) and
the trainer steps (train.py:357-401); every ``update_episodes`` episodes the
model is published to the workers (train.py:516-542).  Here the same cycle
stays on one GPU: ``DeviceGenerator`` plays ``games_per_round`` games with the
current weights, ``DeviceReplay`` holds the newest ``maximum_episodes``,
and ``LearnerStep`` trains on windows gathered from it.

``evaluate_vs_random`` is the batched counterpart of the reference's
evaluation against a random agent (evaluation.py:64-87, agent.py:55-110).
"""

import time

import torch

from .rollout import DeviceGenerator, DeviceReplay, TicTacToeBatch
from .trainer import LearnerStep
from .util import map_r

__all__ = ['SelfPlayTrainer', 'evaluate_vs_random']


class SelfPlayTrainer:
    """``env_cls``: a batched env (TicTacToeBatch, envs.geister.GeisterBatch); recurrent nets
    train from a zero hidden state at every window start (train.py:375)."""

    def __init__(self, net, args, device, games_per_round=4096, capacity=65536, graph=False, seed=0,
                 env_cls=TicTacToeBatch, obs_dtype=torch.uint8):
        self.args = args
        self.device = device
        self.env = env_cls(games_per_round, device)
        self.gen = DeviceGenerator(self.env, net, gamma=args['gamma'])
        self.replay = DeviceReplay(capacity, env_cls.MAX_PLIES, env_cls.OBS_SHAPE, env_cls.A, env_cls.P, device,
                                   maximum_episodes=args.get('maximum_episodes', capacity), obs_dtype=obs_dtype)
        self.learner = LearnerStep(net, args, device, graph=graph)
        self.hidden = None
        if hasattr(net, 'init_hidden'):
            self.hidden = map_r(net.init_hidden([args['batch_size'], env_cls.P]), lambda h: h.to(device))
        self.rng = torch.Generator(device=device).manual_seed(seed)
        self.episodes = 0
        self.steps = 0

    def generate(self):
        ep = self.gen.generate(generator=self.rng)
        self.replay.add(ep)
        self.episodes += ep['length'].shape[0]
        return ep

    def train_steps(self, n):
        B, T = self.args['batch_size'], self.args['forward_steps']
        for _ in range(n):
            batch = self.replay.sample(B, T, generator=self.rng)
            self.learner.step(batch, self.hidden)
            self.steps += 1

    def run(self, rounds, steps_per_round, log=None):
        t0 = time.perf_counter()
        for r in range(rounds):
            self.generate()
            self.train_steps(steps_per_round)
            if log is not None:
                sums, n = self.learner.pop_stats()
                dcnt = max(sums.get('dcnt', 1.0), 1e-9)
                log('round %d episodes %d steps %d loss %s (%.1fs)' % (
                    r, self.episodes, self.steps,
                    ' '.join('%s:%.3f' % (k, sums[k] / dcnt) for k in ('p', 'v', 'ent') if k in sums),
                    time.perf_counter() - t0))


@torch.no_grad()
def evaluate_vs_random(net, device, games=4096, seed=0):
    """Model (sampling its policy over legal moves) vs a uniform random player.

    The model plays black in the first half of the games and white in the
    second.  Returns {'win', 'draw', 'loss'} rates from the model's side.
    """
    env = TicTacToeBatch(games, device)
    g = torch.Generator(device=device).manual_seed(seed)
    model_side = (torch.arange(games, device=device) >= games // 2).long()   # 0 = black
    was = net.training
    net.eval()
    for _ in range(TicTacToeBatch.MAX_PLIES):
        active = ~env.terminal()
        player = env.turn()
        legal = env.legal()
        logits = net(env.observation(player), None)['policy']
        mine = player == model_side
        rand_logits = torch.zeros_like(logits)
        p = torch.where(mine.view(-1, 1), logits, rand_logits) - torch.where(legal, 0.0, 1e32)
        u = torch.rand(p.shape, device=device, generator=g).clamp_(1e-20, 1.0)
        a = torch.argmax(p - torch.log(-torch.log(u)), dim=-1)
        env.step(a, active)
    net.train(was)
    oc = env.outcome()[torch.arange(games, device=device), model_side]
    return {'win': float((oc > 0).float().mean()), 'draw': float((oc == 0).float().mean()),
            'loss': float((oc < 0).float().mean())}
