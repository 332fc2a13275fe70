"""A test-local env plugin that has no batched twin in handyrl_amd: the kind of module a user names in
config.yaml by its import path (``env: tests.plugin_env``).

Simultaneous rock-paper-scissors over five rounds: both players move every turn (``turns()`` = both), the
round's winner gets an immediate reward of +1 and the loser -1 (``reward()``), the outcome is the sign of the
reward difference.  The net is recurrent (``init_hidden``, a GRU cell) so the host generator's per-(game,
player) state and the learner's recurrent unroll are exercised by a plugin the package has never seen.
"""

import random

import numpy as np
import torch
import torch.nn as nn

from handyrl_amd.environment import BaseEnvironment

ROUNDS = 5


class RecurrentNet(nn.Module):
    def __init__(self, hidden=16):
        super().__init__()
        self.hidden = hidden
        self.inp = nn.Linear(8, hidden)
        self.cell = nn.GRUCell(hidden, hidden)
        self.head_p = nn.Linear(hidden, 3)
        self.head_v = nn.Linear(hidden, 1)

    def init_hidden(self, batch_size=None):
        shape = (self.hidden,) if batch_size is None else (*batch_size, self.hidden)
        return torch.zeros(*shape)

    def forward(self, x, hidden):
        h = self.cell(torch.relu(self.inp(x)), hidden)
        return {'policy': self.head_p(h), 'value': torch.tanh(self.head_v(h)), 'hidden': h}


class Environment(BaseEnvironment):
    def __init__(self, args=None):
        super().__init__(args)
        self.reset()

    def reset(self, args=None):
        self.round = 0
        self.last = {0: None, 1: None}
        self.score = {0: 0, 1: 0}
        self.gained = {0: 0, 1: 0}

    def players(self):
        return [0, 1]

    def turns(self):
        return [0, 1]

    def terminal(self):
        return self.round >= ROUNDS

    def legal_actions(self, player=None):
        # a player who won the last round may not repeat its move
        last = self.last[player]
        return [a for a in range(3) if not (last is not None and self.gained[player] > 0 and a == last)]

    def action_length(self):
        return 3

    def step(self, actions):
        a, b = actions[0], actions[1]
        win = (a - b) % 3          # 1: player 0 wins, 2: player 1 wins
        self.gained = {0: 1 if win == 1 else (-1 if win == 2 else 0), 1: 1 if win == 2 else (-1 if win == 1 else 0)}
        for p in (0, 1):
            self.score[p] += self.gained[p]
        self.last = {0: a, 1: b}
        self.round += 1

    def reward(self):
        return dict(self.gained)

    def outcome(self):
        d = np.sign(self.score[0] - self.score[1])
        return {0: float(d), 1: float(-d)}

    def observation(self, player=None):
        o = np.zeros(8, dtype=np.float32)
        for k, p in enumerate((player, 1 - player)):
            if self.last[p] is not None:
                o[3 * k + self.last[p]] = 1
        o[6] = self.round / ROUNDS
        o[7] = player
        return o

    def net(self):
        return RecurrentNet


if __name__ == '__main__':
    e = Environment()
    while not e.terminal():
        e.step({p: random.choice(e.legal_actions(p)) for p in e.turns()})
    print(e.outcome())
