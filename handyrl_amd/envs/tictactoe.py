"""Tic-Tac-Toe plugin: rules + the network the learner benchmark trains.

Behaviour follows handyrl/envs/tictactoe.py (rules :72-172, net :17-69):
players [0, 1], black (player 0) moves first, observation = 3 planes
[turn-view indicator, own stones, opponent stones] of 3x3, action a = row*3+col,
outcome {+1, -1} / {0, 0}.  The network has the reference's architecture and
state_dict key names (conv, blocks.i.{conv,bn}, head_{p,v}.{conv.conv,fc}),
so reference checkpoints load into it unchanged: 29,006 parameters.
"""

import random

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from ..environment import BaseEnvironment


class ConvUnit(nn.Module):
    """kxk conv, 'same' padding; bias only when there is no BatchNorm."""

    def __init__(self, cin, cout, k, bn):
        super().__init__()
        self.conv = nn.Conv2d(cin, cout, k, padding=k // 2, bias=not bn)
        self.bn = nn.BatchNorm2d(cout) if bn else None

    def forward(self, x):
        x = self.conv(x)
        return x if self.bn is None else self.bn(x)


class BoardHead(nn.Module):
    """1x1 conv -> LeakyReLU(0.1) -> flatten -> bias-free linear."""

    LEAKY_SLOPE = 0.1   # nn.fuse_bn_relu fuses the policy/value pair into csrc/hrl_heads.hip

    def __init__(self, cin, hw, cmid, nout):
        super().__init__()
        self.flat = hw * cmid
        self.conv = ConvUnit(cin, cmid, 1, bn=False)
        self.fc = nn.Linear(self.flat, nout, bias=False)

    def forward(self, x):
        h = F.leaky_relu(self.conv(x), 0.1)
        return self.fc(h.reshape(-1, self.flat))


class SimpleConv2dModel(nn.Module):
    """3x3 conv stem + 3 conv-BN-ReLU blocks (32 filters) + policy / value heads."""

    def __init__(self, filters=32, layers=3):
        super().__init__()
        self.conv = nn.Conv2d(3, filters, 3, padding=1)
        self.blocks = nn.ModuleList(ConvUnit(filters, filters, 3, bn=True) for _ in range(layers))
        self.head_p = BoardHead(filters, 9, 2, 9)
        self.head_v = BoardHead(filters, 9, 1, 1)

    def forward(self, x, hidden=None):
        h = F.relu(self.conv(x))
        for blk in self.blocks:
            h = F.relu(blk(h))
        return {'policy': self.head_p(h), 'value': torch.tanh(self.head_v(h))}


class Environment(BaseEnvironment):
    BLACK, WHITE = 1, -1
    MARKS = {0: '_', 1: 'O', -1: 'X'}
    LINES = [(0, 1, 2), (3, 4, 5), (6, 7, 8), (0, 3, 6), (1, 4, 7), (2, 5, 8), (0, 4, 8), (2, 4, 6)]

    def __init__(self, args=None):
        super().__init__(args)
        self.reset()

    def reset(self, args=None):
        self.cells = np.zeros(9, dtype=np.float32)
        self.color = self.BLACK
        self.winner = 0
        self.record = []

    def __str__(self):
        rows = [' '.join(self.MARKS[int(c)] for c in self.cells[r * 3:r * 3 + 3]) for r in range(3)]
        return '\n'.join(rows) + '\nrecord = ' + ' '.join(self.action2str(a) for a in self.record)

    def action2str(self, a, _=None):
        return 'ABC'[a // 3] + '123'[a % 3]

    def str2action(self, s, _=None):
        return 'ABC'.index(s[0]) * 3 + '123'.index(s[1])

    def play(self, action, _=None):
        self.cells[action] = self.color
        if any(all(self.cells[i] == self.color for i in line) for line in self.LINES if action in line):
            self.winner = self.color
        self.color = -self.color
        self.record.append(action)

    def diff_info(self, _=None):
        return self.action2str(self.record[-1]) if self.record else ''

    def update(self, info, reset):
        if reset:
            self.reset()
        else:
            self.play(self.str2action(info))

    def turn(self):
        return len(self.record) % 2

    def terminal(self):
        return self.winner != 0 or len(self.record) == 9

    def outcome(self):
        o = {0: 0, 1: 0}
        if self.winner:
            o = {0: self.winner, 1: -self.winner}
        return o

    def legal_actions(self, _=None):
        return [a for a in range(9) if self.cells[a] == 0]

    def action_length(self):
        return 9

    def players(self):
        return [0, 1]

    def net(self):
        return SimpleConv2dModel

    def observation(self, player=None):
        mine = player is None or player == self.turn()
        me = self.color if mine else -self.color
        board = self.cells.reshape(3, 3)
        return np.stack([np.full((3, 3), 1.0 if mine else 0.0, dtype=np.float32),
                         (board == me).astype(np.float32),
                         (board == -me).astype(np.float32)])


if __name__ == '__main__':
    e = Environment()
    while not e.terminal():
        e.play(random.choice(e.legal_actions()))
    print(e)
    print(e.outcome())
