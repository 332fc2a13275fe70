"""Parallel Tic-Tac-Toe: both players choose a move every turn and one of the
two, picked at random, is played (handyrl/envs/parallel_tictactoe.py:13-61).
A simultaneous-move game (``turns()`` = both players) over the TicTacToe
rules, net and observation of envs/tictactoe.py.
"""

import random

from .tictactoe import Environment as TicTacToe


class Environment(TicTacToe):
    def step(self, actions):
        player = random.choice(list(actions.keys()))
        self._place(actions[player], player)

    def _place(self, action, player):
        colour = (self.BLACK, self.WHITE)[player]
        self.cells[action] = colour
        if any(all(self.cells[i] == colour for i in line) for line in self.LINES if action in line):
            self.winner = colour
        self.record.append((colour, action))

    def terminal(self):
        return self.winner != 0 or len(self.record) == 9

    def diff_info(self, _=None):
        if not self.record:
            return ''
        colour, action = self.record[-1]
        return self.action2str(action) + ':' + self.MARKS[colour]

    def update(self, info, reset):
        if reset:
            self.reset()
        else:
            move, mark = info.split(':')
            self._place(self.str2action(move), 'OX'.index(mark))

    def turn(self):
        # no single turn player (the reference returns an exception object here, which equals no
        # player): observation(p) is then the non-turn view of the black stones' side for both p
        return None

    def turns(self):
        return self.players()
