"""Geister network: the recurrent (DRC ConvLSTM) model of config C3.

Architecture and state_dict keys follow GeisterNet in handyrl/envs/geister.py
(:17-167), and the modules are constructed in the same order, so
``torch.manual_seed(s); GeisterNet()`` yields the reference's initial weights
bit for bit (pinned by tests/golden/geister_net.json):

* input: 18 scalar features broadcast over the 6x6 board, concatenated in
  front of the 7 board planes -> 25 x 6 x 6 (geister.py:151-153);
* stem: 3x3 conv 25->32 (no bias) -> BN -> ReLU = h_e;
* body: DRC, 3 ConvLSTM cells (3x3 conv of [x, h] 64 -> 128 with bias,
  gates i, f, o, g in that channel order) applied 3 times per time step
  (geister.py:66-98); the hidden state is (hs, cs), 3 tensors each;
* heads on [h_e, h_last] (64 x 6 x 6): move policy 3x3 conv 64->8 -> BN ->
  ReLU -> 1x1 conv 8->4 (144 logits), set policy Linear(1, 70) of the turn
  colour (scalar[0]); value / return 1x1 conv 64->1 -> BN -> ReLU -> Linear(36, 1);
  value through tanh.  233,832 parameters.

The rules stay in the reference plugin (handyrl.envs.geister.Environment,
geister.py:170-541): the learner only needs the net and the observation
format {'board': (7, 6, 6), 'scalar': (18,)}, 214 actions.
"""

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

BOARD = (6, 6)
BOARD_PLANES = 7
SCALARS = 18
ACTIONS = 214


class ConvLSTMCell(nn.Module):
    """One ConvLSTM cell: gates = conv([x, h]); c' = f*c + i*g; h' = o*tanh(c')."""

    def __init__(self, input_dim, hidden_dim, kernel_size, bias):
        super().__init__()
        self.input_dim = input_dim
        self.hidden_dim = hidden_dim
        self.kernel_size = kernel_size
        self.conv = nn.Conv2d(input_dim + hidden_dim, 4 * hidden_dim, kernel_size,
                              padding=(kernel_size[0] // 2, kernel_size[1] // 2), bias=bias)

    def init_hidden(self, input_size, batch_size):
        shape = (self.hidden_dim, *input_size)
        if batch_size is None:      # one inference state (numpy, like the reference's agents)
            return np.zeros(shape, np.float32), np.zeros(shape, np.float32)
        return torch.zeros(*batch_size, *shape), torch.zeros(*batch_size, *shape)

    def forward(self, x, state):
        h, c = state
        gates = self.conv(torch.cat([x, h], dim=-3))
        gi, gf, go, gg = gates.chunk(4, dim=-3)
        c = torch.sigmoid(gf) * c + torch.sigmoid(gi) * torch.tanh(gg)
        return torch.sigmoid(go) * torch.tanh(c), c


class DRC(nn.Module):
    """Stack of ConvLSTM cells, each fed the same encoder output, repeated per step."""

    def __init__(self, num_layers, input_dim, hidden_dim, kernel_size=3, bias=True):
        super().__init__()
        self.num_layers = num_layers
        self.blocks = nn.ModuleList(ConvLSTMCell(input_dim, hidden_dim, (kernel_size, kernel_size), bias)
                                    for _ in range(num_layers))

    def init_hidden(self, input_size, batch_size):
        states = [blk.init_hidden(input_size, batch_size) for blk in self.blocks]
        return [s[0] for s in states], [s[1] for s in states]

    def forward(self, x, hidden, num_repeats):
        if hidden is None:
            hidden = self.init_hidden(x.shape[-2:], x.shape[:-3])
        hs, cs = list(hidden[0]), list(hidden[1])
        for _ in range(num_repeats):
            for i, blk in enumerate(self.blocks):
                hs[i], cs[i] = blk(x, (hs[i], cs[i]))
        return hs[-1], (hs, cs)


class Conv2dHead(nn.Module):
    """3x3 conv -> BN -> ReLU -> 1x1 conv, flattened to (N, H*W*output_filters)."""

    def __init__(self, input_shape, filters, output_filters):
        super().__init__()
        self.outputs = input_shape[1] * input_shape[2] * output_filters
        self.conv1 = nn.Conv2d(input_shape[0], filters, 3, padding=1, bias=False)
        self.bn = nn.BatchNorm2d(filters)
        self.conv2 = nn.Conv2d(filters, output_filters, 1, bias=False)

    def forward(self, x):
        return self.conv2(F.relu(self.bn(self.conv1(x)))).reshape(-1, self.outputs)


class ScalarHead(nn.Module):
    """1x1 conv -> BN -> ReLU -> flatten -> bias-free linear."""

    def __init__(self, input_shape, filters, outputs):
        super().__init__()
        self.hidden_units = input_shape[1] * input_shape[2] * filters
        self.conv = nn.Conv2d(input_shape[0], filters, 1, bias=False)
        self.bn = nn.BatchNorm2d(filters)
        self.fc = nn.Linear(self.hidden_units, outputs, bias=False)

    def forward(self, x):
        return self.fc(F.relu(self.bn(self.conv(x))).reshape(-1, self.hidden_units))


class GeisterNet(nn.Module):
    def __init__(self, layers=3, filters=32, p_filters=8, num_repeats=3):
        super().__init__()
        cin = BOARD_PLANES + SCALARS
        self.input_size = (cin, *BOARD)
        self.num_repeats = num_repeats
        # construction order = reference order (RNG stream of the default initialisers)
        self.conv1 = nn.Conv2d(cin, filters, 3, padding=1, bias=False)
        self.bn1 = nn.BatchNorm2d(filters)
        self.body = DRC(layers, filters, filters)
        self.head_p_move = Conv2dHead((2 * filters, *BOARD), p_filters, 4)
        self.head_p_set = nn.Linear(1, 70, bias=True)
        self.head_v = ScalarHead((2 * filters, *BOARD), 1, 1)
        self.head_r = ScalarHead((2 * filters, *BOARD), 1, 1)

    def init_hidden(self, batch_size=None):
        return self.body.init_hidden(BOARD, batch_size)

    def forward(self, x, hidden):
        board, scalar = x['board'], x['scalar']
        planes = scalar[..., None, None].expand(*scalar.shape, *BOARD)
        h_e = F.relu(self.bn1(self.conv1(torch.cat([planes, board], dim=-3))))
        h_last, hidden = self.body(h_e, hidden, self.num_repeats)
        h = torch.cat([h_e, h_last], dim=-3)
        policy = torch.cat([self.head_p_move(h), self.head_p_set(scalar[:, :1])], dim=-1)
        return {'policy': policy, 'value': torch.tanh(self.head_v(h)), 'return': self.head_r(h),
                'hidden': hidden}
