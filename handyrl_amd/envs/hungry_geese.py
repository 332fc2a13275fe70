"""Hungry Geese network: the feed-forward torus-conv model of config C4.

Architecture and state_dict keys follow GeeseNet in
handyrl/envs/kaggle/hungry_geese.py (:23-57), with the modules constructed in
the same order (so ``torch.manual_seed(s); GeeseNet()`` draws the same
initial weights as the reference module would):

* TorusConv2d (:23-35): 3x3 convolution on the 7x11 torus -- the board wraps
  in both directions -- followed by BatchNorm2d when ``bn``; the reference
  builds the wrap with two concatenations and a 'valid' conv;
* stem 17 -> 32, then 12 residual blocks h = relu(h + bn(conv(h))) (:48-51);
* heads (:52-55): h_head = sum over cells of h * x[:, :1] (the goose-head
  plane), h_avg = mean over cells; policy Linear(32, 4), value
  tanh(Linear(64, 1)), both bias-free.  116,928 parameters.

The rules live in kaggle_environments, which is not installed here, so this
module has no rules of its own; ``Environment`` raises an ImportError that
points to the reference plugin by module path (``make_env`` imports any
module path, so ``env: handyrl.envs.kaggle.hungry_geese`` in config.yaml
drops the reference env in unchanged).  The learner trains GeeseNet
on make_batch-layout batches (solo training, turn_based_training=False:
P = Pp = 1, train.py:57-58), see synthetic.geese_batch.

On the GPU the torus convolutions run as csrc/hrl_torus.hip (wrap-around
addressing in the kernel, no padded copy) once ``nn.accelerate`` has swapped
``TorusConv2d`` for its HIP form.
"""

import torch
import torch.nn as nn
import torch.nn.functional as F

BOARD = (7, 11)
PLANES = 17
ACTIONS = 4


class TorusConv2d(nn.Module):
    """kxk convolution with wrap-around (torus) padding, then optional BatchNorm2d."""

    def __init__(self, input_dim, output_dim, kernel_size, bn):
        super().__init__()
        self.edge_size = (kernel_size[0] // 2, kernel_size[1] // 2)
        self.conv = nn.Conv2d(input_dim, output_dim, kernel_size=kernel_size)
        self.bn = nn.BatchNorm2d(output_dim) if bn else None

    def wrap(self, x):
        eh, ew = self.edge_size
        h = torch.cat([x[:, :, :, -ew:], x, x[:, :, :, :ew]], dim=3)
        return torch.cat([h[:, :, -eh:], h, h[:, :, :eh]], dim=2)

    use_hip = False   # set by nn.accelerate: the conv runs as csrc/hrl_torus.hip (no wrapped copy)

    def forward(self, x):
        # a CPU copy of an accelerated net (Trainer.train returns one for the workers) runs the torch form
        if self.use_hip and x.is_cuda:
            from ..nn import torus_conv2d, torus_supported
            if not torus_supported(x, self.conv.weight):
                raise RuntimeError('TorusConv2d: shape %s x %s is outside the HIP torus conv'
                                   % (tuple(x.shape), tuple(self.conv.weight.shape)))
            h = torus_conv2d(x, self.conv.weight, self.conv.bias)
        else:
            h = self.conv(self.wrap(x))
        return self.bn(h) if self.bn is not None else h


class GeeseNet(nn.Module):
    def __init__(self, layers=12, filters=32):
        super().__init__()
        self.conv0 = TorusConv2d(PLANES, filters, (3, 3), True)
        self.blocks = nn.ModuleList([TorusConv2d(filters, filters, (3, 3), True) for _ in range(layers)])
        self.head_p = nn.Linear(filters, ACTIONS, bias=False)
        self.head_v = nn.Linear(filters * 2, 1, bias=False)

    def forward(self, x, _=None):
        if self.training and self.conv0.use_hip and self.conv0.bn is not None and x.is_cuda:
            # accelerated training step: the unit chain is one HIP Function (nn.torus_tower)
            from ..nn import torus_tower
            h = torus_tower(x, [self.conv0, *self.blocks])
        else:
            h = F.relu(self.conv0(x))
            for block in self.blocks:
                h = F.relu(h + block(h))
        n, c = h.size(0), h.size(1)
        if self.conv0.use_hip and h.is_cuda:
            from ..nn import geese_pool
            h_head, h_avg = geese_pool(h, x)   # one HIP pass each way
        else:
            h_head = (h * x[:, :1]).view(n, c, -1).sum(-1)
            h_avg = h.view(n, c, -1).mean(-1)
        p = self.head_p(h_head)
        v = torch.tanh(self.head_v(torch.cat([h_head, h_avg], 1)))
        return {'policy': p, 'value': v}


class Environment:
    """Hungry Geese rules.  The reference's rules wrap kaggle_environments (hungry_geese.py:18, :60-230) and are
    not restated here, and this package never imports the reference.  ``Environment(args)`` raises an
    ImportError naming the way in: with kaggle_environments and a HandyRL checkout importable, name the
    reference plugin by module path in ``config.yaml`` (``env: handyrl.envs.kaggle.hungry_geese``), which
    ``make_env`` imports as given; its ``net()`` has this module's GeeseNet keys, so ``nn.accelerate`` runs it on
    the HIP torus convs."""

    def __init__(self, args=None):
        raise ImportError("Hungry Geese rules live in the reference plugin (they need kaggle_environments): set "
                          "'env: handyrl.envs.kaggle.hungry_geese' in config.yaml with kaggle_environments and a "
                          "HandyRL checkout importable; GeeseNet itself trains on make_batch-layout batches "
                          "without them")

    def net(self):
        return GeeseNet
