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

``GeisterBatch`` restates the rules (geister.py:170-541) as tensor ops over
E concurrent games for device self-play (rollout.DeviceGenerator); the
per-game plugin ``Environment`` (the reference's API, geister.py:170-541) is
one such game on the CPU, so both share one statement of the rules.
Observation format
{'board': (7, 6, 6), 'scalar': (18,)}, 214 actions.
"""

import contextlib
import os

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from ..environment import BaseEnvironment

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


def _stacked(ts):
    """The layers' states as one (E, n*H, *HW) tensor: a view when they are adjacent channel slices of one
    contiguous tensor (GeisterNet.inference_hidden), a concatenation otherwise."""
    t0 = ts[0]
    E, hd = t0.shape[0], t0.shape[1]
    inner = t0[0].numel()
    n = len(ts)
    if (t0[0].is_contiguous() and t0.stride(0) == n * inner
            and all(t.shape == t0.shape and t.stride() == t0.stride()
                    and t.storage_offset() == t0.storage_offset() + i * inner
                    and t.untyped_storage().data_ptr() == t0.untyped_storage().data_ptr()
                    for i, t in enumerate(ts))):
        return t0.as_strided((E, n * hd, *t0.shape[2:]), (n * inner, *t0.stride()[1:]))
    return torch.cat(ts, 1)


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

    use_hip = False   # set by handyrl_amd.nn.accelerate

    def forward(self, x, hidden, num_repeats):
        if hidden is None:
            hidden = tuple([t.to(x.device) for t in ts] for ts in self.init_hidden(x.shape[-2:], x.shape[:-3]))
        hs, cs = list(hidden[0]), list(hidden[1])
        if self.use_hip and x.is_cuda:
            if not torch.is_grad_enabled():
                return self._inference_stacked(x, hs, cs, num_repeats)
            return self._forward_hip(x, hs, cs, num_repeats)
        for _ in range(num_repeats):
            for i, blk in enumerate(self.blocks):
                hs[i], cs[i] = blk(x, (hs[i], cs[i]))
        return hs[-1], (hs, cs)

    def _forward_hip(self, x, hs, cs, num_repeats):
        """Same cells, regrouped: conv([x, h]) = conv_x(x) + conv_h(h).

        Every repeat of every layer sees the same x, so the x halves of the
        three layers run once, as one 32 -> 3*128 convolution (bias folded in);
        each cell then convolves only its h (32 -> 128) and the fused HIP gate
        kernel adds the two (nn.lstm_gates).  A third fewer cell FLOPs, no
        concatenation, one gate launch per cell and direction.
        """
        return self.step_hip(self.x_halves(x), hs, cs, num_repeats)

    _session = None   # the stacked weights of an inference session (DRC.inference_session)
    # the learner's unroll: each repeat's layers as one grouped h-half conv + one grouped gate launch
    # (nn.drc_step) instead of a conv and a gate launch per layer
    group_repeat = os.environ.get('HRL_DRC_GROUPED', '1') == '1'
    _inplace = False  # the session advances a stacked state in place (DeviceGenerator)

    def _stacked_weights(self, out=None):
        """The layers' x-half weights and biases and h-half weights, concatenated along the output channels
        (into ``out``'s tensors when given)."""
        ws = [blk.conv.weight for blk in self.blocks]
        cin = ws[0].shape[1] - self.blocks[0].hidden_dim
        out = out or {}
        w_x = torch.cat([w[:, :cin] for w in ws], out=out.get('w_x'))
        w_h = torch.cat([w[:, cin:] for w in ws], out=out.get('w_h'))
        b_x = None
        if self.blocks[0].conv.bias is not None:
            b_x = torch.cat([blk.conv.bias for blk in self.blocks], out=out.get('b_x'))
        res = {'w_x': w_x, 'w_h': w_h, 'b_x': b_x}
        if self._gboard_ok(w_x, w_h):   # the same weights as hrl_gboard's split fragments, packed once
            from .. import nn as hnn
            res['pk_x'] = hnn.gboard_pack(w_x, out=out.get('pk_x'))
            res['pk_h'] = hnn.gboard_pack(w_h, out=out.get('pk_h'))
        return res

    def _gboard_ok(self, w_x, w_h):
        n = len(self.blocks)
        conv = self.blocks[0].conv
        return (w_x.is_cuda and tuple(conv.kernel_size) == (3, 3) and tuple(conv.padding) == (1, 1)
                and tuple(conv.stride) == (1, 1) and tuple(conv.dilation) == (1, 1) and conv.groups == 1
                and w_x.shape[1] <= 64 and w_h.shape[1] <= 64 and (w_h.shape[0] // n) % 16 == 0)

    @contextlib.contextmanager
    def inference_session(self, inplace_state=False):
        """Within the session the stacked inference weights are built once (refreshed in place from the
        current parameters on entry, so HIP graphs captured in an earlier session stay valid) instead of
        once per forward: DeviceGenerator.generate runs its plies in one.  ``inplace_state``: a state given
        in the stacked layout (GeisterNet.inference_hidden) is advanced in place and returned as views of
        itself -- the caller's state buffers ARE the new state (the generator's own buffers only)."""
        with torch.no_grad():
            self._session_buf = self._stacked_weights(getattr(self, '_session_buf', None))
        self._session = self._session_buf
        self._inplace = inplace_state
        try:
            yield
        finally:
            self._session = None
            self._inplace = False

    def _inference_stacked(self, x, hs, cs, num_repeats):
        """Inference (self-play, no autograd) with the layers stacked along channels.

        Within a repeat the cells are independent (each reads x and its own state), so the n layers' h
        halves run as ONE grouped convolution (n*H -> n*4H, groups = n) and their gates as one HIP
        launch over n*E cells; the x halves are one n*4H-channel convolution as in _forward_hip.  Per
        step n*repeats convolutions and gate passes become repeats of each (9 -> 3 for GeisterNet).
        The grouped convolution computes each group's products as the per-layer one does
        (tests/test_geister.py::test_stacked_inference_matches_cells).  The state comes back as channel
        slices of the stacked tensors."""
        from .. import nn as hnn
        from ..nn import lstm_gates
        n = len(self.blocks)
        ws = [blk.conv.weight for blk in self.blocks]
        pad = self.blocks[0].conv.padding
        hd = self.blocks[0].hidden_dim
        cin = ws[0].shape[1] - hd
        E, HW = x.shape[0], x.shape[-2:]
        cache = self._session
        if cache is None:
            cache = self._stacked_weights()
        w_h = cache['w_h']                                                               # (n*4H, H, 3, 3)
        h, c = _stacked(hs), _stacked(cs)                                                # (E, n*H, *HW)
        # the 6x6 board's convolutions on hrl_gboard (games as MFMA rows, fp32-accurate split)
        gb = 'pk_x' in cache and hnn.gboard_ok(x) and hnn.gboard_ok(h)
        if gb:
            z = hnn.gboard_conv(x, cache['pk_x'], n * 4 * hd, cin)                       # (E, n*4H, *HW)
        else:
            z = F.conv2d(x, cache['w_x'], None, padding=pad)
        # in an in-place session (DeviceGenerator's own stacked state) the gates write the new state over
        # the old one: h is consumed by the convolution before, c read and written at the same index
        inplace = (self._inplace and h.is_contiguous() and c.is_contiguous()
                   and h.data_ptr() == hs[0].data_ptr() and c.data_ptr() == cs[0].data_ptr())
        zx = z.view(E * n, 4 * hd, *HW)
        for _ in range(num_repeats):
            if gb and hnn.gboard_ok(h):
                zh = hnn.gboard_conv(h, cache['pk_h'], n * 4 * hd, hd, groups=n)
            else:
                zh = F.conv2d(h, w_h, None, padding=pad, groups=n)
            out = (h.view(E * n, hd, *HW), c.view(E * n, hd, *HW)) if inplace else None
            # the x half's bias rides in the gate kernel: (zx + b) + zh, the biased convolution's order
            hn, cn = lstm_gates(zx, zh.view(E * n, 4 * hd, *HW), c.view(E * n, hd, *HW), cache['b_x'], n, out=out)
            h, c = hn.view(E, n * hd, *HW), cn.view(E, n * hd, *HW)
        hs, cs = list(h.split(hd, 1)), list(c.split(hd, 1))
        return hs[-1], (hs, cs)

    def x_halves(self, x):
        """conv_x(x) + bias of every cell (the part of conv([x, h]) that does not depend on the state); x may
        hold the encoder outputs of every time step of an unroll at once (GeisterNet.sequence_begin)."""
        from .. import nn as hnn
        from ..nn import conv2d
        cin = x.shape[-3]
        ws = [blk.conv.weight for blk in self.blocks]
        bias = [blk.conv.bias for blk in self.blocks]
        pad = self.blocks[0].conv.padding
        n = len(self.blocks)
        deferred = hnn._DEFER is not None   # LearnerStep batches the weight gradients over the unroll

        def x_half(layers):
            if len(layers) == 1 and deferred:   # the weight's input-channel slice, gradient deferred
                return (conv2d(x, ws[layers[0]], bias[layers[0]], pad, in_slice=(0, cin)),)
            w_x = torch.cat([ws[i][:, :cin] for i in layers])
            b_x = None if bias[0] is None else torch.cat([bias[i] for i in layers])
            if deferred and n > 1 and layers[-1] < n - 1 and hnn.gboard_conv_ok(x, w_x, cin, pad):
                # the learner's layers that reach no output (see below): forward only, on hrl_gboard
                with torch.no_grad():
                    z = hnn.gboard_conv(x, hnn.gboard_pack(w_x), w_x.shape[0], cin,
                                        bias=None if b_x is None else b_x.detach())
                return z.chunk(len(layers), dim=-3)
            return F.conv2d(x, w_x, b_x, padding=pad).chunk(len(layers), dim=-3)
        if torch.is_grad_enabled() and n > 1:
            # Only the last layer reaches the output (every cell reads x and its own state), so the
            # others must stay outside its autograd graph: their weights then get no gradient at
            # all, as with the reference's cells, and the optimizer leaves them alone.
            return list(x_half(list(range(n - 1))) + x_half([n - 1]))
        return list(x_half(list(range(n))))

    def step_hip(self, zx, hs, cs, num_repeats, packed_h=None):
        """One time step of the cells given their x halves zx (DRC.forward's repeats and layers); packed_h:
        the cells' h-half weights packed for the board conv (GeisterNet.sequence_begin), or None."""
        from .. import nn as hnn
        from ..nn import lstm_gates, conv2d
        ws = [blk.conv.weight for blk in self.blocks]
        pad = self.blocks[0].conv.padding
        c_all = ws[0].shape[1]
        cin = c_all - self.blocks[0].hidden_dim
        deferred = hnn._DEFER is not None
        w_h = None if deferred else [w[:, cin:].contiguous() for w in ws]
        if (deferred and isinstance(packed_h, dict) and self.group_repeat
                and hnn.drc_step_ok(zx, hs, cs, ws, pad)):
            # every repeat's layers in two launches (the grouped h-half conv and the grouped gates), the step's
            # repeats under one autograd node (nn.drc_step)
            hs, cs = hnn.drc_step(zx, hs, cs, ws, (cin, c_all), pad, packed_h['grouped'], num_repeats)
            return hs[-1], (hs, cs)
        if isinstance(packed_h, dict):
            packed_h = packed_h['layers']
        for _ in range(num_repeats):
            for i in range(len(self.blocks)):
                if deferred:
                    zh = conv2d(hs[i], ws[i], None, pad, in_slice=(cin, c_all),
                                packed=None if packed_h is None else packed_h[i])
                else:
                    zh = F.conv2d(hs[i], w_h[i], None, padding=pad)
                hs[i], cs[i] = lstm_gates(zx[i], zh, cs[i])
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

    def inference_hidden(self, E, P, device):
        """Self-play state for E games and P players, player-major: leaf l is (P, E, H, 6, 6) and the
        layers' leaves are adjacent channel slices of one (P, E, layers*H, 6, 6) tensor per kind, so the
        mover's state h[p] is already the stacked input of DRC._inference_stacked (no concatenation)."""
        n, hd = len(self.body.blocks), self.body.blocks[0].hidden_dim
        out = []
        for _ in range(2):   # h, c
            buf = torch.zeros(P, E, n * hd, *BOARD, device=device)
            out.append([buf[:, :, i * hd:(i + 1) * hd] for i in range(n)])
        return tuple(out)

    def forward(self, x, hidden):
        if (not self.training and self.body.use_hip and not torch.is_grad_enabled() and x['board'].is_cuda
                and all(b.running_mean is not None for b in self._sequence_bns())):
            return self._forward_inference(x, hidden)
        board, scalar = x['board'], x['scalar']
        planes = scalar[..., None, None].expand(*scalar.shape, *BOARD)
        h_e = F.relu(self.bn1(self.conv1(torch.cat([planes, board], dim=-3))))
        h_last, hidden = self.body(h_e, hidden, self.num_repeats)
        h = torch.cat([h_e, h_last], dim=-3)
        policy = torch.cat([self.head_p_move(h), self.head_p_set(scalar[:, :1])], dim=-1)
        return {'policy': policy, 'value': torch.tanh(self.head_v(h)), 'return': self.head_r(h),
                'hidden': hidden}

    _bn_coef = None   # BatchNorm (alpha, beta) of an inference session, per module
    _vr_session = None   # the value / return heads stacked for an inference session
    _gb_session = None   # hrl_gboard's packed stem / move-head weights of an inference session

    @contextlib.contextmanager
    def inference_session(self, inplace_state=False):
        """Per-call preparation for self-play (DeviceGenerator.generate): the DRC's stacked weights and the
        four BatchNorms' inference coefficients alpha = invstd * weight, beta = bias - mean * alpha
        (hrl_bn_forward_eval's own coefficient kernel) are refreshed in place once, so a ply is only the
        apply passes.  Outside a session every forward derives them itself."""
        from .. import _native
        from .. import nn as hnn
        bufs = getattr(self, '_bn_coef_buf', None) or {}
        with torch.no_grad():
            for name, bn in (('bn1', self.bn1), ('p', self.head_p_move.bn), ('v', self.head_v.bn),
                             ('r', self.head_r.bn)):
                C = bn.num_features
                if name not in bufs:
                    bufs[name] = (torch.empty(2 * C, device=bn.running_mean.device),
                                  torch.zeros(1, C, 1, 1, device=bn.running_mean.device))
                coef, dummy = bufs[name]
                if coef.is_cuda:
                    _native.check(_native.load().hrl_bn_forward_eval(
                        _native.ptr(dummy), 1, C, 1, _native.ptr(bn.weight), _native.ptr(bn.bias),
                        _native.ptr(bn.running_mean), _native.ptr(bn.running_var), float(bn.eps), 1,
                        _native.ptr(torch.empty_like(dummy)), _native.ptr(coef), _native.stream_of(coef.device)),
                        'hrl_bn_forward_eval')
        self._bn_coef_buf = bufs
        self._bn_coef = {id(m): bufs[k][0] for k, m in (('bn1', self.bn1), ('p', self.head_p_move.bn),
                                                         ('v', self.head_v.bn), ('r', self.head_r.bn))}
        gb = getattr(self, '_gb_buf', None) or {}
        self._gb_session = None
        c1, hc = self.conv1, self.head_p_move.conv1
        if (bufs['bn1'][0].is_cuda and BOARD == (6, 6)
                and all(tuple(c.kernel_size) == (3, 3) and tuple(c.padding) == (1, 1) and tuple(c.stride) == (1, 1)
                        and c.groups == 1 and c.bias is None for c in (c1, hc))
                and c1.weight.shape[1] <= 32 and hc.weight.shape[1] == 2 * c1.weight.shape[0] == 64
                and self.head_p_move.conv2.bias is None and self.head_p_move.conv2.weight.shape[0] in (1, 2, 4, 8)
                and tuple(self.head_p_move.conv2.weight.shape[2:]) == (1, 1)):
            with torch.no_grad():   # hrl_gboard's split fragments of the stem and move-head convolutions
                gb['conv1'] = hnn.gboard_pack(c1.weight, out=gb.get('conv1'))
                gb['head'] = hnn.gboard_pack(hc.weight, out=gb.get('head'))
                w2 = self.head_p_move.conv2.weight
                gb['head2'] = w2.detach().clone() if gb.get('head2') is None else gb['head2'].copy_(w2)
            self._gb_buf = gb
            self._gb_session = gb
        hv, hr = self.head_v, self.head_r
        if (bufs['v'][0].is_cuda and hv.conv.weight.shape[0] == 1 and hr.conv.weight.shape[0] == 1
                and hv.bn.num_features == 1 and hr.bn.num_features == 1):
            with torch.no_grad():   # [alpha_v, alpha_r, beta_v, beta_r] and the two 1x1 conv weights
                vr = getattr(self, '_vr_buf', None) or {}
                vr['w'] = torch.cat([hv.conv.weight, hr.conv.weight], out=vr.get('w'))
                cv, cr = bufs['v'][0], bufs['r'][0]
                vr['coef'] = torch.cat([cv[:1], cr[:1], cv[1:], cr[1:]], out=vr.get('coef'))
            self._vr_buf = vr
            self._vr_session = vr
        try:
            with self.body.inference_session(inplace_state):
                yield
        finally:
            self._bn_coef = None
            self._vr_session = None
            self._gb_session = None

    def _forward_inference(self, x, hidden):
        """forward in eval mode without autograd on the HIP path (self-play): the same operations, with each
        BatchNorm's ReLU folded into its HIP inference kernel (4 launches fewer per ply) and the DRC stacked
        (DRC._inference_stacked)."""
        from ..nn import batch_norm_eval

        coefs = self._bn_coef

        def bn_relu(bn, y):
            if coefs is None or id(bn) not in coefs:
                return batch_norm_eval(y, bn.weight, bn.bias, bn.running_mean, bn.running_var, bn.eps, relu=True)
            from .. import _native
            y = y.contiguous()
            out = torch.empty_like(y)
            C = y.shape[1]
            coef = coefs[id(bn)]
            _native.check(_native.load().hrl_bn_apply(
                _native.ptr(y), y.shape[0], C, y[0, 0].numel(), _native.ptr(coef), _native.ptr(coef[C:]), 1,
                _native.ptr(out), _native.stream_of(y.device)), 'hrl_bn_apply')
            return out
        from .. import nn as hnn
        board, scalar = x['board'], x['scalar']
        planes = scalar[..., None, None].expand(*scalar.shape, *BOARD)
        x_in = torch.cat([planes, board], dim=-3)
        gb = self._gb_session
        if gb is not None and hnn.gboard_ok(x_in):   # the conv with the BatchNorm + ReLU in its epilogue
            C = self.bn1.num_features
            c1 = coefs[id(self.bn1)]
            h_e = hnn.gboard_conv(x_in, gb['conv1'], C, x_in.shape[1], alpha=c1[:C], beta=c1[C:], relu=True)
        else:
            h_e = bn_relu(self.bn1, self.conv1(x_in))
        h_last, hidden = self.body(h_e, hidden, self.num_repeats)
        hp, hv, hr = self.head_p_move, self.head_v, self.head_r
        # in a session on the 6x6 board every head convolution is a HIP kernel reading [h_e, h_last] in place
        # (no concatenation): the move head's 3x3 conv with its BatchNorm + ReLU epilogue and its 1x1 conv,
        # and the value / return heads' 1x1 convs as one 2-channel pointwise pass with both BatchNorms + ReLUs
        two = gb is not None and hnn.gboard_ok(h_e, x2=h_last)
        h = None if two else torch.cat([h_e, h_last], dim=-3)
        if two:
            C = hp.bn.num_features
            cp = coefs[id(hp.bn)]
            a = hnn.gboard_conv(h_e, gb['head'], C, 2 * h_e.shape[1], x2=h_last, alpha=cp[:C], beta=cp[C:],
                                relu=True)
            p_move = hnn.gboard_pointwise(a, gb['head2']).reshape(-1, hp.outputs)
        else:
            p_move = hp.conv2(bn_relu(hp.bn, hp.conv1(h))).reshape(-1, hp.outputs)
        policy = torch.cat([p_move, self.head_p_set(scalar[:, :1])], dim=-1)
        vr = self._vr_session
        if vr is not None and hv.hidden_units == hr.hidden_units:
            # in a session the value and return heads' 1x1 convs run as one 2-channel conv and their
            # BatchNorm + ReLU as one apply (per-channel: the same values as the two heads apart)
            from .. import _native
            if two:
                a = hnn.gboard_pointwise(h_e, vr['w'], x2=h_last, alpha=vr['coef'][:2], beta=vr['coef'][2:],
                                         relu=True)
            else:
                y = F.conv2d(h, vr['w'])
                a = torch.empty_like(y)
                _native.check(_native.load().hrl_bn_apply(
                    _native.ptr(y), y.shape[0], 2, y[0, 0].numel(), _native.ptr(vr['coef']),
                    _native.ptr(vr['coef'][2:]), 1, _native.ptr(a), _native.stream_of(y.device)), 'hrl_bn_apply')
            v = hv.fc(a[:, 0].reshape(-1, hv.hidden_units))
            r = hr.fc(a[:, 1].reshape(-1, hr.hidden_units))
        else:
            if h is None:
                h = torch.cat([h_e, h_last], dim=-3)
            v = hv.fc(bn_relu(hv.bn, hv.conv(h)).reshape(-1, hv.hidden_units))
            r = hr.fc(bn_relu(hr.bn, hr.conv(h)).reshape(-1, hr.hidden_units))
        return {'policy': policy, 'value': torch.tanh(v), 'return': r, 'hidden': hidden}

    # ---- the learner's unroll in three parts (train._unroll_sequence) ----
    # forward_prediction runs the net once per time step (train.py:155-174).  Only the cells depend on
    # the state, so on the HIP path the stem, the cells' x halves and the heads run once over all T
    # steps (rows time-major, T*N), with every BatchNorm normalising each step's rows with that step's
    # own statistics and advancing its running statistics once per step, in order
    # (nn.batch_norm_train(groups=T)): the same results as T calls of forward, in far fewer launches.

    def _sequence_bns(self):
        return (self.bn1, self.head_p_move.bn, self.head_v.bn, self.head_r.bn)

    def sequence_ok(self, x):
        from .. import nn as hnn
        return (self.training and self.body.use_hip and torch.is_grad_enabled() and x['board'].is_cuda
                and x['board'].dtype == torch.float32
                and all(isinstance(b, hnn.BatchNorm2d) and b.momentum is not None and b.track_running_stats
                        and b.affine for b in self._sequence_bns()))

    @staticmethod
    def _bn_steps(bn, y, T):
        """relu(bn(y)) for T time steps' rows (time-major) with per-step statistics."""
        from .. import nn as hnn
        from ..nn import batch_norm_train
        if bn.momentum is None or not hnn._defer_counters([bn.num_batches_tracked], T):
            bn.num_batches_tracked.add_(T)      # else advanced by the learner's step tail
        return batch_norm_train(y, bn.weight, bn.bias, bn.running_mean, bn.running_var, bn.momentum, bn.eps,
                                relu=True, groups=T)

    def sequence_begin(self, x, T):
        """Stem and the cells' x halves for all T steps; x: observations with rows (t, n)."""
        board, scalar = x['board'], x['scalar']
        planes = scalar[..., None, None].expand(*scalar.shape, *BOARD)
        h_e = self._bn_steps(self.bn1, self.conv1(torch.cat([planes, board], dim=-3)), T)
        N = board.shape[0] // T
        # per-step views under ONE autograd node: the backward is a single concatenation, not T slice
        # gradients accumulated
        zx = [z.split(N) for z in self.body.x_halves(h_e)]
        # the cells' h-half weights packed once for the whole unroll (T * repeats uses each)
        from .. import nn as hnn
        cells = [blk.conv for blk in self.body.blocks]
        cin = cells[0].weight.shape[1] - self.body.blocks[0].hidden_dim
        packed_h = None
        hd = self.body.blocks[0].hidden_dim
        if hnn._DEFER is not None and hnn.gboard_conv_ok(h_e[:1, :hd], cells[0].weight, hd, cells[0].padding):
            w_h = torch.cat([c.weight.detach()[:, cin:] for c in cells])
            packed_h = {'layers': [hnn.gboard_pack(c.weight.detach(), hd, cin) for c in cells],
                        'grouped': hnn.gboard_pack(w_h)}
        elif hnn._DEFER is not None and hnn.board_conv_ok(h_e[:1], cells[0].weight, cin, cells[0].padding):
            packed_h = [hnn.board_conv_pack(c.weight.detach(), cin) for c in cells]
        return {'T': T, 'N': N, 'h_e': h_e, 'zx': zx, 'scalar': scalar, 'packed_h': packed_h}

    def sequence_step(self, seq, t, hidden):
        """The cells at step t from the unroll's hidden state: (h_last, hidden)."""
        hs, cs = list(hidden[0]), list(hidden[1])
        return self.body.step_hip([z[t] for z in seq['zx']], hs, cs, self.num_repeats, seq['packed_h'])

    def sequence_end(self, seq, h_lasts):
        """The heads over all T steps: {'policy', 'value', 'return'} with rows (t, n)."""
        T, scalar = seq['T'], seq['scalar']
        h = torch.cat([seq['h_e'], torch.cat(h_lasts)], dim=-3)
        hp, hv, hr = self.head_p_move, self.head_v, self.head_r
        p_move = hp.conv2(self._bn_steps(hp.bn, hp.conv1(h), T)).reshape(-1, hp.outputs)
        policy = torch.cat([p_move, self.head_p_set(scalar[:, :1])], dim=-1)
        v = hv.fc(self._bn_steps(hv.bn, hv.conv(h), T).reshape(-1, hv.hidden_units))
        r = hr.fc(self._bn_steps(hr.bn, hr.conv(h), T).reshape(-1, hr.hidden_units))
        return {'policy': policy, 'value': torch.tanh(v), 'return': r}


class GeisterBatch:
    """E Geister games advanced together on one device (rules of geister.py:170-541).

    State per game: ``board`` (E, 36) int8 piece codes in the reference's
    absolute frame (cell = x*6 + y; -1 empty, piece = colour*2 + type, type 0
    blue / 1 red), ``color`` to move, ``turn_count`` (-2, -1: setting the
    layouts; 200 moves end in a draw), ``win`` (-1 none, 0 black, 1 white,
    2 draw) and the piece counts ``cnt`` (E, 4).  Actions are the reference's
    labels: 0..143 = direction*36 + cell in the mover's frame (white's frame
    is the board rotated 180 degrees, so white's label is 143 minus the
    absolute one), 144 + k = initial layout k of C(8, 4).
    """

    A = 214
    P = 2
    MAX_PLIES = 202
    ALTERNATING = True   # the mover is ply % 2 in every live game (colours alternate, geister.py:389)
    REWARD_STATELESS = True   # reward() does not depend on the state: the generator may read it before step()
    OBS_SHAPE = {'board': (BOARD_PLANES, *BOARD), 'scalar': (SCALARS,)}
    MOVES = 144
    # initial squares of the 8 pieces of each colour (geister.py:179-182); 'B2' = x 1, y 1
    OPOS_NAMES = (('B2', 'C2', 'D2', 'E2', 'B1', 'C1', 'D1', 'E1'), ('E5', 'D5', 'C5', 'B5', 'E6', 'D6', 'C6', 'B6'))
    OPOS = tuple(tuple('ABCDEF'.index(s[0]) * 6 + '123456'.index(s[1]) for s in names) for names in OPOS_NAMES)
    DIRS = ((-1, 0), (0, -1), (0, 1), (1, 0))
    GOALS = (((-1, 5), (6, 5)), ((-1, 0), (6, 0)))
    MAX_MOVES = 200

    def __init__(self, E, device):
        import itertools
        self.E, self.device = E, device
        dev = device
        # target cell of (direction, cell), -1 off the board; off-board goal flags per colour
        tgt = torch.full((4, 36), -1, dtype=torch.long)
        goal = torch.zeros(2, 4, 36, dtype=torch.bool)
        for d, (dx, dy) in enumerate(self.DIRS):
            for x in range(6):
                for y in range(6):
                    nx, ny = x + dx, y + dy
                    if 0 <= nx < 6 and 0 <= ny < 6:
                        tgt[d, x * 6 + y] = nx * 6 + ny
                    else:
                        for c in range(2):
                            goal[c, d, x * 6 + y] = (nx, ny) in self.GOALS[c]
        self.tgt = tgt.to(dev)
        self.tgt_safe = tgt.clamp(min=0).to(dev)
        self.goal = goal.view(2, 144).to(dev)
        # layout k: blue flags of the 8 pieces (geister.py:189, 227-234; OSEQ = combinations(range(8), 4))
        blue = torch.zeros(70, 8, dtype=torch.bool)
        for k, seq in enumerate(itertools.combinations(range(8), 4)):
            blue[k, list(seq)] = True
        self.layout_type = (~blue).to(torch.int8).to(dev)      # piece type per slot: 0 blue, 1 red
        self.opos = torch.tensor(self.OPOS, dtype=torch.long, device=dev)
        self.reset()

    def reset(self):
        """State is allocated once, then reset and advanced in place (a captured ply keeps addressing it)."""
        E, dev = self.E, self.device
        if not hasattr(self, 'board'):
            self.board = torch.full((E, 36), -1, dtype=torch.int8, device=dev)
            self.color = torch.zeros(E, dtype=torch.long, device=dev)
            self.turn_count = torch.full((E,), -2, dtype=torch.long, device=dev)
            self.win = torch.full((E,), -1, dtype=torch.long, device=dev)
            self.cnt = torch.zeros(E, 4, dtype=torch.long, device=dev)
            self.live = torch.ones(E, dtype=torch.bool, device=dev)   # ~terminal(), kept by the HIP step
            self._reward = torch.full((E, 2), -0.01, dtype=torch.float64, device=dev)
        self.live.fill_(True)
        self.board.fill_(-1)
        self.color.zero_()
        self.turn_count.fill_(-2)
        self.win.fill_(-1)
        self.cnt.zero_()
        if getattr(self, 'pidx', None) is not None:
            self.pidx.fill_(-1)

    pidx = None   # (E, 36) piece index (colour*8 + slot) per cell, kept only when piece_order(True) asked for it

    def piece_order(self, on=True):
        """Keep each cell's piece index (the reference's piece numbering, geister.py:227-234, 380-386), so that
        legal_rank() can give the reference's legal-action order; off by default (the rules do not need it)."""
        self.pidx = torch.full((self.E, 36), -1, dtype=torch.long, device=self.device) if on else None

    def legal_rank(self):
        """(E, 214) sort key of every action in the reference's legal_actions order (geister.py:472-486): the
        layouts 144..213 ascending; a move by the mover's piece of slot s in absolute direction d at s*4 + d (the
        pieces by index, each piece's directions in order).  Needs piece_order(True) before reset()."""
        assert self.pidx is not None, 'legal_rank needs piece_order(True)'
        a = torch.arange(self.MOVES, device=self.device).view(1, -1)
        c = self.color.view(-1, 1)
        a_abs = torch.where(c == 1, self.MOVES - 1 - a, a)
        cell = (a_abs % 36).expand(self.E, -1)
        slot = torch.gather(self.pidx, 1, cell) - c * 8
        key = slot.clamp(min=0) * 4 + a_abs // 36
        lay = torch.arange(self.A - self.MOVES, device=self.device).view(1, -1).expand(self.E, -1)
        return torch.cat([key, lay], 1)

    def _track_pieces(self, action, active):
        """pidx through one step (before the rules move the board): a layout puts the mover's pieces 0..7 on
        their initial squares, a move carries the piece's index to its target (off the board: gone)."""
        E, rows, c = self.E, torch.arange(self.E, device=self.device), self.color
        setting = active & (self.turn_count < 0)
        moving = active & (self.turn_count >= 0)
        cells = self.opos[c]
        cur = torch.gather(self.pidx, 1, cells)
        new = c.view(-1, 1) * 8 + torch.arange(8, device=self.device).view(1, -1)
        self.pidx.scatter_(1, cells, torch.where(setting.view(-1, 1), new, cur))
        a_abs = torch.where(c == 1, self.MOVES - 1 - action, action).clamp(0, self.MOVES - 1)
        src, dst = a_abs % 36, self.tgt[a_abs // 36, a_abs % 36]
        piece = self.pidx[rows, src]
        self.pidx[rows, src] = torch.where(moving, torch.full_like(piece, -1), piece)
        on = moving & (dst >= 0)
        dst_s = dst.clamp(min=0)
        self.pidx[rows, dst_s] = torch.where(on, piece, self.pidx[rows, dst_s])

    def turn(self):
        return self.color

    def plies(self):
        return self.turn_count + 2

    def terminal(self):
        return self.win >= 0

    def _hip(self):
        """On a GPU the rules run as csrc/hrl_geister.hip (one launch per call instead of ~30-95 torch ops);
        the torch formulation below is the CPU path and the GPU rules test's twin."""
        return self.board.is_cuda

    def legal(self):
        """(E, 214) bool legal-action mask of the side to move (geister.py:460-487)."""
        if self._hip():
            from .._native import load, check, ptr, stream_of
            out = torch.empty(self.E, self.A, dtype=torch.bool, device=self.device)
            check(load().hrl_geister_legal(ptr(self.board), ptr(self.color), ptr(self.turn_count), self.E, ptr(out),
                                           stream_of(self.board.device)), 'hrl_geister_legal')
            return out
        b = self.board.long()
        own = (b >= 0) & (b // 2 == self.color.view(-1, 1))                     # (E, 36)
        own_blue = own & (b % 2 == 0)
        own_t = torch.gather(own, 1, self.tgt_safe.view(1, -1).expand(self.E, -1)).view(-1, 4, 36)
        on = (self.tgt >= 0).view(1, 4, 36)
        to_goal = own_blue.view(-1, 1, 36) & self.goal[self.color].view(-1, 4, 36)
        moves = own.view(-1, 1, 36) & torch.where(on, ~own_t, to_goal)          # absolute frame (E, 4, 36)
        moves = moves.view(-1, 144)
        moves = torch.where((self.color == 1).view(-1, 1), moves.flip(-1), moves)
        setting = (self.turn_count < 0).view(-1, 1)
        lay = setting.expand(-1, 70)
        return torch.cat([moves & ~setting, lay], dim=1)

    def step(self, action, active):
        """Play `action` (E,) for the side to move in every `active` game (geister.py:359-394)."""
        E, dev = self.E, self.device
        if self.pidx is not None:
            self._track_pieces(action.to(torch.long), active.to(torch.bool))
        if self._hip():
            from .._native import load, check, ptr, stream_of
            assert action.shape == (E,) and active.shape == (E,)
            action = action.to(torch.long).contiguous()
            active = active.to(torch.bool).contiguous()
            check(load().hrl_geister_step(ptr(self.board), ptr(self.color), ptr(self.turn_count), ptr(self.win),
                                          ptr(self.cnt), ptr(action), ptr(active), ptr(self.layout_type),
                                          ptr(self.opos), E, ptr(self.live), stream_of(self.board.device)),
                  'hrl_geister_step')
            return
        rows = torch.arange(E, device=dev)
        c = self.color
        setting = active & (self.turn_count < 0)
        moving = active & (self.turn_count >= 0)
        # -- layout actions: place the mover's 8 pieces
        lay = (action - self.MOVES).clamp(0, 69)
        pieces = (c.view(-1, 1) * 2 + self.layout_type[lay].long())             # (E, 8)
        cells = self.opos[c]                                                   # (E, 8)
        cur = torch.gather(self.board, 1, cells)
        self.board.scatter_(1, cells, torch.where(setting.view(-1, 1), pieces.to(torch.int8), cur))
        add = torch.zeros(E, 4, dtype=torch.long, device=dev)
        add.scatter_(1, torch.stack([c * 2, c * 2 + 1], 1), torch.full((E, 2), 4, dtype=torch.long, device=dev))
        self.cnt += add * setting.long().view(-1, 1)
        # -- moves
        a_abs = torch.where(c == 1, self.MOVES - 1 - action, action).clamp(0, self.MOVES - 1)
        d, src = a_abs // 36, a_abs % 36
        dst = self.tgt[d, src]
        piece = self.board[rows, src].long()
        off = moving & (dst < 0)
        on = moving & (dst >= 0)
        dst_s = dst.clamp(min=0)
        cap = self.board[rows, dst_s].long()
        captured = on & (cap >= 0)
        cnt_dec = torch.zeros(E, 4, dtype=torch.long, device=dev)
        cnt_dec[rows, cap.clamp(min=0)] += captured.long()
        cnt_dec[rows, piece.clamp(min=0)] += off.long()                          # piece leaves by the goal
        self.cnt -= cnt_dec
        gone = captured & (self.cnt[rows, cap.clamp(min=0)] == 0)
        win = torch.where(off, c, self.win)
        win = torch.where(gone, torch.where(cap % 2 == 0, c, 1 - c), win)
        # board: source emptied, piece lands on an on-board target
        src_val = torch.where(moving, torch.full_like(piece, -1), self.board[rows, src].long())
        self.board[rows, src] = src_val.to(torch.int8)
        dst_val = torch.where(on, piece, self.board[rows, dst_s].long())
        self.board[rows, dst_s] = dst_val.to(torch.int8)
        self.color.copy_(torch.where(active, 1 - c, c))
        self.turn_count.add_(active.long())
        draw = moving & (self.turn_count >= self.MAX_MOVES) & (win < 0)
        self.win.copy_(torch.where(draw, torch.full_like(win, 2), win))

    COMPLETE_INFO = False   # CIGeister (ci_geister.py:520-568) shows the opponent's colours in every view

    def observation_record(self, player, rec, t, active):
        """observation(player) on the GPU that also writes slot t (device scalar) of the episode record
        rec = {'board': (E, Tm, 7, 6, 6), 'scalar': (E, Tm, 18)}: the view where `active`, zeros elsewhere --
        DeviceGenerator's obs record in the same launch."""
        from .._native import load, check, ptr, stream_of
        player = player.to(torch.long).contiguous()
        active = active.contiguous()
        assert player.shape == (self.E,) and active.shape == (self.E,) and active.dtype == torch.bool
        Tm = rec['board'].shape[1]
        assert rec['board'].shape == (self.E, Tm, BOARD_PLANES, *BOARD) and rec['board'].is_contiguous()
        assert rec['scalar'].shape == (self.E, Tm, SCALARS) and rec['scalar'].is_contiguous()
        planes = torch.empty(self.E, BOARD_PLANES, *BOARD, device=self.device)
        scalar = torch.empty(self.E, SCALARS, device=self.device)
        check(load().hrl_geister_observation_record(
            ptr(self.board), ptr(self.color), ptr(self.cnt), ptr(player), self.E, int(bool(self.COMPLETE_INFO)),
            ptr(planes), ptr(scalar), ptr(active), ptr(t), Tm, ptr(rec['board']), ptr(rec['scalar']),
            stream_of(self.board.device)), 'hrl_geister_observation_record')
        return {'board': planes, 'scalar': scalar}

    def observation(self, player, full=False):
        """{'board': (E,7,6,6), 'scalar': (E,18)} seen by `player` (E,) (geister.py:495-535, player given);
        ``full``: the reference's ``observation(None)`` view, which also shows the opponent's colours."""
        if self._hip():
            from .._native import load, check, ptr, stream_of
            player = player.to(torch.long).contiguous()
            assert player.shape == (self.E,)
            planes = torch.empty(self.E, BOARD_PLANES, *BOARD, device=self.device)
            scalar = torch.empty(self.E, SCALARS, device=self.device)
            check(load().hrl_geister_observation(ptr(self.board), ptr(self.color), ptr(self.cnt), ptr(player), self.E,
                                                 int(bool(full or self.COMPLETE_INFO)), ptr(planes), ptr(scalar),
                                                 stream_of(self.board.device)), 'hrl_geister_observation')
            return {'board': planes, 'scalar': scalar}
        turn_view = player == self.color
        me = torch.where(turn_view, self.color, 1 - self.color)
        opp = 1 - me
        b = self.board.long()
        cnt = self.cnt
        rows = torch.arange(self.E, device=self.device)
        counts = torch.stack([cnt[rows, me * 2], cnt[rows, me * 2 + 1], cnt[rows, opp * 2], cnt[rows, opp * 2 + 1]], 1)
        onehot = (counts.view(-1, 4, 1) == torch.arange(1, 5, device=self.device).view(1, 1, 4)).view(-1, 16)
        scalar = torch.cat([(me == 0).view(-1, 1), turn_view.view(-1, 1), onehot], 1).float()
        blue_c = b == (me * 2).view(-1, 1)
        red_c = b == (me * 2 + 1).view(-1, 1)
        own_all = blue_c | red_c
        opp_all = (b >= 0) & ~own_all
        if full or self.COMPLETE_INFO:
            blue_o, red_o = b == (opp * 2).view(-1, 1), b == (opp * 2 + 1).view(-1, 1)
        else:
            blue_o = red_o = torch.zeros_like(own_all)
        planes = torch.stack([torch.ones_like(own_all), own_all, opp_all, blue_c, red_c, blue_o, red_o], 1).float()
        planes = torch.where((me == 1).view(-1, 1, 1), planes.flip(-1), planes)   # white: rotate 180 degrees
        return {'board': planes.view(-1, BOARD_PLANES, *BOARD), 'scalar': scalar}

    def reward(self):
        """(E, 2) fp64: -0.01 per ply for both players (geister.py:427-429; a Python float there).  One constant
        tensor (read-only for callers)."""
        return self._reward

    def active(self):
        """(E,) bool games still running: ~terminal(); on the GPU the step kernel keeps it, so the self-play
        ply reads it without a launch (read-only for callers)."""
        return self.live if self._hip() else ~self.terminal()

    def outcome(self):
        """(E, 2): +1/-1 for the winning colour, 0/0 for a draw (geister.py:431-438)."""
        w = torch.where(self.win == 0, 1.0, torch.where(self.win == 1, -1.0, 0.0))
        return torch.stack([w, -w], dim=1)


class _OneGame:
    """One game's state in plain Python for the host plugin env: GeisterBatch's rules (same state fields, same
    operations) with E = 1 and no tensor ops.  A one-game GeisterBatch on the CPU paid ~150 torch launches per
    ply (≈1.3 ms); this is ≈20-40 µs, so a host Environment steps about as fast as the reference's pure-Python
    one (geister.py:359-394, 460-535).  tests/test_geister_rules.py replays the reference games through it."""

    TGT = None          # TGT[d][cell]: target cell of absolute direction d, -1 off the board
    GOAL = None         # GOAL[c][d][cell]: leaving the board that way is colour c's goal
    LAYOUT = None       # LAYOUT[k][slot]: piece type (0 blue, 1 red) of layout k

    @classmethod
    def _tables(cls):
        import itertools
        if cls.TGT is not None:
            return
        tgt = [[-1] * 36 for _ in range(4)]
        goal = [[[False] * 36 for _ in range(4)] for _ in range(2)]
        for d, (dx, dy) in enumerate(GeisterBatch.DIRS):
            for x in range(6):
                for y in range(6):
                    nx, ny = x + dx, y + dy
                    if 0 <= nx < 6 and 0 <= ny < 6:
                        tgt[d][x * 6 + y] = nx * 6 + ny
                    else:
                        for c in range(2):
                            goal[c][d][x * 6 + y] = (nx, ny) in GeisterBatch.GOALS[c]
        lay = []
        for seq in itertools.combinations(range(8), 4):
            lay.append([0 if i in seq else 1 for i in range(8)])
        cls.TGT, cls.GOAL, cls.LAYOUT = tgt, goal, lay

    def __init__(self, complete_info=False):
        self._tables()
        self.complete_info = complete_info
        self.reset()

    def reset(self):
        self.board = [-1] * 36
        self.color = 0
        self.turn_count = -2
        self.win = -1
        self.cnt = [0, 0, 0, 0]

    def move_legal(self, d, cell):
        """Absolute move (direction d, cell) of the side to move: GeisterBatch.legal's per-move test."""
        dst = self.TGT[d][cell]
        if dst >= 0:
            t = self.board[dst]
            return t < 0 or t // 2 != self.color
        return self.board[cell] % 2 == 0 and self.GOAL[self.color][d][cell]

    def step(self, action):
        """GeisterBatch.step for one active game."""
        c = self.color
        if self.turn_count < 0:                                  # a layout: the mover's 8 pieces
            types = self.LAYOUT[action - GeisterBatch.MOVES]
            for cell, t in zip(GeisterBatch.OPOS[c], types):
                self.board[cell] = c * 2 + t
            self.cnt[c * 2] += 4
            self.cnt[c * 2 + 1] += 4
        else:
            a = GeisterBatch.MOVES - 1 - action if c == 1 else action
            d, src = divmod(a, 36)
            dst = self.TGT[d][src]
            piece = self.board[src]
            if dst < 0:                                          # leaves by the goal
                self.cnt[piece] -= 1
                self.win = c
            else:
                cap = self.board[dst]
                if cap >= 0:
                    self.cnt[cap] -= 1
                    if self.cnt[cap] == 0:
                        self.win = c if cap % 2 == 0 else 1 - c
                self.board[dst] = piece
            self.board[src] = -1
        moving = self.turn_count >= 0
        self.color = 1 - c
        self.turn_count += 1
        if moving and self.turn_count >= GeisterBatch.MAX_MOVES and self.win < 0:
            self.win = 2

    def observation(self, player, full=False):
        """GeisterBatch.observation for one game: {'board': (7, 6, 6), 'scalar': (18,)} float32."""
        me, opp = player, 1 - player
        cnt = self.cnt
        scalar = np.zeros(SCALARS, dtype=np.float32)
        scalar[0] = me == 0
        scalar[1] = player == self.color
        for i, n in enumerate((cnt[me * 2], cnt[me * 2 + 1], cnt[opp * 2], cnt[opp * 2 + 1])):
            if 1 <= n <= 4:
                scalar[2 + 4 * i + n - 1] = 1
        b = np.array(self.board, dtype=np.int8)
        if me == 1:
            b = b[::-1]                                          # white: the board rotated 180 degrees
        planes = np.empty((BOARD_PLANES, 36), dtype=np.float32)
        planes[0] = 1
        blue_c, red_c = b == me * 2, b == me * 2 + 1
        own = blue_c | red_c
        planes[1] = own
        planes[2] = (b >= 0) & ~own
        planes[3] = blue_c
        planes[4] = red_c
        if full or self.complete_info:
            planes[5] = b == opp * 2
            planes[6] = b == opp * 2 + 1
        else:
            planes[5:] = 0
        return {'board': planes.reshape(BOARD_PLANES, *BOARD), 'scalar': scalar}


class Environment(BaseEnvironment):
    """One Geister game behind the reference plugin API (geister.py:170-541).

    The state is a ``_OneGame`` (GeisterBatch's rules in plain Python: the tensor rules the device self-play
    runs, restated for one game; pinned to the reference env by tests/test_geister_rules.py).  Actions and
    observations are the reference's: 214 labels, ``{'board': (7, 6, 6), 'scalar': (18,)}`` numpy arrays;
    ``observation(None)`` is the turn player's view with the opponent's colours shown, ``observation(p)``
    hides them.
    """

    BATCH = GeisterBatch
    X, Y = 'ABCDEF', '123456'

    def __init__(self, args=None):
        super().__init__(args)
        self.game = _OneGame(self.BATCH.COMPLETE_INFO)
        self.reset()

    def reset(self, args=None):
        self.game.reset()
        self.record = []
        # piece identities (geister.py:202-227: board_index / piece_position): the reference lists legal
        # moves piece by piece in this order, and seeded samplers draw over that list (generation.py:53)
        self._where = [-1] * 16         # piece index (colour * 8 + initial slot) -> cell x*6+y, -1 off board
        self._who = [-1] * 36           # cell -> piece index
        self._layouts_set = 0

    def __str__(self):
        marks = {-1: '_', 0: 'B', 1: 'R', 2: 'b', 3: 'r'}
        b = self.game.board
        rows = ['  ' + ' '.join(self.Y)] + [self.X[i] + ' ' + ' '.join(marks[v] for v in b[i * 6:(i + 1) * 6])
                                           for i in range(6)]
        return '\n'.join(rows) + '\ncolor = ' + 'BW'[self.turn()] + '\nrecord = ' + ' '.join(
            self.action2str(a, i % 2) for i, a in enumerate(self.record))

    def play(self, action, _=None):
        action = int(action)
        self._track(action, self.turn())
        self.game.step(action)
        if action < GeisterBatch.MOVES:
            self.record.append(action)

    def _track(self, action, c):
        """Follow the pieces' identities through a move (geister.py:208-236, 359-393)."""
        if action >= GeisterBatch.MOVES:                       # a layout: pieces c*8 .. c*8+7 placed
            for idx, cell in enumerate(GeisterBatch.OPOS[c]):
                self._where[c * 8 + idx] = cell
                self._who[cell] = c * 8 + idx
            return
        d, x, y = action // 36, (action % 36) // 6, action % 6
        if c == 1:
            d, x, y = 3 - d, 5 - x, 5 - y
        dx, dy = GeisterBatch.DIRS[d]
        src, nx, ny = x * 6 + y, x + dx, y + dy
        piece = self._who[src]
        self._who[src] = -1
        if not (0 <= nx < 6 and 0 <= ny < 6):                 # off the board through a goal
            self._where[piece] = -1
            return
        dst = nx * 6 + ny
        if self._who[dst] >= 0:                                # capture
            self._where[self._who[dst]] = -1
        self._who[dst] = piece
        self._where[piece] = dst

    def turn(self):
        return self.game.color

    def terminal(self):
        return self.game.win >= 0

    def reward(self):
        return {p: -0.01 for p in self.players()}

    def outcome(self):
        w = self.game.win
        v = 1.0 if w == 0 else (-1.0 if w == 1 else 0.0)       # GeisterBatch.outcome
        return {0: v, 1: -v}

    def legal_actions(self, _=None):
        """In the reference's order (geister.py:472-486): layouts 144..213 before the game, then the mover's
        pieces by index, each piece's directions 0..3 (absolute; white's labels in its rotated frame)."""
        g = self.game
        if g.turn_count < 0:
            return list(range(GeisterBatch.MOVES, ACTIONS))
        c = g.color
        out = []
        for cell in self._where[c * 8:(c + 1) * 8]:
            if cell < 0:
                continue
            for d in range(4):
                if g.move_legal(d, cell):
                    out.append((3 - d) * 36 + 35 - cell if c == 1 else d * 36 + cell)
        return out

    def action_length(self):
        return ACTIONS

    def players(self):
        return [0, 1]

    def observation(self, player=None):
        who = self.turn() if player is None else player
        obs = self.game.observation(who, full=player is None)
        return {'scalar': obs['scalar'], 'board': obs['board']}

    def net(self):
        return GeisterNet

    # -- move notation (geister.py:263-330): 'B2C2' from/to in absolute squares, '**' = off the board by
    # a goal, 's<k>' = initial layout k; white's labels are in its 180-degree rotated frame
    def _square(self, x, y):
        return self.X[x] + self.Y[y] if 0 <= x < 6 and 0 <= y < 6 else '**'

    def action2str(self, a, player):
        a = int(a)
        if a >= GeisterBatch.MOVES:
            return 's' + str(a - GeisterBatch.MOVES)
        d, x, y = a // 36, (a % 36) // 6, a % 6
        if player == 1:
            d, x, y = 3 - d, 5 - x, 5 - y
        dx, dy = GeisterBatch.DIRS[d]
        return self._square(x, y) + self._square(x + dx, y + dy)

    def str2action(self, s, player):
        if s[0] == 's':
            return GeisterBatch.MOVES + int(s[1:])
        x, y = self.X.index(s[0]), self.Y.index(s[1])
        if s[2:] == '**':
            d = next(d for d, (dx, dy) in enumerate(GeisterBatch.DIRS) if (x + dx, y + dy) in GeisterBatch.GOALS[player])
        else:
            tx, ty = self.X.index(s[2]), self.Y.index(s[3])
            d = GeisterBatch.DIRS.index((tx - x, ty - y))
        if player == 1:
            d, x, y = 3 - d, 5 - x, 5 - y
        return d * 36 + x * 6 + y
