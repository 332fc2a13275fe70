"""Recurrent branch of forward_prediction (train.py:155-174) vs the oracle.

A small recurrent net with a nested (list-of-tuple) hidden state, like
GeisterNet's DRC ConvLSTM (geister.py:66-98, init_hidden :148-149), in the
three training configurations the reference distinguishes: turn-based without
opponent observation (hidden summed over players), turn-based with
observation, and solo.  forward_prediction is plain torch, so this runs on the
CPU; the GPU test runs the whole compute_loss.
"""

import pytest
import torch
import torch.nn as nn

from oracle import learner as ol


class TinyRecurrent(nn.Module):
    def __init__(self, A=9, H=6):
        super().__init__()
        self.H = H
        self.inp = nn.Linear(27, 2 * H)
        self.rec = nn.Linear(H, 2 * H)
        self.head_p = nn.Linear(H, A)
        self.head_v = nn.Linear(H, 1)
        self.head_r = nn.Linear(H, 1)

    def init_hidden(self, batch_size=None):
        shape = (self.H,) if batch_size is None else (*batch_size, self.H)
        return [(torch.zeros(shape), torch.zeros(shape))]

    def forward(self, x, hidden):
        h, c = hidden[0]
        g = self.inp(x.flatten(1)) + self.rec(h)
        i, f = g.chunk(2, -1)
        c = torch.sigmoid(f) * c + torch.tanh(i)
        h = torch.tanh(c)
        return {'policy': self.head_p(h), 'value': torch.tanh(self.head_v(h)), 'return': self.head_r(h),
                'hidden': [(h, c)]}


def _batch(tbt, obs, B=5, T=7, seed=0):
    from handyrl_amd.synthetic import tictactoe_batch, default_args
    batch = tictactoe_batch(B, T, torch.device('cpu'), seed=seed)
    args = default_args(T, B)
    args.update(turn_based_training=tbt, observation=obs)
    if obs or not tbt:   # policy-side tensors carry every player (Pp = P) in these modes
        P = 2 if obs else 1
        for k in ('observation', 'policy', 'action', 'action_mask'):
            batch[k] = batch[k].expand(-1, -1, P, *batch[k].shape[3:]).contiguous()
        if not tbt:
            for k in ('value', 'reward', 'return', 'turn_mask', 'observation_mask', 'outcome'):
                batch[k] = batch[k][:, :, :1].contiguous()
            batch['turn_mask'] = batch['episode_mask'].clone()
            batch['observation_mask'] = batch['episode_mask'].clone()
    batch['reward'] = torch.randn_like(batch['reward']) * 0.01
    batch['return'] = torch.randn_like(batch['return'])
    return batch, args


@pytest.mark.parametrize('tbt,obs', [(True, False), (True, True), (False, False)])
def test_recurrent_forward_prediction_matches_oracle(tbt, obs):
    from handyrl_amd.train import forward_prediction
    batch, args = _batch(tbt, obs)
    torch.manual_seed(1)
    net = TinyRecurrent()
    B, P = batch['value'].size(0), batch['value'].size(2)
    a = forward_prediction(net, net.init_hidden([B, P]), batch, args)
    b = ol.forward_prediction(net, net.init_hidden([B, P]), batch, args)
    assert set(a) == set(b) == {'policy', 'value', 'return'}
    for k in a:
        assert torch.equal(a[k], b[k]), k


@pytest.mark.gpu
@pytest.mark.parametrize('tbt,obs', [(True, False), (True, True), (False, False)])
def test_recurrent_compute_loss_gpu(cuda, tbt, obs):
    from handyrl_amd.train import compute_loss
    batch, args = _batch(tbt, obs, B=64, T=12, seed=3)
    torch.manual_seed(2)
    net_cpu = TinyRecurrent()
    net_gpu = TinyRecurrent()
    net_gpu.load_state_dict(net_cpu.state_dict())
    net_gpu = net_gpu.to(cuda)
    B, P = batch['value'].size(0), batch['value'].size(2)
    ref, ref_dcnt = ol.compute_loss(batch, net_cpu, net_cpu.init_hidden([B, P]), args)
    hid = [(h.to(cuda), c.to(cuda)) for h, c in net_gpu.init_hidden([B, P])]
    out, dcnt = compute_loss({k: v.to(cuda) for k, v in batch.items()}, net_gpu, hid, args)
    assert dcnt == ref_dcnt
    for k in ref:
        a, b = out[k].item(), ref[k].item()
        assert abs(a - b) <= 1e-5 * max(1.0, abs(b)), (k, a, b)
    ref['total'].backward()
    out['total'].backward()
    for (n, p), q in zip(net_cpu.named_parameters(), net_gpu.parameters()):
        assert torch.allclose(q.grad.cpu(), p.grad, rtol=1e-4, atol=1e-5), n
