"""Pin the CPU learner oracle (oracle/learner.py) and the TicTacToe net to the reference.

* compute_loss on the reference's own make_batch batches with fixed network
  outputs: every loss term, dcnt, the composed advantages and the gradients
  w.r.t. the outputs (tests/golden/loss.*);
* three full learner steps of the TicTacToe SimpleConv2dModel, starting from
  the reference's initial state_dict loaded into handyrl_amd's net
  (tests/golden/learner.*): per-step losses, grad norm and final weights.
Also checks handyrl_amd.train.forward_prediction (pure torch) against it.
"""

import numpy as np
import torch
import torch.nn as nn

from oracle import learner as ol

BATCH_KEYS = ('policy', 'value', 'action', 'outcome', 'reward', 'return', 'episode_mask', 'turn_mask',
              'observation_mask', 'action_mask', 'progress')


class FixedOutputs(nn.Module):
    def __init__(self, p, v, r=None):
        super().__init__()
        self.p = nn.Parameter(torch.from_numpy(p.copy()))
        self.v = nn.Parameter(torch.from_numpy(v.copy()))
        self.r = None if r is None else nn.Parameter(torch.from_numpy(r.copy()))

    def forward(self, x, hidden=None):
        out = {'policy': self.p, 'value': self.v}
        if self.r is not None:
            out['return'] = self.r
        return out


def loss_case(arrays, c):
    pre = '%d:' % c['id']
    batch = {k: torch.from_numpy(arrays[pre + 'batch.' + k].copy()) for k in BATCH_KEYS}
    B, T, Pp = c['B'], c['T'], c['Pp']
    batch['observation'] = torch.zeros(B, T, Pp, 1)
    net = FixedOutputs(arrays[pre + 'out.policy'], arrays[pre + 'out.value'],
                       arrays[pre + 'out.return'] if c['has_return'] else None)
    return batch, net


def test_loss_golden(golden_loss):
    meta, arrays = golden_loss
    for c in meta:
        batch, net = loss_case(arrays, c)
        rec = {}
        outputs = ol.forward_prediction(net, None, batch, c['args'])
        losses, dcnt = ol.loss_from_outputs(outputs, batch, c['args'], record=rec)
        assert dcnt == c['dcnt']
        for k, v in c['losses'].items():
            assert abs(losses[k].item() - v) <= 1e-5 * max(1.0, abs(v)), (c['name'], k, losses[k].item(), v)
        pre = '%d:' % c['id']
        np.testing.assert_allclose(rec['total_adv'].numpy(), arrays[pre + 'total_adv'], rtol=0, atol=1e-6)
        np.testing.assert_allclose(rec['log_sel'].numpy(), arrays[pre + 'log_sel'], rtol=0, atol=1e-6)
        losses['total'].backward()
        np.testing.assert_allclose(net.p.grad.numpy(), arrays[pre + 'grad.policy'], rtol=1e-5, atol=1e-6)
        np.testing.assert_allclose(net.v.grad.numpy(), arrays[pre + 'grad.value'], rtol=1e-5, atol=1e-6)
        if c['has_return']:
            np.testing.assert_allclose(net.r.grad.numpy(), arrays[pre + 'grad.return'], rtol=1e-5, atol=1e-6)


def test_product_forward_prediction_matches_oracle(golden_loss):
    """handyrl_amd.train.forward_prediction is plain torch: check it on the CPU."""
    from handyrl_amd.train import forward_prediction
    meta, arrays = golden_loss
    for c in meta:
        batch, net = loss_case(arrays, c)
        a = forward_prediction(net, None, batch, c['args'])
        b = ol.forward_prediction(net, None, batch, c['args'])
        assert set(a) == set(b)
        for k in a:
            assert torch.equal(a[k], b[k]), k


def learner_setup(golden_learner):
    from handyrl_amd.envs.tictactoe import SimpleConv2dModel
    meta, arrays = golden_learner
    net = SimpleConv2dModel()
    sd = {k: torch.from_numpy(arrays['init.' + k].copy()) for k in meta['state_names']}
    net.load_state_dict(sd, strict=True)
    batch = {k[len('batch.'):]: torch.from_numpy(arrays[k].copy()) for k in arrays.files if k.startswith('batch.')}
    return meta, arrays, net, batch


def test_tictactoe_net_matches_reference_state_dict(golden_learner):
    meta, arrays, net, _ = learner_setup(golden_learner)
    assert sum(p.numel() for p in net.parameters()) == 29006
    assert list(net.state_dict().keys()) == meta['state_names']


def test_learner_steps_golden(golden_learner):
    meta, arrays, net, batch = learner_setup(golden_learner)
    torch.set_num_threads(1)
    learner = ol.CpuLearner(net, meta['args'], lr=meta['lr'])
    for s, ref in enumerate(meta['steps']):
        out = learner.step(batch)
        for k in ('p', 'v', 'ent', 'total', 'grad_norm'):
            assert abs(out[k] - ref[k]) <= 1e-5 * max(1.0, abs(ref[k])), (s, k, out[k], ref[k])
        assert out['dcnt'] == ref['dcnt']
    for k, v in net.state_dict().items():
        np.testing.assert_allclose(v.numpy(), arrays['final.' + k], rtol=1e-5, atol=1e-6, err_msg=k)
