"""Trainer epochs vs the reference Trainer.train (handyrl/train.py:312-401).

tests/golden/trainer.* holds two reference epochs (2 and 3 batches) over fixed
TicTacToe make_batch batches: after each epoch the lr and data_cnt_ema of the
epoch-end schedule (train.py:396-398: EMA of the per-batch data count, lr =
3e-8 * ema / (1 + steps * 1e-5)), and the final weights.  handyrl_amd's
Trainer runs the same epochs from the same seeded net: on the CPU with the
oracle's loss (the HIP loss needs a GPU), and on the GPU with the product
path.  The schedule values are float64 host arithmetic over the dcnt sums:
equal to 1e-12.
"""

import numpy as np
import pytest
import torch

from tests.conftest import load_golden


@pytest.fixture(scope='module')
def golden():
    return load_golden('trainer')


def _batches(arrays, device):
    out = []
    i = 0
    while ('batch%d.value' % i) in arrays.files:
        pre = 'batch%d.' % i
        out.append({k[len(pre):]: torch.from_numpy(arrays[k]).to(device) for k in arrays.files if k.startswith(pre)})
        i += 1
    return out


def _run(golden, device, loss_fn=None, graph=False):
    from handyrl_amd.envs.tictactoe import SimpleConv2dModel
    from handyrl_amd.trainer import Trainer
    meta, arrays = golden
    batches = _batches(arrays, device)
    torch.manual_seed(meta['seed'])
    net = SimpleConv2dModel()
    tr = None

    class ListBatcher:
        def __init__(self, items):
            self.items = list(items)

        def batch(self):
            b = self.items.pop(0)
            if not self.items:
                tr.update_flag = True
            return b
    tr = Trainer(dict(meta['args']), net, None, device=device, graph=graph, loss_fn=loss_fn)
    for ep in meta['epochs']:
        lo, hi = ep['batches']
        tr.update_flag = False
        tr.batcher = ListBatcher(batches[lo:hi])
        model = tr.train()
        assert not next(model.parameters()).is_cuda and not model.training
        assert tr.steps == ep['steps']
        assert tr.data_cnt_ema == pytest.approx(ep['data_cnt_ema'], rel=1e-12)
        assert tr.lr == pytest.approx(ep['lr'], rel=1e-12)
        assert tr.learner.current_lr() == pytest.approx(ep['lr'], rel=1e-6)
    state = tr.model.state_dict()
    for k in arrays.files:
        if k.startswith('final.'):
            n = k[len('final.'):]
            torch.testing.assert_close(state[n].detach().cpu(), torch.from_numpy(arrays[k]), rtol=1e-5, atol=1e-6,
                                       msg=n)


def test_trainer_epochs_cpu_oracle_loss(golden):
    def oracle_loss(outputs, batch, args):
        from oracle.learner import loss_from_outputs
        losses, dcnt = loss_from_outputs(outputs, batch, args)
        return losses, torch.tensor(dcnt)
    _run(golden, torch.device('cpu'), loss_fn=oracle_loss)


@pytest.mark.gpu
@pytest.mark.parametrize('graph', [False, True])
def test_trainer_epochs_gpu(golden, cuda, graph):
    _run(golden, cuda, graph=graph)
