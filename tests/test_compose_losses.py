"""Public compose_losses keeps the reference's return types (train.py:188-215): dcnt is a Python float
(tmasks.sum().item(), train.py:199) and the losses equal the CPU oracle's restatement on the same inputs."""

import torch

from handyrl_amd.train import compose_losses
from oracle import learner as ol


def test_compose_losses_matches_oracle_and_returns_float_dcnt():
    g = torch.Generator().manual_seed(0)
    B, T, P, A = 4, 5, 2, 9
    outputs = {'policy': torch.randn(B, T, 1, A, generator=g), 'value': torch.tanh(torch.randn(B, T, P, 1, generator=g))}
    log_sel = torch.randn(B, T, 1, 1, generator=g)
    total_adv = torch.randn(B, T, P, 1, generator=g)
    targets = {'value': torch.randn(B, T, P, 1, generator=g)}
    turn = torch.arange(T) % 2
    batch = {'turn_mask': torch.stack([1 - turn, turn], -1).float().view(1, T, P, 1).expand(B, T, P, 1),
             'observation_mask': torch.ones(B, T, P, 1), 'progress': torch.rand(B, T, 1, generator=g)}
    args = {'entropy_regularization': 0.1, 'entropy_regularization_decay': 0.3}
    losses, dcnt = compose_losses(outputs, log_sel, total_adv, targets, batch, args)
    ref, ref_dcnt = ol.compose_losses(outputs, log_sel, total_adv, targets, batch, args)
    assert isinstance(dcnt, float) and dcnt == float(ref_dcnt) == B * T
    for k in ref:
        torch.testing.assert_close(losses[k], ref[k], rtol=1e-6, atol=1e-6)
