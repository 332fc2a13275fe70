"""Config-driven learner entry (handyrl_amd.main; the reference's main.py --train + config.yaml)."""

import os

import pytest
import torch

from handyrl_amd.main import load_config, train_main, main

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _oracle_loss(outputs, batch, args):
    from oracle.learner import loss_from_outputs
    losses, dcnt = loss_from_outputs(outputs, batch, args)
    return losses, torch.tensor(dcnt)


def _small(env='TicTacToe'):
    args = load_config(os.path.join(ROOT, 'config.yaml'))
    args['env_args']['env'] = env
    args['train_args'].update(update_episodes=16, minimum_episodes=32, maximum_episodes=64, batch_size=8,
                              forward_steps=6, epochs=2)
    return args


def test_repo_config_has_reference_keys():
    args = load_config(os.path.join(ROOT, 'config.yaml'))
    for k in ('turn_based_training', 'observation', 'gamma', 'forward_steps', 'compress_steps',
              'entropy_regularization', 'entropy_regularization_decay', 'update_episodes', 'batch_size',
              'minimum_episodes', 'maximum_episodes', 'epochs', 'lambda', 'policy_target', 'value_target',
              'seed', 'restart_epoch'):
        assert k in args['train_args'], k
    assert args['env_args']['env'] == 'TicTacToe'


def test_usage_without_mode():
    assert main([]) == 1


@pytest.mark.parametrize('env', ['TicTacToe', 'Geister'])
def test_train_main_cpu_two_epochs(tmp_path, env):
    """The whole cycle on the CPU (oracle loss; the HIP loss needs a GPU): self-play, replay, two Trainer
    epochs, models/<epoch>.pth written and loadable into env.net(); restart_epoch resumes from it."""
    args = _small(env)
    if env == 'Geister':
        args['train_args'].update(update_episodes=4, minimum_episodes=4, batch_size=2, forward_steps=4, epochs=1)
    logs = []
    model = train_main(args, device=torch.device('cpu'), loss_fn=_oracle_loss, model_dir=str(tmp_path),
                       log=logs.append)
    epochs = args['train_args']['epochs']
    assert len(logs) == epochs
    saved = torch.load(os.path.join(tmp_path, '%d.pth' % epochs), weights_only=True)
    assert set(saved) == set(model.state_dict())
    args['train_args'].update(restart_epoch=epochs, epochs=1)
    train_main(args, device=torch.device('cpu'), loss_fn=_oracle_loss, model_dir=str(tmp_path), log=logs.append)
    assert os.path.exists(os.path.join(tmp_path, '%d.pth' % (epochs + 1)))


@pytest.mark.gpu
def test_train_main_gpu(tmp_path, cuda):
    args = _small()
    model = train_main(args, device=cuda, model_dir=str(tmp_path), log=lambda *_: None)
    assert os.path.exists(os.path.join(tmp_path, '2.pth'))
    assert not next(model.parameters()).is_cuda
