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


@pytest.mark.parametrize('env,obs,tbt', [('ParallelTicTacToe', False, True), ('ParallelTicTacToe', True, True),
                                          ('TicTacToe', True, True), ('TicTacToe', False, False),
                                          ('tests.plugin_env', True, True), ('tests.plugin_env', False, False)])
def test_train_main_host_generator_cpu(tmp_path, env, obs, tbt):
    """Envs without a batched twin, or with observation / solo training, train through the plugin API: the
    host generator plays them (generation.py semantics) into the moment replay; the learner trains on the
    make_batch layout of the mode (oracle loss on the CPU)."""
    args = _small(env)
    args['train_args'].update(observation=obs, turn_based_training=tbt, epochs=2, generator='host')
    logs = []
    model = train_main(args, device=torch.device('cpu'), loss_fn=_oracle_loss, model_dir=str(tmp_path),
                       log=logs.append)
    assert len(logs) == 2
    saved = torch.load(os.path.join(tmp_path, '2.pth'), weights_only=True)
    assert set(saved) == set(model.state_dict())
    for v in saved.values():
        assert torch.isfinite(v.float()).all()


@pytest.mark.parametrize('env,obs,tbt', [('ParallelTicTacToe', False, True), ('ParallelTicTacToe', True, True),
                                          ('TicTacToe', True, True), ('TicTacToe', False, False),
                                          ('Geister', True, True)])
def test_train_main_device_player_modes_cpu(tmp_path, env, obs, tbt):
    """Batched envs with observation, solo training or simultaneous moves are played by the device generator's
    per-player ply into the PlayerReplay (no host env in the loop); two epochs train on its batches."""
    import handyrl_amd.main as hm
    args = _small(env)
    args['train_args'].update(observation=obs, turn_based_training=tbt, epochs=2)
    if env == 'Geister':
        args['train_args'].update(update_episodes=4, minimum_episodes=4, batch_size=2, forward_steps=4, epochs=1)
    built = []
    real = hm.PlayerReplay

    def spy(*a, **k):
        built.append(k)
        return real(*a, **k)
    hm.PlayerReplay = spy
    try:
        model = train_main(args, device=torch.device('cpu'), loss_fn=_oracle_loss, model_dir=str(tmp_path),
                           log=lambda *_: None)
    finally:
        hm.PlayerReplay = real
    assert built and built[0]['solo'] == (not tbt) and built[0]['mover'] == (tbt and not obs)
    for v in model.state_dict().values():
        assert torch.isfinite(v.float()).all()


def test_main_cli_trains_a_plugin_module(tmp_path, monkeypatch):
    """``python -m handyrl_amd.main --train config.yaml`` with a plugin named by module path."""
    import yaml
    cfg = _small('tests.plugin_env')
    cfg['train_args'].update(observation=True, epochs=1)
    path = tmp_path / 'config.yaml'
    path.write_text(yaml.safe_dump(cfg))
    calls = []
    import handyrl_amd.main as hm
    real = hm.train_main

    def cpu_train_main(args):
        calls.append(args)
        return real(args, device=torch.device('cpu'), loss_fn=_oracle_loss, model_dir=str(tmp_path / 'models'),
                    log=lambda *_: None)
    monkeypatch.setattr(hm, 'train_main', cpu_train_main)
    assert hm.main(['--train', str(path)]) == 0
    assert calls and calls[0]['env_args']['env'] == 'tests.plugin_env'
    assert os.path.exists(tmp_path / 'models' / '1.pth')


def _rank_main(rank, world, port, tmp, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR='127.0.0.1',
                      MASTER_PORT=str(port))
    import torch.distributed as dist
    torch.set_num_threads(1)
    try:
        args = _small('Geister')
        # Geister games run 2-202 plies: the ranks' own episode lengths differ, the step count must not
        args['train_args'].update(update_episodes=4, minimum_episodes=4, batch_size=2, forward_steps=4, epochs=2,
                                  generator='host')
        import handyrl_amd.trainer as ht
        counts = []
        real = ht.Trainer.train

        def counting(self, max_steps=None):
            counts.append(max_steps)
            return real(self, max_steps=max_steps)
        ht.Trainer.train = counting
        train_main(args, device=torch.device('cpu'), loss_fn=_oracle_loss, model_dir=tmp, log=lambda *_: None)
        q.put((rank, counts))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def test_train_main_two_ranks_agree_on_steps(tmp_path):
    """Under torchrun every rank derives the epoch's step count from ALL ranks' new env-steps, so the
    gradient all-reduces pair up even when the ranks' episodes differ in length (2 gloo ranks)."""
    import socket
    import torch.multiprocessing as mp
    with socket.socket() as sk:
        sk.bind(('127.0.0.1', 0))
        port = sk.getsockname()[1]
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    procs = [ctx.Process(target=_rank_main, args=(r, 2, port, str(tmp_path), q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=600) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[0] == res[1] and len(res[0]) == 2


@pytest.mark.gpu
@pytest.mark.parametrize('env,obs', [('ParallelTicTacToe', True), ('tests.plugin_env', True), ('Geister', True)])
def test_train_main_host_generator_gpu(tmp_path, cuda, env, obs):
    """The host generator path on the GPU: batched HIP / torch inference per ply, HIP learner step."""
    args = _small(env)
    args['train_args'].update(observation=obs, generator='host')
    if env == 'Geister':
        args['train_args'].update(update_episodes=8, minimum_episodes=8, batch_size=4, forward_steps=8, epochs=1)
    model = train_main(args, device=cuda, model_dir=str(tmp_path), log=lambda *_: None)
    assert os.path.exists(tmp_path / ('%d.pth' % args['train_args']['epochs']))
    for v in model.state_dict().values():
        assert torch.isfinite(v.float()).all()


@pytest.mark.gpu
@pytest.mark.parametrize('env,obs,tbt', [('ParallelTicTacToe', False, True), ('TicTacToe', True, True),
                                          ('Geister', True, True)])
def test_train_main_device_player_modes_gpu(tmp_path, cuda, env, obs, tbt):
    """The per-player device generator (captured ply graph) and PlayerReplay feeding the HIP learner step."""
    args = _small(env)
    args['train_args'].update(observation=obs, turn_based_training=tbt)
    if env == 'Geister':
        args['train_args'].update(update_episodes=8, minimum_episodes=8, batch_size=4, forward_steps=8, epochs=1)
    model = train_main(args, device=cuda, model_dir=str(tmp_path), log=lambda *_: None)
    assert os.path.exists(tmp_path / ('%d.pth' % args['train_args']['epochs']))
    for v in model.state_dict().values():
        assert torch.isfinite(v.float()).all()


@pytest.mark.gpu
def test_train_main_gpu(tmp_path, cuda):
    args = _small()
    model = train_main(args, device=cuda, model_dir=str(tmp_path), log=lambda *_: None)
    assert os.path.exists(os.path.join(tmp_path, '2.pth'))
    assert not next(model.parameters()).is_cuda
