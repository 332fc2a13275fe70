"""Config-driven learner entry point: the reference's ``main.py --train`` on one GPU node.

    python -m handyrl_amd.main --train [config.yaml]
    python -m torch.distributed.run --nproc-per-node N -m handyrl_amd.main --train [config.yaml]

Reads the reference's ``config.yaml`` (main.py:13-15; config.yaml:1-35;
docs/parameters.md) -- ``env_args`` and ``train_args`` -- and runs the
reference's training cycle (train.py:425-560: workers generate episodes,
the trainer steps on recency-weighted windows, every ``update_episodes``
episodes an epoch ends, the lr is rescheduled and ``models/<epoch>.pth`` is
written) with the actors and the learner on the GPU:

* ``prepare_env`` / ``make_env`` resolve the env by name or module path
  (environment.py:18-39) and ``env.net()`` gives the model class;
* generation: an env module with a batched (device) twin (TicTacToe,
  ParallelTicTacToe, Geister, CIGeister) is played by
  ``rollout.DeviceGenerator``: in the stock layout of an alternating env
  (turn_based_training, no opponent observation) the mover-only ply into
  ``rollout.DeviceReplay``; with ``observation: True``, solo training or a
  simultaneous-move env the per-player ply (every player's view, records
  with a player axis) into ``rollout.PlayerReplay``.  ANY other env -- a
  user's module, the reference's own plugins named by module path -- is
  played through the plugin API by ``hostgen.HostBatchGenerator`` (host
  envs, one batched GPU forward per ply, generation.py's semantics) into
  ``hostgen.MomentReplay``; ``generator: host`` in train_args forces that
  path for every env;
* ``update_episodes`` games per epoch with the current weights (the
  reference's workers hold the latest published model), recency-weighted
  replay of ``maximum_episodes``; training starts once ``minimum_episodes``
  are stored.  The three counts are global, as in the reference: under
  torchrun each rank generates and keeps 1/world of them;
* ``trainer.Trainer`` runs the epoch (its lr / data-count EMA schedule is the
  reference's, train.py:394-401) for ``steps_per_epoch`` steps (default: the
  epoch's new env-steps of ALL ranks over the global batch world*B*T, at
  least 1 -- every rank runs the same count, so their collectives pair up);
* data parallel under torchrun: every rank generates and trains its own
  shard, the gradients are SUMmed over RCCL (distributed.py), rank 0 saves.

The worker/server network plane, evaluation servers and the other CLI modes
are not rebuilt.
"""

import math
import os
import sys
import time

import torch
import yaml

from . import distributed as hdist
from .environment import make_env, prepare_env
from .hostgen import HostBatchGenerator, MomentReplay
from .rollout import DeviceGenerator, DeviceReplay, ParallelTicTacToeBatch, PlayerReplay, TicTacToeBatch
from .trainer import Trainer


def _batched_envs():
    from .envs.geister import GeisterBatch
    from .envs.ci_geister import CIGeisterBatch
    return {'handyrl_amd.envs.tictactoe': TicTacToeBatch, 'handyrl_amd.envs.geister': GeisterBatch,
            'handyrl_amd.envs.ci_geister': CIGeisterBatch,
            'handyrl_amd.envs.parallel_tictactoe': ParallelTicTacToeBatch}


TRAIN_DEFAULTS = {   # config.yaml:9-31
    'turn_based_training': True, 'observation': False, 'gamma': 0.8, 'forward_steps': 16,
    'compress_steps': 4, 'entropy_regularization': 1.0e-1, 'entropy_regularization_decay': 0.1,
    'update_episodes': 200, 'batch_size': 256, 'minimum_episodes': 400, 'maximum_episodes': 100000,
    'epochs': -1, 'lambda': 0.7, 'policy_target': 'UPGO', 'value_target': 'VTRACE', 'seed': 0,
    'restart_epoch': 0,
}


def load_config(path='config.yaml'):
    with open(path) as f:
        args = yaml.safe_load(f)
    args['train_args'] = {**TRAIN_DEFAULTS, **(args.get('train_args') or {})}
    return args


class ReplayBatcher:
    """``batch()`` for Trainer: one window batch gathered on the device from the replay (train.py:284-309)."""

    def __init__(self, replay, args, generator):
        self.replay, self.args, self.g = replay, args, generator

    def batch(self):
        return self.replay.sample(self.args['batch_size'], self.args['forward_steps'], generator=self.g)


def _per_rank(n, world):
    return max(1, -(-int(n) // world))


def train_main(args, device=None, loss_fn=None, model_dir='models', log=print):
    """The learner cycle of train.py:425-560 on the device; returns the trained model (CPU copy)."""
    env_args, targs = args['env_args'], {**TRAIN_DEFAULTS, **args['train_args']}
    rank, world, local = hdist.init_process_group('cuda' if device is None else device.type)
    if device is None:
        if not torch.cuda.is_available():
            raise RuntimeError('handyrl_amd.main trains on the GPU (HIP kernels); no GPU is visible')
        device = torch.device('cuda', local)
        torch.cuda.set_device(device)
    prepare_env(env_args)
    env = make_env(env_args)
    module = type(env).__module__
    batched = _batched_envs().get(module)
    mode = targs.get('generator', 'auto')
    if mode not in ('auto', 'device', 'host'):
        raise ValueError("train_args['generator'] must be auto, device or host, not %r" % (mode,))
    # the mover-only ply for the stock mode of an alternating env, the per-player ply (every player's view,
    # records with a player axis) with observation, for simultaneous envs and for solo training
    tbt, observe = targs['turn_based_training'], targs['observation']
    per_player = observe or not tbt or getattr(batched, 'SIMULTANEOUS', False)
    if mode == 'device' and batched is None:
        raise ValueError('no batched (device) form of env %r' % module)
    use_device = batched is not None and mode != 'host'
    seed = int(targs['seed']) + rank
    torch.manual_seed(targs['seed'])            # the same initial weights on every rank
    net = env.net()()
    restart = int(targs['restart_epoch'])
    if restart > 0:
        net.load_state_dict(torch.load(os.path.join(model_dir, '%d.pth' % restart), map_location='cpu',
                                       weights_only=True))
    net = net.to(device)
    # the episode counts are global (train.py:480-503, 549-552): each rank plays and keeps 1/world of them
    games = _per_rank(targs['update_episodes'], world)
    minimum = _per_rank(targs['minimum_episodes'], world)
    maximum = _per_rank(targs['maximum_episodes'], world)
    rng = torch.Generator(device=device).manual_seed(seed)
    if use_device:
        gen = DeviceGenerator(batched(games, device), net, gamma=targs['gamma'], observation=observe,
                              per_player=per_player)
        # binary observation planes live in HBM as uint8 (widened by the gather)
        if per_player:
            replay = PlayerReplay(maximum, batched.MAX_PLIES, batched.OBS_SHAPE, batched.A, batched.P, device,
                                  maximum_episodes=maximum, obs_dtype=torch.uint8, solo=not tbt,
                                  mover=tbt and not observe)
        else:
            replay = DeviceReplay(maximum, batched.MAX_PLIES, batched.OBS_SHAPE, batched.A, batched.P, device,
                                  maximum_episodes=maximum, obs_dtype=torch.uint8)

        def play():
            ep = gen.generate(generator=rng)
            replay.add(ep)
            return float(ep['length'].float().sum())
    else:
        slots = min(games, int(targs.get('host_envs', 256)))
        gen = HostBatchGenerator(lambda: make_env(env_args), net, targs, E=slots, seed=seed)
        replay = MomentReplay({**targs, 'maximum_episodes': maximum}, device, maximum_episodes=maximum)

        def play():
            eps = gen.generate(games)
            replay.add(eps)
            return float(sum(ep['steps'] for ep in eps))
    trainer = Trainer(targs, net, ReplayBatcher(replay, targs, rng), device=device, world_size=world,
                      loss_fn=loss_fn)
    episodes = 0
    t0 = time.perf_counter()

    def generate():
        nonlocal episodes
        episodes += games
        return play()

    def global_steps(n):
        """Every rank's new env-steps summed: all ranks derive the same step count from it."""
        if world == 1:
            return n
        t = torch.tensor([n], dtype=torch.float64, device=device if device.type == 'cuda' else 'cpu')
        return float(hdist.all_reduce_sum_([t])[0].item())

    new_steps = 0.0
    while episodes < minimum:
        new_steps += generate()
    epoch = restart
    model = None
    while targs['epochs'] < 0 or epoch < restart + targs['epochs']:
        new_steps += generate()
        steps = targs.get('steps_per_epoch') or max(1, math.ceil(
            global_steps(new_steps) / (world * targs['batch_size'] * targs['forward_steps'])))
        new_steps = 0.0
        model = trainer.train(max_steps=int(steps))
        epoch += 1
        if rank == 0:
            os.makedirs(model_dir, exist_ok=True)
            torch.save(model.state_dict(), os.path.join(model_dir, '%d.pth' % epoch))
            log('epoch %d: episodes %d, steps %d, lr %.3e (%.1fs)' % (epoch, episodes * world, trainer.steps,
                                                                     trainer.lr, time.perf_counter() - t0))
    return model


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    if not argv or argv[0] not in ('--train', '-t'):
        print('usage: python -m handyrl_amd.main --train [config.yaml]  (the learner side of main.py)')
        return 1
    args = load_config(argv[1] if len(argv) > 1 else 'config.yaml')
    print(args)
    train_main(args)
    return 0


if __name__ == '__main__':
    sys.exit(main())
