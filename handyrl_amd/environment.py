"""Environment plugin API — kept identical to handyrl/environment.py.

Existing HandyRL environments drop in unchanged: an env module exposes
``Environment(args)`` (a ``BaseEnvironment``) and optionally ``prepare()``;
it is named either by a registry key or by its import path
(handyrl/environment.py:9-39).  ``env.net()`` returns the ``nn.Module`` class
the learner trains (forward(x, hidden) -> {'policy', 'value'[, 'return'][,
'hidden']}, optional init_hidden(batch_size)).

Every registry key resolves to this package's own env module; any other
module path (e.g. a user's ``my_envs.go`` or ``handyrl.envs.geister`` from a
HandyRL checkout on ``sys.path``) is imported as given.
"""

import importlib

ENVS = {   # environment.py:9-15, every key resolved inside this package
    'TicTacToe': 'handyrl_amd.envs.tictactoe',
    'Geister': 'handyrl_amd.envs.geister',
    'CIGeister': 'handyrl_amd.envs.ci_geister',
    'ParallelTicTacToe': 'handyrl_amd.envs.parallel_tictactoe',
    'HungryGeese': 'handyrl_amd.envs.hungry_geese',
}


def _env_module(env_args):
    name = env_args['env']
    return importlib.import_module(ENVS.get(name, name))


def prepare_env(env_args):
    """Run the env module's optional one-time ``prepare()`` (environment.py:18-26)."""
    module = _env_module(env_args)
    if hasattr(module, 'prepare'):
        module.prepare()


def make_env(env_args):
    """Instantiate ``Environment(env_args)`` of the named module (environment.py:29-37)."""
    return _env_module(env_args).Environment(env_args)


class BaseEnvironment:
    """Abstract game API (environment.py:43-146); subclasses override what they use."""

    def __init__(self, args=None):
        pass

    def __str__(self):
        return ''

    # required of every game
    def reset(self, args=None):
        raise NotImplementedError()

    # required unless step() is overridden
    def play(self, action, player):
        raise NotImplementedError()

    # simultaneous-move games override step(); turn games get it from play()
    def step(self, actions):
        for p, a in actions.items():
            if a is not None:
                self.play(a, p)

    def turn(self):
        return 0

    def turns(self):
        return [self.turn()]

    def terminal(self):
        raise NotImplementedError()

    # immediate rewards (None when the game has none)
    def reward(self):
        return {}

    def outcome(self):
        raise NotImplementedError()

    def legal_actions(self, player):
        raise NotImplementedError()

    def action_length(self):
        raise NotImplementedError()

    def players(self):
        return [0]

    def observation(self, player=None):
        raise NotImplementedError()

    # network battle helpers
    def action2str(self, a, player=None):
        return str(a)

    def str2action(self, s, player=None):
        return int(s)

    def diff_info(self, player=None):
        return ''

    def update(self, info, reset):
        raise NotImplementedError()
