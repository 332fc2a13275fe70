"""Env plugin API (handyrl/environment.py:9-146) over this package's env modules.

* every ENVS key resolves in-tree; make_env / prepare_env behave as the
  reference's (environment.py:18-39);
* the single-game Geister ``Environment`` (one-game GeisterBatch on the CPU)
  replays the 24 reference games of tests/golden/geister_rules.* through the
  plugin API: turn, legal_actions, both players' observations, outcome;
* move notation round trips (geister.py:263-330);
* CIGeister shows the opponent's colours in every view (ci_geister.py:520-568);
* ParallelTicTacToe plays simultaneous turns (parallel_tictactoe.py:13-61).
"""

import random

import numpy as np
import pytest

from handyrl_amd.environment import ENVS, BaseEnvironment, make_env, prepare_env
from tests.test_geister_rules import games  # noqa: F401  (fixture)


def test_registry_resolves_in_tree():
    for name, mod in ENVS.items():
        assert mod.startswith('handyrl_amd.envs.'), name


@pytest.mark.parametrize('name', ['TicTacToe', 'Geister', 'CIGeister', 'ParallelTicTacToe'])
def test_make_env_and_prepare_env(name):
    prepare_env({'env': name})
    env = make_env({'env': name})
    assert isinstance(env, BaseEnvironment)
    env.reset()
    assert env.players() == [0, 1]
    net = env.net()()
    assert sum(p.numel() for p in net.parameters()) > 0
    # play one random game through the API
    steps = 0
    while not env.terminal():
        acts = {p: random.choice(env.legal_actions(p)) for p in env.turns()}
        env.step(acts)
        steps += 1
    assert 1 <= steps <= 202
    o = env.outcome()
    assert o[0] == -o[1]


def test_make_env_by_module_path():
    env = make_env({'env': 'handyrl_amd.envs.tictactoe'})
    assert env.action_length() == 9


def test_hungry_geese_points_to_the_reference_plugin():
    """The rules need kaggle_environments (hungry_geese.py:18); this package never imports the reference, it
    raises an ImportError naming the module path that drops the reference env in; the net is available."""
    with pytest.raises(ImportError, match='handyrl.envs.kaggle.hungry_geese'):
        make_env({'env': 'HungryGeese'})
    from handyrl_amd.envs.hungry_geese import Environment
    assert Environment.net(None).__name__ == 'GeeseNet'


def test_make_env_imports_a_plugin_module_path(monkeypatch):
    """A plugin named by module path in config.yaml (e.g. the reference's handyrl.envs.kaggle.hungry_geese)
    is imported as given and instantiated with the env args (environment.py:29-37)."""
    import sys
    import types
    calls = []

    class PluginEnv(BaseEnvironment):
        def __init__(self, args):
            calls.append(args)

    plugin = types.ModuleType('my_plugin_envs_geese')
    plugin.Environment = PluginEnv
    monkeypatch.setitem(sys.modules, 'my_plugin_envs_geese', plugin)
    env = make_env({'env': 'my_plugin_envs_geese', 'x': 1})
    assert isinstance(env, PluginEnv) and calls == [{'env': 'my_plugin_envs_geese', 'x': 1}]


def test_geister_plugin_replays_reference_games(games):   # noqa: F811
    from handyrl_amd.envs.geister import Environment
    env = Environment()
    for g in games:
        env.reset()
        for t in range(g['plies']):
            assert not env.terminal()
            assert env.turn() == g['turn'][t]
            assert sorted(env.legal_actions()) == list(np.nonzero(g['legal'][t])[0])
            for q in (0, 1):
                obs = env.observation(q)
                np.testing.assert_array_equal(obs['board'], g['board'][t, q])
                np.testing.assert_array_equal(obs['scalar'], g['scalar'][t, q])
            full = env.observation(None)
            mine = env.observation(env.turn())
            np.testing.assert_array_equal(full['board'][:5], mine['board'][:5])
            np.testing.assert_array_equal(full['scalar'], mine['scalar'])
            env.play(int(g['action'][t]))
        assert env.terminal()
        o = env.outcome()
        assert [o[0], o[1]] == list(g['outcome'])
        assert env.reward() == {0: -0.01, 1: -0.01}


def test_geister_full_view_shows_opponent_colours(games):   # noqa: F811
    from handyrl_amd.envs.geister import Environment
    env = Environment()
    g = games[0]
    for t in range(4):
        env.play(int(g['action'][t]))
    full = env.observation(None)['board']
    # the opponent's blue + red planes are exactly its pieces (plane 2)
    np.testing.assert_array_equal(full[5] + full[6], full[2])
    assert full[5].sum() == 4 and full[6].sum() == 4
    hidden = env.observation(env.turn())['board']
    assert hidden[5:].sum() == 0


def test_ci_geister_shows_colours_in_every_view(games):   # noqa: F811
    from handyrl_amd.envs.ci_geister import Environment
    env = Environment()
    g = games[1]
    for t in range(6):
        env.play(int(g['action'][t]))
    for q in (0, 1):
        b = env.observation(q)['board']
        np.testing.assert_array_equal(b[5] + b[6], b[2])
        np.testing.assert_array_equal(b[:5], g['board'][6, q][:5])


def test_geister_move_notation_round_trips(games):   # noqa: F811
    from handyrl_amd.envs.geister import Environment
    env = Environment()
    seen = 0
    for g in games[:6]:
        env.reset()
        for t in range(g['plies']):
            p = env.turn()
            for a in env.legal_actions():
                s = env.action2str(a, p)
                assert env.str2action(s, p) == a, (a, s, p)
                seen += 1
            env.play(int(g['action'][t]))
    assert seen > 1000
    assert env.action2str(144, 0) == 's0' and env.str2action('s69', 1) == 213
    assert env.action2str(0 * 36 + 1 * 6 + 1, 0) == 'B2A2'     # direction 0 = (-1, 0) from B2


def test_parallel_tictactoe_simultaneous_turns():
    from handyrl_amd.envs.parallel_tictactoe import Environment
    random.seed(3)
    env, mirror = Environment(), Environment()
    assert env.turns() == [0, 1]
    while not env.terminal():
        env.step({p: random.choice(env.legal_actions(p)) for p in env.turns()})
        mirror.update(env.diff_info(), False)
    assert (mirror.cells == env.cells).all() and mirror.outcome() == env.outcome()
    assert env.observation(0).shape == (3, 3, 3)
