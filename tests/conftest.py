import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, 'tests', 'golden')


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs an MI355X (runs through libhrl.so on cuda:0)')


def load_golden(name):
    with open(os.path.join(GOLDEN, name + '.json')) as f:
        meta = json.load(f)
    arrays = np.load(os.path.join(GOLDEN, name + '.npz'))
    return meta, arrays


@pytest.fixture(scope='session')
def golden_targets():
    return load_golden('targets')


@pytest.fixture(scope='session')
def golden_loss():
    return load_golden('loss')


@pytest.fixture(scope='session')
def golden_learner():
    return load_golden('learner')


@pytest.fixture(scope='session')
def cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip('no GPU in this environment')
    from handyrl_amd import _native
    _native.load()  # the HIP library must load on a GPU box: no fallback
    return torch.device('cuda', 0)
