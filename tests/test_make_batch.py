"""handyrl_amd.batch.make_batch vs the reference make_batch (train.py:33-133).

The golden windows (tests/golden/make_batch.*) hold seeded TicTacToe and
Geister self-play episodes, stored pickle-free; this test re-packs them into
the reference wire format (bz2(pickle(moments)) blocks of compress_steps,
generation.py:79-86) with its own code and checks every output tensor
bit for bit, including nested (Geister dict) observations, the solo-mode
random player draw and the padding of short windows.
"""

import bz2
import pickle
import random

import numpy as np
import pytest
import torch

from tests.conftest import load_golden


def decode(obj, arrays):
    if isinstance(obj, dict):
        if '__nd__' in obj:
            return arrays[obj['__nd__']]
        if '__dict__' in obj:
            return {k: decode(v, arrays) for k, v in obj['__dict__']}
    if isinstance(obj, list):
        return [decode(v, arrays) for v in obj]
    return obj


def wire_episode(w, arrays, compress_steps=4):
    moments = decode(w['moments'], arrays)
    blocks = [bz2.compress(pickle.dumps(moments[i:i + compress_steps]))
              for i in range(0, len(moments), compress_steps)]
    return {'args': {}, 'outcome': decode(w['outcome'], arrays), 'moment': blocks,
            'base': w['base'], 'start': w['start'], 'end': w['end'], 'total': w['total']}


@pytest.fixture(scope='module')
def golden_make_batch():
    return load_golden('make_batch')


def test_make_batch_matches_reference(golden_make_batch):
    from handyrl_amd.batch import make_batch
    meta, arrays = golden_make_batch
    for c in meta:
        eps = [wire_episode(w, arrays) for w in c['windows']]
        random.seed(c['seed'])
        batch = make_batch(eps, c['args'])
        got = {}
        for k, v in batch.items():
            if isinstance(v, dict):
                for kk, vv in v.items():
                    got['%s.%s' % (k, kk)] = vv
            else:
                got[k] = v
        assert sorted(got) == sorted(c['out_keys']), c['name']
        for k in c['out_keys']:
            ref = arrays['%d:out.%s' % (c['id'], k)]
            val = got[k].numpy()
            assert val.dtype == ref.dtype and val.shape == ref.shape, (c['name'], k, val.shape, ref.shape)
            np.testing.assert_array_equal(val, ref, err_msg='%s %s' % (c['name'], k))


def test_make_batch_feeds_the_learner_layout(golden_make_batch):
    """Shapes the learner consumes: value-side P, policy-side P'."""
    from handyrl_amd.batch import make_batch
    meta, arrays = golden_make_batch
    c = next(m for m in meta if m['name'] == 'ttt_tbt')
    batch = make_batch([wire_episode(w, arrays) for w in c['windows']], c['args'])
    B, T = len(c['windows']), c['args']['forward_steps']
    assert batch['observation'].shape == (B, T, 1, 3, 3, 3)
    assert batch['policy'].shape == (B, T, 1, 9) and batch['action'].dtype == torch.int64
    assert batch['value'].shape == (B, T, 2, 1) and batch['outcome'].shape == (B, 1, 2, 1)
    assert batch['progress'].shape == (B, T, 1)
