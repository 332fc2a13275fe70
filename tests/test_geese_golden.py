"""GeeseNet pinned to the reference's own outputs (config C4, hungry_geese.py:23-57).

The fixtures ``tests/golden/geese_net.*`` come from the reference GeeseNet,
imported in the build container with ``kaggle_environments`` stubbed in
``sys.modules`` (the module imports only ``make`` from it and the net never
calls it; ``tests/golden/make_golden.py geese``):

* seeded initial weights (per-tensor float64 sum and sum of squares);
* the train-mode forward (batch statistics; running statistics afterwards)
  and the eval-mode forward on 10 observations;
* ``compute_loss`` (train.py:218-258) in the solo layout of config C4
  (turn_based_training=False, P = Pp = 1, A = 4) with every parameter's
  gradient;
* three ``Trainer.train`` steps (train.py:375-385: backward, clip 4.0,
  Adam(lr = 3e-8*B*T, weight_decay = 1e-5)) and the final state_dict.

Tolerances.  Loss sums: rel 1e-5 (the north-star bound).  Forward outputs:
1e-5.  Gradients: per-tensor norm-relative 1e-5, except the 13 conv biases,
which sit in front of a training-mode BatchNorm: their exact gradient is 0 and
every implementation (the reference included) produces rounding noise there,
so they are compared in absolute terms against the gradient scale.  Final
weights: the same bias exception (and for the running means, which see the
bias); Adam maps a noise gradient to a +-lr step.
"""

import numpy as np
import pytest
import torch

from handyrl_amd.envs.hungry_geese import GeeseNet
from oracle import learner as ol
from tests.conftest import load_golden


@pytest.fixture(scope='module')
def golden():
    return load_golden('geese_net')


def seeded_net():
    torch.manual_seed(21)
    return GeeseNet()


def golden_batch(arrays, device='cpu'):
    return {k[len('batch.'):]: torch.from_numpy(arrays[k]).to(device) for k in arrays.files
            if k.startswith('batch.')}


def _is_noise_bias(name):
    return name.endswith('conv.bias')        # conv bias in front of a training-mode BatchNorm


def check_loss(losses, dcnt, meta, rtol=1e-5):
    ref = meta['loss']
    assert float(dcnt) == ref['dcnt']
    for k, v in ref['losses'].items():
        got = float(losses[k].detach())
        assert abs(got - v) <= rtol * max(1.0, abs(v)), (k, got, v)


def check_grads(named, arrays, rtol=1e-5):
    scale = float(torch.stack([torch.from_numpy(arrays[k]).double().norm() for k in arrays.files
                               if k.startswith('grad.')]).norm())    # the global gradient norm
    worst = {}
    for n, p in named:
        ref = torch.from_numpy(arrays['grad.' + n])
        g = p.grad.detach().cpu()
        if _is_noise_bias(n):
            # exact gradient 0; the reference's own value is rounding noise of the BN backward
            assert float(g.abs().max()) <= 1e-6 * scale and float(ref.abs().max()) <= 1e-6 * scale, n
            continue
        worst[n] = float((g - ref).norm() / ref.norm().clamp(min=1e-30))
    bad = {n: e for n, e in worst.items() if e > rtol}
    assert not bad, sorted(bad.items(), key=lambda kv: -kv[1])[:5]


def check_final(state, arrays, lr, steps=3, atol=2e-7):
    for k in arrays.files:
        if not k.startswith('final.'):
            continue
        n = k[len('final.'):]
        ref = torch.from_numpy(arrays[k])
        got = state[n].detach().cpu()
        if _is_noise_bias(n) or n.endswith('running_mean'):
            # a noise-driven bias step shifts the next BatchNorm's batch mean by the same amount
            assert float((got - ref).abs().max()) <= 2 * steps * lr + atol, n
        elif n.endswith('num_batches_tracked'):
            assert int(got) == int(ref), n
        else:
            torch.testing.assert_close(got, ref, rtol=1e-5, atol=atol, msg=n)


# ---------------------------------------------------------------------------
# the torch-CPU restatement (the oracle's net) against the reference
# ---------------------------------------------------------------------------

def test_seeded_init_matches_reference(golden):
    meta, _ = golden
    net = seeded_net()
    state = net.state_dict()
    assert list(state) == list(meta['state'])
    for k, (shape, s, sq) in meta['state'].items():
        v = state[k].double()
        assert list(v.shape) == shape, k
        assert float(v.sum()) == s and float((v * v).sum()) == sq, k


def _forward_check(net, arrays, device, atol):
    x = torch.from_numpy(arrays['fwd.x']).to(device)
    net.train()
    out = net(x)
    torch.testing.assert_close(out['policy'].detach().cpu(), torch.from_numpy(arrays['fwd.train_policy']),
                               rtol=1e-5, atol=atol)
    torch.testing.assert_close(out['value'].detach().cpu(), torch.from_numpy(arrays['fwd.train_value']),
                               rtol=1e-5, atol=atol)
    state = net.state_dict()
    for k in arrays.files:
        if k.startswith('fwd.after.'):
            torch.testing.assert_close(state[k[len('fwd.after.'):]].cpu(), torch.from_numpy(arrays[k]),
                                       rtol=1e-5, atol=1e-6, msg=k)
    net.eval()
    with torch.no_grad():
        out = net(x)
    torch.testing.assert_close(out['policy'].cpu(), torch.from_numpy(arrays['fwd.eval_policy']), rtol=1e-5, atol=atol)
    torch.testing.assert_close(out['value'].cpu(), torch.from_numpy(arrays['fwd.eval_value']), rtol=1e-5, atol=atol)


def test_cpu_forward_matches_reference(golden):
    _, arrays = golden
    _forward_check(seeded_net(), arrays, 'cpu', atol=1e-6)


def test_cpu_compute_loss_matches_reference(golden):
    meta, arrays = golden
    net = seeded_net()
    net.train()
    losses, dcnt = ol.compute_loss(golden_batch(arrays), net, None, meta['loss']['args'])
    losses['total'].backward()
    check_loss(losses, dcnt, meta)
    check_grads(net.named_parameters(), arrays)


def test_cpu_learner_steps_match_reference(golden):
    meta, arrays = golden
    lm = meta['learner']
    net = seeded_net()
    learner = ol.CpuLearner(net, meta['loss']['args'], lr=lm['lr'])
    batch = golden_batch(arrays)
    for ref in lm['steps']:
        out = learner.step(batch)
        for k in ('p', 'v', 'ent', 'total', 'grad_norm'):
            assert abs(out[k] - ref[k]) <= 1e-5 * max(1.0, abs(ref[k])), (k, out[k], ref[k])
    check_final(net.state_dict(), arrays, lm['lr'])


# ---------------------------------------------------------------------------
# the HIP path (torus MFMA convs, fused conv->BN->[+h]->ReLU units, fused loss)
# ---------------------------------------------------------------------------

@pytest.mark.gpu
def test_gpu_forward_matches_reference(golden, cuda):
    from handyrl_amd.nn import accelerate
    _, arrays = golden
    net = accelerate(seeded_net().to(cuda))
    _forward_check(net, arrays, cuda, atol=1e-5)


@pytest.mark.gpu
def test_gpu_compute_loss_matches_reference(golden, cuda):
    """Product compute_loss (fused torus units, HIP BN, fused loss and scans) vs the reference."""
    from handyrl_amd.nn import accelerate
    from handyrl_amd.train import compute_loss
    meta, arrays = golden
    net = accelerate(seeded_net().to(cuda))
    net.train()
    losses, dcnt = compute_loss(golden_batch(arrays, cuda), net, None, meta['loss']['args'])
    losses['total'].backward()
    check_loss(losses, dcnt, meta)
    check_grads(net.named_parameters(), arrays)


@pytest.mark.gpu
@pytest.mark.parametrize('graph', [False, True])
def test_gpu_learner_steps_match_reference(golden, cuda, graph):
    """Three LearnerStep updates (eager or HIP graph) vs the reference Trainer's three steps."""
    from handyrl_amd.trainer import LearnerStep
    meta, arrays = golden
    lm = meta['learner']
    step = LearnerStep(seeded_net(), meta['loss']['args'], cuda, lr=lm['lr'], graph=graph)
    batch = golden_batch(arrays, cuda)
    for i, ref in enumerate(lm['steps']):
        out = step.step(batch)
        for k in ('p', 'v', 'ent', 'total', 'grad_norm'):
            assert abs(float(out[k]) - ref[k]) <= 1e-5 * max(1.0, abs(ref[k])), (i, k, float(out[k]), ref[k])
    check_final(step.net.state_dict(), arrays, lm['lr'])


@pytest.mark.gpu
def test_trainer_returned_model_runs_on_cpu(golden, cuda):
    """Trainer.train returns a CPU copy of the accelerated net for the workers (train.py:399-401):
    its forward must run on CPU tensors (the torch form) and equal the GPU net's eval forward."""
    from handyrl_amd.trainer import Trainer
    meta, arrays = golden
    batch = golden_batch(arrays)

    class Batcher:
        def batch(self):
            return batch
    tr = Trainer(dict(meta['loss']['args']), seeded_net(), Batcher(), device=cuda)
    model = tr.train(max_steps=2)
    assert not next(model.parameters()).is_cuda
    x = torch.from_numpy(arrays['fwd.x'])
    with torch.no_grad():
        cpu_out = model(x)
        tr.model.eval()
        gpu_out = tr.model(x.to(cuda))
    for k in ('policy', 'value'):
        torch.testing.assert_close(cpu_out[k], gpu_out[k].cpu(), rtol=1e-5, atol=1e-5, msg=k)
