"""Learner parity on the GPU: handyrl_amd.train / trainer vs the reference.

* compute_loss (HIP fused target scans + PyTorch-ROCm) on the reference's
  make_batch batches with fixed network outputs: losses to rel 1e-5, dcnt
  exact, gradients w.r.t. the outputs;
* three learner steps of the TicTacToe net from the reference's initial
  weights: per-step losses and final weights vs the reference's;
* the HIP-graph-captured step equals the eager step;
* the BASELINE-size synthetic batch (B=4096, T=32) against the CPU oracle: the fused loss on fixed outputs,
  and one full learner step of the real SimpleConv2dModel (HIP net, BN, chain block backward, clip, Adam)
  at B=4096 with T=32 and T=9 (configs[1]).
"""

import numpy as np
import pytest
import torch

from oracle import learner as ol

from tests.test_oracle_learner import FixedOutputs, loss_case, learner_setup

pytestmark = pytest.mark.gpu

RTOL = 1e-5


def _to(batch, dev):
    return {k: (v.to(dev) if isinstance(v, torch.Tensor) else {kk: vv.to(dev) for kk, vv in v.items()})
            for k, v in batch.items()}


def _close(a, b, rtol=RTOL, what=''):
    assert abs(a - b) <= rtol * max(1.0, abs(b)), (what, a, b)


def test_compute_loss_golden(cuda, golden_loss):
    from handyrl_amd.train import compute_loss
    meta, arrays = golden_loss
    for c in meta:
        batch, net = loss_case(arrays, c)
        net = net.to(cuda)
        losses, dcnt = compute_loss(_to(batch, cuda), net, None, c['args'])
        assert dcnt == c['dcnt']
        for k, v in c['losses'].items():
            _close(losses[k].item(), v, what=(c['name'], k))
        losses['total'].backward()
        pre = '%d:' % c['id']
        np.testing.assert_allclose(net.p.grad.cpu().numpy(), arrays[pre + 'grad.policy'], rtol=1e-5, atol=1e-6)
        np.testing.assert_allclose(net.v.grad.cpu().numpy(), arrays[pre + 'grad.value'], rtol=1e-5, atol=1e-6)
        if c['has_return']:
            np.testing.assert_allclose(net.r.grad.cpu().numpy(), arrays[pre + 'grad.return'], rtol=1e-5, atol=1e-6)


def test_learner_steps_golden(cuda, golden_learner):
    from handyrl_amd.trainer import LearnerStep
    meta, arrays, net, batch = learner_setup(golden_learner)
    step = LearnerStep(net, meta['args'], cuda, lr=meta['lr'], graph=False)
    net.train()
    b = _to(batch, cuda)
    for s, ref in enumerate(meta['steps']):
        out = step.step(b)
        for k in ('p', 'v', 'ent', 'total', 'grad_norm'):
            _close(out[k].item(), ref[k], what=(s, k))
        assert out['dcnt'].item() == ref['dcnt']
    for k, v in net.state_dict().items():
        np.testing.assert_allclose(v.cpu().numpy(), arrays['final.' + k], rtol=1e-5, atol=1e-6, err_msg=k)
    # the rewritten forward ran the chain + heads as one Function with the value head's tanh in its kernels
    gm = getattr(net, '_hrl_graph', None)
    assert gm is not None and gm.get_submodule('_hrl_chain_heads').tanh_v


def test_graph_step_equals_eager(cuda):
    from handyrl_amd.envs.tictactoe import SimpleConv2dModel
    from handyrl_amd.synthetic import tictactoe_batch, default_args
    from handyrl_amd.trainer import LearnerStep
    B, T = 256, 9
    args = default_args(T, B)
    batch = tictactoe_batch(B, T, cuda, seed=3)
    torch.manual_seed(0)
    ref_net = SimpleConv2dModel()
    g_net = SimpleConv2dModel()
    g_net.load_state_dict(ref_net.state_dict())
    eager = LearnerStep(ref_net, args, cuda, graph=False)
    graph = LearnerStep(g_net, args, cuda, graph=True)
    for _ in range(5):
        e_out = eager.step(batch)
    for _ in range(5):         # the capture's warm-up updates are rolled back: 5 replays = 5 updates
        g_out = graph.step(batch)
    torch.cuda.synchronize()
    for k in ('p', 'v', 'ent', 'total'):
        _close(g_out[k].item(), e_out[k].item(), rtol=1e-5, what=k)
    # hipBLASLt may pick a different (split-K) GEMM schedule under capture, so the
    # two runs differ by fp32 summation order; Adam's m/sqrt(v) amplifies that on
    # near-zero gradients to ~1e-6 absolute after five updates.
    for (k, a), b in zip(ref_net.state_dict().items(), g_net.state_dict().values()):
        np.testing.assert_allclose(b.cpu().numpy(), a.cpu().numpy(), rtol=1e-5, atol=5e-6, err_msg=k)


@pytest.mark.parametrize('graph', [False, True])
def test_running_stats_summed_by_step_tail(cuda, graph):
    """pop_stats() after k steps = the host sum of the k steps' outputs; the tail's second launch does the adds
    (no stack + add launches per step), the capture's warm-up steps are not counted, and pop_stats restarts the
    sums."""
    from handyrl_amd.envs.tictactoe import SimpleConv2dModel
    from handyrl_amd.synthetic import tictactoe_batch, default_args
    from handyrl_amd.trainer import LearnerStep
    B, T = 64, 9
    args = default_args(T, B)
    torch.manual_seed(1)
    step = LearnerStep(SimpleConv2dModel(), args, cuda, graph=graph)
    assert step.tail is not None
    for rnd in range(2):
        want = {}
        for s in range(3):
            out = step.step(tictactoe_batch(B, T, cuda, seed=10 * rnd + s))
            for k, v in out.items():
                want[k] = want.get(k, 0.0) + float(v)
        assert step._tail_stats
        got, n = step.pop_stats()
        assert n == 3 and set(got) == set(want)
        for k in want:
            _close(got[k], want[k], rtol=1e-6, what=(rnd, k))
    assert step.pop_stats() == ({}, 0)


@pytest.mark.parametrize('B,T', [(4096, 32), (4096, 9)])
def test_baseline_batch_losses_vs_oracle(cuda, B, T):
    from handyrl_amd.synthetic import tictactoe_batch, default_args
    from handyrl_amd.train import loss_terms, forward_prediction
    args = default_args(T, B)
    batch = tictactoe_batch(B, T, cuda, seed=B + T)
    g = torch.Generator().manual_seed(5)
    p = torch.randn(B * T, 9, generator=g)
    v = torch.tanh(torch.randn(B * T, 1, generator=g))
    net_gpu = FixedOutputs(p.numpy(), v.numpy()).to(cuda)
    net_cpu = FixedOutputs(p.numpy(), v.numpy())
    losses, dcnt = loss_terms(forward_prediction(net_gpu, None, batch, args), batch, args)
    cpu_batch = {k: t.cpu() for k, t in batch.items()}
    ref, ref_dcnt = ol.compute_loss(cpu_batch, net_cpu, None, args)
    assert dcnt.item() == ref_dcnt
    for k in ref:
        _close(losses[k].item(), ref[k].item(), what=k)
    losses['total'].backward()
    ref['total'].backward()
    np.testing.assert_allclose(net_gpu.p.grad.cpu().numpy(), net_cpu.p.grad.numpy(), rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(net_gpu.v.grad.cpu().numpy(), net_cpu.v.grad.numpy(), rtol=1e-5, atol=1e-6)


def oracle_step_grads(net_cls, state, batch, args, seed_threads=8):
    """One CPU oracle learner step in fp32 (the reference's arithmetic: losses, grad norm, clipped gradients)
    and in fp64 (the gradients' exact value to ~1e-15) from the same weights and batch."""
    out = {}
    threads = torch.get_num_threads()
    torch.set_num_threads(seed_threads)
    try:
        for dt in (torch.float32, torch.float64):
            net = net_cls()
            net.load_state_dict(state)
            net = net.to(dt)
            b = {k: (v.cpu().to(dt) if v.is_floating_point() else v.cpu()) for k, v in batch.items()}
            r = ol.CpuLearner(net, args).step(b)
            r['grads'] = {n: p.grad.double().clone() for n, p in net.named_parameters()}
            r['buffers'] = {n: t.clone() for n, t in net.named_buffers()}
            out[dt] = r
    finally:
        torch.set_num_threads(threads)
    return out[torch.float32], out[torch.float64]


def check_grads_vs_fp64(got, r32, r64, factor=4.0, floor=1e-4):
    """Every parameter's clipped gradient: its norm-relative error against the fp64 oracle may not exceed
    `factor` times the fp32 CPU oracle's own, nor `floor` when the CPU's is smaller.  Returns the worst
    (name, gpu error, cpu error).

    Why a factor and a floor rather than a tight bound: a ReLU decides on a pre-activation's sign, and a
    board net's pre-activations repeat exactly across rows (binary planes: every row with the same 3x3
    neighbourhood gets the same value, padded rows are all zero), so a value within fp32 rounding of zero
    flips for a whole group of rows at once, in one fp32 implementation and not in another.  Each flip moves
    the gradient by a discrete amount that no summation order avoids (tools/grad_diag.py on the GPU,
    profiles/r03_grad_diag.txt: TicTacToe T=9 errors up to 8e-5 from block 1 down, where the CPU's are
    4e-7, while the stem's weight-gradient kernel alone is within 3e-8 of fp64 from the same dY; GeeseNet
    T=64: the CPU's own errors reach 1e-3).  The kernels' arithmetic is pinned tightly elsewhere
    (tests/test_bn_gpu.py: the stem, the block chain and the BatchNorm kernels at norm-relative 1e-6, or exact on
    integer data)."""
    worst = None
    for n, g64 in r64['grads'].items():
        den = float(g64.norm())
        if den == 0.0:
            continue
        e_gpu = float((got[n] - g64).norm()) / den
        e_cpu = float((r32['grads'][n] - g64).norm()) / den
        assert e_gpu <= max(factor * e_cpu, floor), (n, e_gpu, e_cpu)
        if worst is None or e_gpu > worst[1]:
            worst = (n, e_gpu, e_cpu)
    return worst


@pytest.mark.parametrize('T', [32, 9])
def test_full_size_learner_step_vs_oracle(cuda, T):
    """One LearnerStep of the real TicTacToe net at the metric's B=4096 (T=32, and configs[1]'s T=9) vs
    oracle.learner.CpuLearner on the same batch from the same seeded weights: losses and the clipped
    gradient norm at rel 1e-5 against the fp32 oracle, dcnt exact, every parameter's clipped gradient against
    the same step in fp64 (check_grads_vs_fp64: within 4x the fp32 oracle's own error or 1e-4), and the
    BatchNorm running statistics after the step."""
    from handyrl_amd.envs.tictactoe import SimpleConv2dModel
    from handyrl_amd.synthetic import tictactoe_batch, default_args
    from handyrl_amd.trainer import LearnerStep
    B = 4096
    args = default_args(T, B)
    batch = tictactoe_batch(B, T, cuda, seed=11 + T)
    torch.manual_seed(1)
    state = SimpleConv2dModel().state_dict()
    r32, r64 = oracle_step_grads(SimpleConv2dModel, state, batch, args)
    net = SimpleConv2dModel()
    net.load_state_dict(state)
    step = LearnerStep(net, args, cuda, graph=False)
    out = step.step(batch)
    torch.cuda.synchronize()
    assert out['dcnt'].item() == r32['dcnt']
    for k in ('p', 'v', 'ent', 'total', 'grad_norm'):
        _close(float(out[k]), r32[k], what=k)
    got = {n: p.grad.detach().cpu().double() for n, p in step.net.named_parameters()}
    check_grads_vs_fp64(got, r32, r64)
    for n, b in step.net.named_buffers():
        if n in r32['buffers'] and b.dtype.is_floating_point:
            torch.testing.assert_close(b.cpu(), r32['buffers'][n], rtol=1e-5, atol=1e-6, msg=n)


ALGS = ('MC', 'TD', 'UPGO', 'VTRACE')


@pytest.mark.parametrize('vt', ALGS)
@pytest.mark.parametrize('pt', ALGS)
def test_fused_loss_all_target_pairs(cuda, golden_loss, vt, pt):
    """Fused HIP loss vs the CPU oracle for every (value_target, policy_target),
    on the Geister batch with a return head (A = 214, rewards, gamma = 0.8)."""
    from handyrl_amd.train import compute_loss
    meta, arrays = golden_loss
    c = next(m for m in meta if m['name'] == 'geister_ret')
    args = dict(c['args'], value_target=vt, policy_target=pt)
    batch, net_cpu = loss_case(arrays, c)
    _, net_gpu = loss_case(arrays, c)
    net_gpu = net_gpu.to(cuda)
    ref, ref_dcnt = ol.compute_loss(batch, net_cpu, None, args)
    out, dcnt = compute_loss(_to(batch, cuda), net_gpu, None, args)
    assert dcnt == ref_dcnt
    for k in ref:
        _close(out[k].item(), ref[k].item(), what=(vt, pt, k))
    ref['total'].backward()
    out['total'].backward()
    for a, b in ((net_gpu.p, net_cpu.p), (net_gpu.v, net_cpu.v), (net_gpu.r, net_cpu.r)):
        np.testing.assert_allclose(a.grad.cpu().numpy(), b.grad.numpy(), rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize('weights', [(1, 0, 0, 0, 0), (0, 0, 0, 1, 0), (0.5, 2.0, -1.0, 0.25, 1.0)])
def test_fused_loss_arbitrary_upstream_grads(cuda, golden_loss, weights):
    """Backward from any combination of the five losses (not only 'total')."""
    from handyrl_amd.train import compute_loss
    meta, arrays = golden_loss
    c = next(m for m in meta if m['name'] == 'geister_ret')
    batch, net_cpu = loss_case(arrays, c)
    _, net_gpu = loss_case(arrays, c)
    net_gpu = net_gpu.to(cuda)
    ref, _ = ol.compute_loss(batch, net_cpu, None, c['args'])
    out, _ = compute_loss(_to(batch, cuda), net_gpu, None, c['args'])
    keys = ('p', 'v', 'r', 'ent', 'total')
    sum(w * ref[k] for w, k in zip(weights, keys)).backward()
    sum(w * out[k] for w, k in zip(weights, keys)).backward()
    for a, b in ((net_gpu.p, net_cpu.p), (net_gpu.v, net_cpu.v), (net_gpu.r, net_cpu.r)):
        np.testing.assert_allclose(a.grad.cpu().numpy(), b.grad.numpy(), rtol=1e-5, atol=1e-6)


def test_fused_loss_deterministic(cuda):
    from handyrl_amd.synthetic import tictactoe_batch, default_args
    from handyrl_amd.train import loss_terms, forward_prediction
    B, T = 4096, 32
    args = default_args(T, B)
    batch = tictactoe_batch(B, T, cuda, seed=9)
    g = torch.Generator().manual_seed(1)
    net = FixedOutputs(torch.randn(B * T, 9, generator=g).numpy(),
                       torch.tanh(torch.randn(B * T, 1, generator=g)).numpy()).to(cuda)
    runs = []
    for _ in range(2):
        net.zero_grad()
        losses, dcnt = loss_terms(forward_prediction(net, None, batch, args), batch, args)
        losses['total'].backward()
        runs.append((torch.stack([losses[k] for k in ('p', 'v', 'ent', 'total')]).cpu(), net.p.grad.clone()))
    assert torch.equal(runs[0][0], runs[1][0]) and torch.equal(runs[0][1], runs[1][1])


@pytest.mark.gpu
@pytest.mark.parametrize('Pq', [1, 2])
def test_output_mask_kernels_match_torch(Pq):
    """forward_prediction's masking (train.py:176-183) as one HIP launch each way (_OutputMask) vs the torch ops."""
    if not torch.cuda.is_available():
        pytest.skip('no GPU')
    from handyrl_amd.train import _OutputMask
    dev = torch.device('cuda', 0)
    g = torch.Generator().manual_seed(Pq)
    B, T, P, A = 37, 9, 2, 9
    opol = torch.randn(B, T, Pq, A, generator=g)
    oval = torch.randn(B, T, Pq, 1, generator=g)
    tmask = (torch.rand(B, T, P, 1, generator=g) > 0.5).float()
    omask = (torch.rand(B, T, P, 1, generator=g) > 0.3).float()
    amask = (torch.rand(B, T, 1, A, generator=g) > 0.7).float() * 1e32
    gp, gv = torch.randn(B, T, 1, A, generator=g), torch.randn(B, T, P, 1, generator=g)
    ref_in = [opol.clone().requires_grad_(True), oval.clone().requires_grad_(True)]
    rp = ref_in[0].mul(tmask).sum(2, keepdim=True) - amask
    rv = ref_in[1].mul(omask)
    torch.autograd.backward([rp, rv], [gp, gv])
    hip_in = [opol.to(dev).requires_grad_(True), oval.to(dev).requires_grad_(True)]
    hp, hv = _OutputMask.apply(hip_in[0], hip_in[1], tmask.to(dev), omask.to(dev), amask.to(dev))
    torch.autograd.backward([hp, hv], [gp.to(dev), gv.to(dev)])
    assert torch.equal(hp.detach().cpu(), rp.detach()) and torch.equal(hv.detach().cpu(), rv.detach())
    assert torch.equal(hip_in[0].grad.cpu(), ref_in[0].grad) and torch.equal(hip_in[1].grad.cpu(), ref_in[1].grad)
