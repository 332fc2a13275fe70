"""GeisterNet (config C3, recurrent DRC ConvLSTM) against the reference.

Golden data (tests/golden/geister_net.*, made by make_golden.py from
handyrl/envs/geister.py:17-167 and train.py:136-258):
* per-tensor sum / sum of squares of the seeded initial state_dict
  (torch.manual_seed(11); GeisterNet()): same keys, shapes, values;
* one training-mode forward with a non-zero hidden state;
* compute_loss through the recurrent branch of forward_prediction on a
  reference make_batch batch of real Geister windows, with the per-parameter
  squared gradient norms of the summed loss.
CPU tests pin handyrl_amd.envs.geister.GeisterNet and the oracle; the GPU test
runs the product path (HIP BatchNorm, HIP target scans, fused HIP loss) on it.
"""

import numpy as np
import pytest
import torch

from tests.conftest import load_golden
from oracle import learner as ol
from handyrl_amd.envs.geister import GeisterNet


@pytest.fixture(scope='module')
def golden():
    return load_golden('geister_net')


def seeded_net():
    torch.manual_seed(11)
    return GeisterNet()


def test_init_matches_reference(golden):
    meta, _ = golden
    sd = seeded_net().state_dict()
    assert list(sd) == list(meta['state'])
    for k, (shape, s, sq) in meta['state'].items():
        v = sd[k].double()
        assert list(v.shape) == shape, k
        # fp64 sums of fp32 weights: identical weights agree to reduction-order rounding
        assert abs(float(v.sum()) - s) <= 1e-12 * max(1.0, abs(s)), k
        assert abs(float((v * v).sum()) - sq) <= 1e-12 * max(1.0, sq), k
    assert sum(p.numel() for p in seeded_net().parameters()) == 233832


def fwd_inputs(arrays):
    obs = {'board': torch.from_numpy(arrays['fwd.board'].copy()),
           'scalar': torch.from_numpy(arrays['fwd.scalar'].copy())}
    hs = [torch.from_numpy(arrays['fwd.h%d' % i].copy()) for i in range(3)]
    cs = [torch.from_numpy(arrays['fwd.c%d' % i].copy()) for i in range(3)]
    return obs, (hs, cs)


def check_forward(out, arrays, atol):
    for k in ('policy', 'value', 'return'):
        np.testing.assert_allclose(out[k].detach().cpu().numpy(), arrays['fwd.out_' + k], rtol=0, atol=atol)
    for i in range(3):
        np.testing.assert_allclose(out['hidden'][0][i].detach().cpu().numpy(), arrays['fwd.out_h%d' % i],
                                   rtol=0, atol=atol)
        np.testing.assert_allclose(out['hidden'][1][i].detach().cpu().numpy(), arrays['fwd.out_c%d' % i],
                                   rtol=0, atol=atol)


def test_forward_matches_reference(golden):
    _, arrays = golden
    obs, hidden = fwd_inputs(arrays)
    hs_in = list(hidden[0])
    out = seeded_net()(obs, hidden)
    check_forward(out, arrays, atol=1e-6)
    assert all(a is b for a, b in zip(hidden[0], hs_in))  # caller's hidden lists left untouched


def golden_batch(arrays):
    batch = {}
    for k in arrays.files:
        if not k.startswith('batch.'):
            continue
        parts = k.split('.')[1:]
        v = torch.from_numpy(arrays[k].copy())
        if len(parts) == 2:
            batch.setdefault(parts[0], {})[parts[1]] = v
        else:
            batch[parts[0]] = v
    return batch


def check_loss(losses, dcnt, grads, meta, rtol):
    ref = meta['loss']
    assert dcnt == ref['dcnt']
    for k, v in ref['losses'].items():
        assert abs(float(losses[k].detach()) - v) <= rtol * max(1.0, abs(v)), (k, float(losses[k].detach()), v)
    for n, sq in ref['grad_sq'].items():
        assert abs(grads[n] - sq) <= rtol * max(1e-6, sq) + 1e-9, (n, grads[n], sq)


def test_oracle_rnn_compute_loss_matches_reference(golden):
    meta, arrays = golden
    batch = golden_batch(arrays)
    net = seeded_net()
    B, P = batch['value'].shape[0], batch['value'].shape[2]
    losses, dcnt = ol.compute_loss(batch, net, net.init_hidden([B, P]), meta['loss']['args'])
    losses['total'].backward()
    grads = {n: float((p.grad.double() ** 2).sum()) for n, p in net.named_parameters() if p.grad is not None}
    check_loss(losses, dcnt, grads, meta, rtol=1e-5)


@pytest.mark.gpu
def test_gpu_forward_matches_reference(golden, cuda):
    from handyrl_amd.nn import accelerate
    _, arrays = golden
    net = seeded_net().to(cuda)
    accelerate(net)
    obs, hidden = fwd_inputs(arrays)
    obs = {k: v.to(cuda) for k, v in obs.items()}
    hidden = ([h.to(cuda) for h in hidden[0]], [c.to(cuda) for c in hidden[1]])
    check_forward(net(obs, hidden), arrays, atol=2e-5)


@pytest.mark.gpu
def test_gpu_rnn_compute_loss_matches_reference(golden, cuda):
    """Product compute_loss (HIP BN / scans / fused loss) through the recurrent branch."""
    from handyrl_amd.nn import accelerate
    from handyrl_amd.train import compute_loss
    meta, arrays = golden
    batch = {k: ({kk: vv.to(cuda) for kk, vv in v.items()} if isinstance(v, dict) else v.to(cuda))
             for k, v in golden_batch(arrays).items()}
    net = seeded_net().to(cuda)
    accelerate(net)
    B, P = batch['value'].shape[0], batch['value'].shape[2]
    hidden = net.init_hidden([B, P])
    hidden = ([h.to(cuda) for h in hidden[0]], [c.to(cuda) for c in hidden[1]])
    losses, dcnt = compute_loss(batch, net, hidden, meta['loss']['args'])
    losses['total'].backward()
    grads = {n: float((p.grad.double() ** 2).sum()) for n, p in net.named_parameters() if p.grad is not None}
    check_loss(losses, dcnt, grads, meta, rtol=1e-5)


@pytest.mark.gpu
@pytest.mark.parametrize('hw', [(6, 6), (3, 5)])
def test_lstm_gates_kernel_vs_torch(cuda, hw):
    """csrc/hrl_lstm.hip vs the fp32 torch ConvLSTM cell tail (geister.py:52-63), forward and backward.

    zx is a channel slice of a wider tensor (the fused x-half convolution); (3, 5)
    boards take the scalar (non-float4) path.  Tolerance: 2e-6 abs (transcendental ulps).
    """
    from handyrl_amd.nn import lstm_gates
    g = torch.Generator(device=cuda).manual_seed(0)
    N, H = 37, 32
    wide = torch.randn(N, 3 * 4 * H, *hw, device=cuda, generator=g).requires_grad_()
    zh = torch.randn(N, 4 * H, *hw, device=cuda, generator=g).requires_grad_()
    c = torch.randn(N, H, *hw, device=cuda, generator=g).requires_grad_()
    dh = torch.randn(N, H, *hw, device=cuda, generator=g)
    dc = torch.randn(N, H, *hw, device=cuda, generator=g)

    def ref(zx, zh, c):
        i, f, o, gg = (zx + zh).chunk(4, 1)
        c2 = torch.sigmoid(f) * c + torch.sigmoid(i) * torch.tanh(gg)
        return torch.sigmoid(o) * torch.tanh(c2), c2

    for use_dc in (True, False):
        outs, grads = [], []
        for fn in (lstm_gates, ref):
            for t in (wide, zh, c):
                t.grad = None
            h2, c2 = fn(wide[:, 4 * H:8 * H], zh, c)
            loss = (h2 * dh).sum() + ((c2 * dc).sum() if use_dc else 0)
            loss.backward()
            outs.append((h2.detach(), c2.detach()))
            grads.append((wide.grad.clone(), zh.grad.clone(), c.grad.clone()))
        for a, b in zip(outs[0], outs[1]):
            torch.testing.assert_close(a, b, rtol=0, atol=2e-6)
        for a, b in zip(grads[0], grads[1]):
            torch.testing.assert_close(a, b, rtol=0, atol=2e-6)
        assert float(grads[0][0][:, :4 * H].abs().sum()) == 0.0


@pytest.mark.gpu
def test_drc_hip_path_matches_reference_cells(golden, cuda):
    """accelerate(GeisterNet) regroups the DRC (x half once, fused gates); same outputs and gradients."""
    from handyrl_amd.nn import accelerate
    _, arrays = golden
    plain = seeded_net().to(cuda)
    fast = accelerate(seeded_net().to(cuda))
    assert fast.body.use_hip and not plain.body.use_hip
    obs, hidden = fwd_inputs(arrays)
    obs = {k: v.to(cuda) for k, v in obs.items()}
    res = []
    ref64 = seeded_net().double()           # the gradients' exact value (fp64, CPU)
    for net in (plain, fast, ref64):
        dev = next(net.parameters()).device
        dt = next(net.parameters()).dtype
        h = ([t.to(dev, dt) for t in hidden[0]], [t.to(dev, dt) for t in hidden[1]])
        out = net({k: v.to(dev, dt) for k, v in obs.items()}, h)
        loss = out['policy'].square().sum() + out['value'].sum() + sum(t.square().sum() for t in out['hidden'][1])
        loss.backward()
        res.append((out, {n: p.grad.detach().cpu().double().clone() for n, p in net.named_parameters()
                          if p.grad is not None}))
    check_forward(res[1][0], arrays, atol=2e-5)
    assert set(res[0][1]) == set(res[1][1]) == set(res[2][1])
    # every gradient against the fp64 one: the HIP path (x/h halves summed in the gate kernel, HIP BN, split
    # convolutions) within 4x the plain fp32 path's own error, or norm-relative 1e-5 (the north-star bound)
    for n, g64 in res[2][1].items():
        den = float(g64.norm())
        if den == 0.0:
            continue
        e_fast = float((res[1][1][n] - g64).norm()) / den
        e_plain = float((res[0][1][n] - g64).norm()) / den
        assert e_fast <= max(4 * e_plain, 1e-5), (n, e_fast, e_plain)


@pytest.mark.gpu
def test_stacked_inference_matches_cells(golden, cuda):
    """Inference (no autograd) stacks the DRC layers: one grouped h convolution and one gate launch per
    repeat instead of one per layer.  Same outputs and states as the per-layer HIP path, and the reference
    golden forward still holds."""
    from handyrl_amd.nn import accelerate
    _, arrays = golden
    net = accelerate(seeded_net().to(cuda)).eval()
    obs, hidden = fwd_inputs(arrays)
    obs = {k: v.to(cuda) for k, v in obs.items()}
    torch.manual_seed(3)
    x = torch.randn(96, 32, 6, 6, device=cuda)
    hs = [torch.randn(96, 32, 6, 6, device=cuda) for _ in range(3)]
    cs = [torch.randn(96, 32, 6, 6, device=cuda) for _ in range(3)]
    with torch.no_grad():
        h_a, (hs_a, cs_a) = net.body._inference_stacked(x, list(hs), list(cs), 3)
        h_b, (hs_b, cs_b) = net.body._forward_hip(x, list(hs), list(cs), 3)
        for a, b in zip([h_a] + hs_a + cs_a, [h_b] + hs_b + cs_b):
            torch.testing.assert_close(a, b, rtol=1e-6, atol=1e-6)
        h = ([t.to(cuda) for t in hidden[0]], [t.to(cuda) for t in hidden[1]])
        net.train()
        out = net(obs, h)       # training-mode BatchNorm as in the golden, stacked DRC (no autograd)
    check_forward(out, arrays, atol=2e-5)


@pytest.mark.gpu
def test_inference_forward_matches_module_path(golden, cuda):
    """Self-play's eval forward on the HIP path (GeisterNet._forward_inference: BatchNorm + ReLU in one HIP
    launch, stacked DRC, and inside an inference session the stacked weights built once) vs the plain
    module forward of the same net on the CPU: policy, value, return and every state tensor."""
    from handyrl_amd.nn import accelerate
    _, arrays = golden
    cpu = seeded_net().eval()
    with torch.no_grad():   # non-trivial running statistics
        for b in cpu._sequence_bns():
            b.running_mean.uniform_(-0.5, 0.5)
            b.running_var.uniform_(0.5, 2.0)
    gpu = accelerate(seeded_net().to(cuda)).eval()
    gpu.load_state_dict(cpu.state_dict())
    obs, hidden = fwd_inputs(arrays)
    with torch.no_grad():
        ref = cpu(obs, hidden)
        h = ([t.to(cuda) for t in hidden[0]], [t.to(cuda) for t in hidden[1]])
        outs = [gpu({k: v.to(cuda) for k, v in obs.items()}, h)]
        with gpu.inference_session():
            outs.append(gpu({k: v.to(cuda) for k, v in obs.items()}, h))
    for out in outs:
        for k in ('policy', 'value', 'return'):
            torch.testing.assert_close(out[k].cpu(), ref[k], rtol=1e-5, atol=2e-5, msg=k)
        for a, b in zip(out['hidden'][0] + out['hidden'][1], ref['hidden'][0] + ref['hidden'][1]):
            torch.testing.assert_close(a.cpu(), b, rtol=1e-5, atol=2e-5)


@pytest.mark.gpu
@pytest.mark.parametrize('graph', [False, True])
def test_gpu_recurrent_learner_matches_cpu_oracle(cuda, graph):
    """Three recurrent learner steps (LearnerStep on the GPU, HIP graph or eager) vs the oracle's
    CPU learner (train.py:375-385) from the same seeded GeisterNet on the same batch: per-step
    losses and grad norms, and every parameter afterwards.  GeisterNet's first two DRC blocks never
    reach an output (geister.py:91-94): their .grad stays None under the reference's autograd, so
    Adam leaves them untouched -- they must be bit-identical to their initial values."""
    from handyrl_amd.synthetic import geister_batch, default_args
    from handyrl_amd.trainer import LearnerStep
    B, T = 8, 8
    args = default_args(T, B)
    batch = geister_batch(B, T, cuda, seed=3)
    cpu_batch = {k: ({kk: vv.cpu() for kk, vv in v.items()} if isinstance(v, dict) else v.cpu())
                 for k, v in batch.items()}
    ref = seeded_net()
    init = {n: p.detach().clone() for n, p in ref.named_parameters()}
    oracle = ol.CpuLearner(ref, args)
    ref64 = seeded_net().double()           # the same three steps in fp64: the weights' exact trajectory
    oracle64 = ol.CpuLearner(ref64, args)
    batch64 = {k: ({kk: vv.double() for kk, vv in v.items()} if isinstance(v, dict) else
                   (v.double() if v.is_floating_point() else v)) for k, v in cpu_batch.items()}
    net = seeded_net()
    step = LearnerStep(net, args, cuda, graph=graph)

    def zeros(device, dt=torch.float32):
        return tuple([h.to(device, dt) for h in hs] for hs in net.init_hidden([B, 2]))
    for i in range(3):
        r = oracle.step(cpu_batch, zeros('cpu'))
        oracle64.step(batch64, zeros('cpu', torch.float64))
        out = step.step(batch, zeros(cuda))
        for k in ('p', 'v', 'r', 'ent', 'total'):
            assert abs(float(out[k]) - r[k]) <= 1e-5 * max(1.0, abs(r[k])), (i, k, float(out[k]), r[k])
        assert abs(float(out['grad_norm']) - r['grad_norm']) <= 1e-5 * max(1e-3, r['grad_norm']), \
            (i, float(out['grad_norm']), r['grad_norm'])
    dead = [n for (n, _), live in zip(step.net.named_parameters(), step.live) if not live]
    assert sorted(dead) == sorted('body.blocks.%d.conv.%s' % (i, k) for i in (0, 1) for k in ('weight', 'bias'))
    # the weights after three updates against the fp64 trajectory: within 4x the fp32 CPU oracle's own distance
    # from it, or norm-relative 1e-5 (Adam's m / sqrt(v) turns near-zero gradient differences into whole
    # lr-sized steps in either fp32 implementation, so a fixed elementwise tolerance would bound noise)
    got = dict(step.net.named_parameters())
    w64 = dict(ref64.named_parameters())
    for n, p in ref.named_parameters():
        if n in dead:
            assert torch.equal(got[n].detach().cpu(), init[n]), n
            continue
        exact = w64[n].detach()
        den = max(float(exact.norm()), 1e-12)
        e_gpu = float((got[n].detach().cpu().double() - exact).norm()) / den
        e_cpu = float((p.detach().double() - exact).norm()) / den
        assert e_gpu <= max(4 * e_cpu, 1e-5), (n, e_gpu, e_cpu)


@pytest.mark.gpu
def test_sequence_unroll_matches_per_step_unroll(cuda):
    """GeisterNet's three-part unroll (stem, x halves and heads once over all T steps, per-step BatchNorm
    statistics through nn.batch_norm_train(groups=T)) vs the per-step forward loop: outputs, every
    gradient, and the BatchNorm running statistics and batch counters."""
    from handyrl_amd import train as tr
    from handyrl_amd.nn import accelerate
    from handyrl_amd.synthetic import geister_batch, default_args
    B, T = 16, 6
    args = default_args(T, B)
    batch = geister_batch(B, T, cuda, seed=5)
    res = []
    for seq in (False, True):
        net = accelerate(seeded_net().to(cuda))
        net.train()
        hidden = tuple([h.to(cuda) for h in hs] for hs in net.init_hidden([B, 2]))
        prev = tr.SEQUENCE_UNROLL
        tr.SEQUENCE_UNROLL = seq
        try:
            out = tr.forward_prediction(net, hidden, batch, args)
        finally:
            tr.SEQUENCE_UNROLL = prev
        if not res:
            gen = torch.Generator(device=cuda).manual_seed(1)
            wts = {k: torch.randn(o.shape, device=cuda, generator=gen) for k, o in out.items()}
        # linear in the outputs: the masked policy holds -1e32 entries (action_mask), a square would overflow
        loss = sum((out[k] * wts[k]).sum() for k in out)
        loss.backward()
        res.append((out, {n: p.grad.clone() for n, p in net.named_parameters() if p.grad is not None},
                    {n: b.clone() for n, b in net.named_buffers()}))
    (o0, g0, b0), (o1, g1, b1) = res
    for k in o0:
        torch.testing.assert_close(o1[k], o0[k], rtol=1e-5, atol=1e-5, msg=k)
    assert set(g0) == set(g1)
    errs = {n: float((g1[n] - g).norm() / g.norm().clamp(min=1e-12)) for n, g in g0.items()}
    assert max(errs.values()) < 1e-5, sorted(errs.items(), key=lambda kv: -kv[1])[:5]
    for n, b in b0.items():
        if n.endswith('num_batches_tracked'):
            assert int(b1[n]) == int(b) == T, n
        else:
            torch.testing.assert_close(b1[n], b, rtol=1e-5, atol=1e-6, msg=n)


@pytest.mark.gpu
@pytest.mark.parametrize('graph', [False, True])
def test_grouped_drc_step_matches_per_layer_unroll(cuda, graph):
    """The learner's unroll with each time step's DRC repeats under one autograd node (nn.drc_step: per repeat one
    grouped h-half conv + one grouped gate launch, hrl_gboard_forward_groups / hrl_lstm_gates_forward_grouped;
    backward with the K-split adjoint's partials summed inside hrl_lstm_gates_backward_ex) against the per-layer
    launches (_DeferredConv + lstm_gates): from the same seeded net on the same batch (ragged game count) the
    forward -- every loss -- is bit-identical (the per-layer kernels' float operations); the gradient (its norm)
    and the updated weights agree to 1e-6 (the partial input gradients are added in a different order)."""
    from handyrl_amd.envs.geister import DRC
    from handyrl_amd.synthetic import geister_batch, default_args
    from handyrl_amd.trainer import LearnerStep
    B, T = 13, 5
    args = default_args(T, B)
    batch = geister_batch(B, T, cuda, seed=7)
    res = []
    prev = DRC.group_repeat
    try:
        for grouped in (False, True):
            DRC.group_repeat = grouped
            net = seeded_net()
            step = LearnerStep(net, args, cuda, graph=graph)
            hidden = tuple([h.to(cuda) for h in hs] for hs in net.init_hidden([B, 2]))
            out = step.step(batch, hidden)
            res.append(({k: float(out[k]) for k in ('p', 'v', 'r', 'ent', 'total', 'grad_norm')},
                        {n: p.detach().clone() for n, p in step.net.named_parameters()}))
    finally:
        DRC.group_repeat = prev
    (o0, w0), (o1, w1) = res
    for k in ('p', 'v', 'r', 'ent', 'total'):
        assert o0[k] == o1[k], (k, o0[k], o1[k])
    assert abs(o1['grad_norm'] - o0['grad_norm']) <= 1e-6 * o0['grad_norm'], (o0['grad_norm'], o1['grad_norm'])
    for n in w0:
        den = max(float(w0[n].norm()), 1e-12)
        assert float((w1[n] - w0[n]).norm()) / den <= 1e-6, n


@pytest.mark.gpu
@pytest.mark.parametrize('graph', [False, True])
def test_recurrent_learner_step_at_bench_size_vs_oracle(cuda, graph):
    """One LearnerStep of GeisterNet at the size the bench's geister_learner leg and the reference's stock learner
    run (config.yaml:13,18: B = 256, forward_steps = 16; train.py:155-174 for the recurrent unroll) against
    oracle.learner.CpuLearner on the same batch from the same seeded weights: losses and the clipped gradient norm
    at rel 1e-5 against the fp32 oracle, every live parameter's clipped gradient against the same step in fp64
    (check_grads_vs_fp64), the dead DRC blocks untouched.  At this size the gboard launchers pick forms the small
    oracle tests never reach; hrl_gboard_launch_stats asserts they ran: whole-tile launches (one task per workgroup),
    the h halves' K-split adjoint (groups = 4), and games-as-K weight gradients over many recorded uses (segments)
    whose workgroups carry their accumulators over several 16-game tiles (> 256 tiles)."""
    import ctypes
    from handyrl_amd import _native
    from handyrl_amd.synthetic import geister_batch, default_args
    from handyrl_amd.trainer import LearnerStep
    from tests.test_learner_gpu import check_grads_vs_fp64
    B, T = 256, 16
    args = default_args(T, B)
    batch = geister_batch(B, T, cuda, seed=17)
    cpu_batch = {k: ({kk: vv.cpu() for kk, vv in v.items()} if isinstance(v, dict) else v.cpu())
                 for k, v in batch.items()}
    state = seeded_net().state_dict()
    res = {}
    threads = torch.get_num_threads()
    torch.set_num_threads(8)
    try:
        for dt in (torch.float32, torch.float64):
            net = seeded_net().to(dt)
            net.load_state_dict(state)
            b = {k: ({kk: vv.to(dt) for kk, vv in v.items()} if isinstance(v, dict) else
                     (v.to(dt) if v.is_floating_point() else v)) for k, v in cpu_batch.items()}
            hidden = tuple([h.to(dt) for h in hs] for hs in net.init_hidden([B, 2]))
            r = ol.CpuLearner(net, args).step(b, hidden)
            r['grads'] = {n: p.grad.double().clone() for n, p in net.named_parameters() if p.grad is not None}
            res[dt] = r
    finally:
        torch.set_num_threads(threads)
    r32, r64 = res[torch.float32], res[torch.float64]
    lib = _native.load()
    n_stats = lib.hrl_gboard_launch_stats(None, 0, 1)            # reset
    net = seeded_net()
    net.load_state_dict(state)
    init = {n: p.detach().clone() for n, p in net.named_parameters()}
    step = LearnerStep(net, args, cuda, graph=graph)
    hidden = tuple([h.to(cuda) for h in hs] for hs in net.init_hidden([B, 2]))
    out = step.step(batch, hidden)
    torch.cuda.synchronize()
    stats = (ctypes.c_int64 * n_stats)()
    lib.hrl_gboard_launch_stats(ctypes.cast(stats, ctypes.c_void_p), n_stats, 0)
    st = list(stats)
    for k in ('p', 'v', 'r', 'ent', 'total'):
        assert abs(float(out[k]) - r32[k]) <= 1e-5 * max(1.0, abs(r32[k])), (k, float(out[k]), r32[k])
    assert abs(float(out['grad_norm']) - r32['grad_norm']) <= 1e-5 * r32['grad_norm'], \
        (float(out['grad_norm']), r32['grad_norm'])
    dead = {n for (n, _), live in zip(step.net.named_parameters(), step.live) if not live}
    assert dead == set(init) - set(r32['grads'])
    got = {n: p.grad.detach().cpu().double() for n, p in step.net.named_parameters() if n not in dead}
    check_grads_vs_fp64(got, r32, r64)
    for n in dead:
        assert torch.equal(dict(step.net.named_parameters())[n].detach().cpu(), init[n]), n
    # the launch forms of the bench-size step (counted once per captured / eager launch)
    assert st[1] > 0, st                   # whole-tile launches: B = 256 games are 16 tiles, one task per workgroup
    assert st[5] > 0, st                   # the h halves' input gradient as the K-split adjoint (S = 4 groups)
    assert st[6] > 0, st                   # each repeat's h halves as one grouped launch over the layers' states
    assert st[7] > 0 and st[8] >= 3 * T, st    # weight gradients over the unroll's recorded uses (3T for the cell)
    assert st[9] > 256 and st[10] > 0, st  # > 256 tiles: workgroups carry accumulators over several tiles


@pytest.mark.gpu
@pytest.mark.parametrize('graph', [False, True])
def test_fused_update_gather_is_bit_identical(cuda, graph):
    """The recurrent unroll with step t's state update and step t+1's gather fused (train.FUSE_UPDATE_GATHER,
    nn._HiddenUpdateGather, hrl_hidden_update_gather[_backward]) against the two separate Functions: one GeisterNet
    LearnerStep (B=32, T=6) from the same weights and batch, losses and every parameter gradient bit for bit."""
    from handyrl_amd import train as htrain
    from handyrl_amd.synthetic import geister_batch, default_args
    from handyrl_amd.trainer import LearnerStep
    B, T = 32, 6
    args = default_args(T, B)
    batch = geister_batch(B, T, cuda, seed=23)
    state = seeded_net().state_dict()

    def run(fuse):
        prev = htrain.FUSE_UPDATE_GATHER
        htrain.FUSE_UPDATE_GATHER = fuse
        try:
            net = seeded_net()
            net.load_state_dict(state)
            step = LearnerStep(net, args, cuda, graph=graph)
            hidden = tuple([h.to(cuda) for h in hs] for hs in net.init_hidden([B, 2]))
            out = step.step(batch, hidden)
            torch.cuda.synchronize()
            return ({k: float(v) for k, v in out.items()},
                    {n: p.grad.detach().clone() for n, p in step.net.named_parameters() if p.grad is not None})
        finally:
            htrain.FUSE_UPDATE_GATHER = prev

    (o0, g0), (o1, g1) = run(False), run(True)
    assert o0 == o1
    assert g0.keys() == g1.keys()
    for n in g0:
        assert torch.equal(g0[n], g1[n]), n
