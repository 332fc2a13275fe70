"""HIP BatchNorm2d (csrc/hrl_bn.hip) vs torch's CPU BatchNorm2d — the reference
learner's BatchNorm (it trains on the CPU, train.py:364-385).

Forward output, running statistics, num_batches_tracked and the gradients
w.r.t. input, weight and bias, over the board shapes of the reference nets
(TicTacToe 3x3, Geister 6x6, Geese 7x11), odd row widths (scalar path) and
the BASELINE size.
"""

import numpy as np
import pytest
import torch
import torch.nn as nn

pytestmark = pytest.mark.gpu


def _pair(C, momentum=0.1, affine=True, track=True):
    from handyrl_amd.nn import BatchNorm2d
    ref = nn.BatchNorm2d(C, momentum=momentum, affine=affine, track_running_stats=track)
    if affine:
        with torch.no_grad():
            ref.weight.uniform_(0.5, 1.5)
            ref.bias.uniform_(-0.5, 0.5)
    hip = BatchNorm2d(C, momentum=momentum, affine=affine, track_running_stats=track)
    hip.load_state_dict(ref.state_dict())
    return ref, hip


@pytest.mark.parametrize('N,C,H,W', [
    (1000, 32, 3, 3),    # TicTacToe block (float4 path, 3 rows per pass)
    (37, 32, 6, 6),      # Geister board
    (13, 32, 7, 11),     # Geese board: rows wider than a workgroup (3 column slots)
    (9, 3, 3, 3),        # odd row width: scalar path
    (1, 32, 3, 3),       # single sample
    (4099, 8, 1, 1),     # 1x1 "board", many rows per pass
])
@pytest.mark.parametrize('affine', [True, False])
def test_bn_matches_torch_cpu(cuda, N, C, H, W, affine):
    torch.manual_seed(N + C)
    ref, hip = _pair(C, affine=affine)
    hip = hip.to(cuda)
    x = torch.randn(N, C, H, W) * 2 + 0.5
    dy = torch.randn(N, C, H, W)
    xr = x.clone().requires_grad_(True)
    xh = x.to(cuda).requires_grad_(True)
    for _ in range(2):  # two steps: running stats accumulate
        yr = ref(xr)
        yh = hip(xh)
    np.testing.assert_allclose(yh.detach().cpu().numpy(), yr.detach().numpy(), rtol=1e-5, atol=2e-5)
    yr.backward(dy)
    yh.backward(dy.to(cuda))
    np.testing.assert_allclose(xh.grad.cpu().numpy(), xr.grad.numpy(), rtol=1e-4, atol=1e-5)
    if affine:
        np.testing.assert_allclose(hip.weight.grad.cpu().numpy(), ref.weight.grad.numpy(), rtol=1e-4, atol=1e-4)
        np.testing.assert_allclose(hip.bias.grad.cpu().numpy(), ref.bias.grad.numpy(), rtol=1e-4, atol=1e-4)
    for k in ('running_mean', 'running_var'):
        np.testing.assert_allclose(getattr(hip, k).cpu().numpy(), getattr(ref, k).numpy(), rtol=1e-5, atol=1e-6)
    assert hip.num_batches_tracked.item() == ref.num_batches_tracked.item() == 2


def test_bn_cumulative_momentum_and_eval(cuda):
    ref, hip = _pair(16, momentum=None)
    hip = hip.to(cuda)
    for i in range(3):
        x = torch.randn(50, 16, 3, 3) + i
        ref(x)
        hip(x.to(cuda))
    np.testing.assert_allclose(hip.running_var.cpu().numpy(), ref.running_var.numpy(), rtol=1e-5, atol=1e-6)
    ref.eval(); hip.eval()
    x = torch.randn(20, 16, 3, 3)
    np.testing.assert_allclose(hip(x.to(cuda)).detach().cpu().numpy(), ref(x).detach().numpy(), rtol=1e-5, atol=1e-5)


def test_bn_baseline_size_deterministic(cuda):
    """N = B*T = 131072 TicTacToe activations: two runs bit-identical, close to torch fp64."""
    from handyrl_amd.nn import batch_norm_train
    g = torch.Generator(device=cuda).manual_seed(0)
    x = torch.randn(131072, 32, 3, 3, device=cuda, generator=g) * 3 + 1
    w = torch.rand(32, device=cuda, generator=g) + 0.5
    b = torch.randn(32, device=cuda, generator=g)
    y1 = batch_norm_train(x, w, b, None, None, 0.1, 1e-5)
    y2 = batch_norm_train(x, w, b, None, None, 0.1, 1e-5)
    assert torch.equal(y1, y2)
    ref = torch.nn.functional.batch_norm(x.double(), None, None, w.double(), b.double(), True, 0.1, 1e-5)
    assert (y1.double() - ref).abs().max().item() < 2e-5


def test_accelerate_keeps_state_dict(cuda):
    from handyrl_amd.envs.tictactoe import SimpleConv2dModel
    from handyrl_amd.nn import accelerate, BatchNorm2d, BoardConv2d
    net = SimpleConv2dModel()
    sd = {k: v.clone() for k, v in net.state_dict().items()}
    accelerate(net)
    assert sum(isinstance(m, BatchNorm2d) for m in net.modules()) == 3
    assert sum(isinstance(m, BoardConv2d) for m in net.modules()) == 6  # stem, 3 blocks, 2 heads
    from handyrl_amd.nn import Linear
    assert sum(isinstance(m, Linear) for m in net.modules()) == 2
    assert list(net.state_dict()) == list(sd)
    for k, v in net.state_dict().items():
        assert torch.equal(v, sd[k])


@pytest.mark.parametrize('cin,cout,k,H,W,bias', [
    (3, 32, 3, 3, 3, True),    # TicTacToe stem
    (32, 32, 3, 3, 3, False),  # TicTacToe block (BN follows, no bias)
    (32, 2, 1, 3, 3, True),    # TicTacToe policy head 1x1
    (5, 7, 3, 4, 4, True),     # 16-cell board
    (4, 3, 5, 3, 3, True),     # 5x5 kernel on a 3x3 board
])
def test_board_conv_matches_torch_cpu(cuda, cin, cout, k, H, W, bias):
    from handyrl_amd.nn import BoardConv2d
    torch.manual_seed(cin * cout)
    ref = nn.Conv2d(cin, cout, k, padding=k // 2, bias=bias)
    hip = BoardConv2d(cin, cout, k, padding=k // 2, bias=bias)
    hip.load_state_dict(ref.state_dict())
    hip = hip.to(cuda)
    x = torch.randn(777, cin, H, W)
    dy = torch.randn(777, cout, H, W)
    xr = x.clone().requires_grad_(True)
    xh = x.to(cuda).requires_grad_(True)
    yr, yh = ref(xr), hip(xh)
    np.testing.assert_allclose(yh.detach().cpu().numpy(), yr.detach().numpy(), rtol=1e-5, atol=1e-5)
    yr.backward(dy)
    yh.backward(dy.to(cuda))
    np.testing.assert_allclose(xh.grad.cpu().numpy(), xr.grad.numpy(), rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(hip.weight.grad.cpu().numpy(), ref.weight.grad.numpy(), rtol=1e-4, atol=1e-3)
    if bias:
        np.testing.assert_allclose(hip.bias.grad.cpu().numpy(), ref.bias.grad.numpy(), rtol=1e-4, atol=1e-3)


def test_board_conv_large_board_uses_plain_conv(cuda):
    from handyrl_amd.nn import BoardConv2d
    m = BoardConv2d(4, 4, 3, padding=1).to(cuda)
    x = torch.randn(3, 4, 6, 6, device=cuda)   # 36 cells > BOARD_MAX_CELLS
    ref = torch.nn.functional.conv2d(x, m.weight, m.bias, padding=1)
    assert torch.allclose(m(x), ref, atol=1e-5)
    assert '_board_cache' not in m.__dict__ or not m.__dict__['_board_cache']


def test_linear_chunked_weight_grad(cuda):
    from handyrl_amd.nn import Linear
    torch.manual_seed(0)
    ref = nn.Linear(18, 9)
    hip = Linear(18, 9)
    hip.load_state_dict(ref.state_dict())
    hip = hip.to(cuda)
    x = torch.randn(8192, 18)
    dy = torch.randn(8192, 9)
    xr, xh = x.clone().requires_grad_(True), x.to(cuda).requires_grad_(True)
    yr, yh = ref(xr), hip(xh)
    np.testing.assert_allclose(yh.detach().cpu().numpy(), yr.detach().numpy(), rtol=1e-5, atol=1e-5)
    yr.backward(dy)
    yh.backward(dy.to(cuda))
    np.testing.assert_allclose(xh.grad.cpu().numpy(), xr.grad.numpy(), rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(hip.weight.grad.cpu().numpy(), ref.weight.grad.numpy(), rtol=1e-4, atol=1e-3)
    np.testing.assert_allclose(hip.bias.grad.cpu().numpy(), ref.bias.grad.numpy(), rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize('N,C,H,W', [(1000, 32, 3, 3), (9, 3, 3, 3), (13, 32, 7, 11)])
def test_bn_relu_fused_matches_torch_cpu(cuda, N, C, H, W):
    torch.manual_seed(N)
    ref, hip = _pair(C)
    hip.fused_relu = True
    hip = hip.to(cuda)
    x = torch.randn(N, C, H, W) * 2 + 0.3
    dy = torch.randn(N, C, H, W)
    xr, xh = x.clone().requires_grad_(True), x.to(cuda).requires_grad_(True)
    yr = torch.relu(ref(xr))
    yh = hip(xh)
    np.testing.assert_allclose(yh.detach().cpu().numpy(), yr.detach().numpy(), rtol=1e-5, atol=2e-5)
    yr.backward(dy)
    yh.backward(dy.to(cuda))
    np.testing.assert_allclose(xh.grad.cpu().numpy(), xr.grad.numpy(), rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(hip.weight.grad.cpu().numpy(), ref.weight.grad.numpy(), rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(hip.bias.grad.cpu().numpy(), ref.bias.grad.numpy(), rtol=1e-4, atol=1e-4)


def test_fx_fusion_in_learner(cuda):
    """LearnerStep fuses the TicTacToe net's three BN->ReLU pairs and keeps the state_dict keys."""
    from handyrl_amd.envs.tictactoe import SimpleConv2dModel
    from handyrl_amd.nn import BatchNorm2d
    from handyrl_amd.synthetic import tictactoe_batch, default_args
    from handyrl_amd.trainer import LearnerStep
    net = SimpleConv2dModel()
    keys = list(net.state_dict())
    step = LearnerStep(net, default_args(9, 64), cuda)
    step.step(tictactoe_batch(64, 9, cuda, seed=0))
    assert step.fused_pairs == 6   # three BN->ReLU folds + one conv-BN chain + the two heads + chain and heads joined
    assert all(m.fused_relu for m in net.modules() if isinstance(m, BatchNorm2d))
    assert hasattr(step.net, '_hrl_heads') if hasattr(step.net, 'graph') else True
    assert list(net.state_dict()) == keys


@pytest.mark.parametrize('N', [1, 15, 16, 17, 1000, 4099])
@pytest.mark.parametrize('bias', [False, True])
def test_conv3x3_mfma_matches_torch_cpu(cuda, N, bias):
    """csrc/hrl_conv.hip (block-sparse fp32 MFMA): forward, input and weight gradients."""
    from handyrl_amd.nn import BoardConv2d
    torch.manual_seed(N)
    ref = nn.Conv2d(32, 32, 3, padding=1, bias=bias)
    hip = BoardConv2d(32, 32, 3, padding=1, bias=bias)
    hip.load_state_dict(ref.state_dict())
    hip = hip.to(cuda)
    x = torch.randn(N, 32, 3, 3)
    dy = torch.randn(N, 32, 3, 3)
    xr, xh = x.clone().requires_grad_(True), x.to(cuda).requires_grad_(True)
    yr, yh = ref(xr), hip(xh)
    np.testing.assert_allclose(yh.detach().cpu().numpy(), yr.detach().numpy(), rtol=1e-5, atol=2e-5)
    yr.backward(dy)
    yh.backward(dy.to(cuda))
    np.testing.assert_allclose(xh.grad.cpu().numpy(), xr.grad.numpy(), rtol=1e-5, atol=2e-5)
    scale = max(1.0, float(ref.weight.grad.abs().max()))
    np.testing.assert_allclose(hip.weight.grad.cpu().numpy(), ref.weight.grad.numpy(), rtol=1e-4, atol=1e-5 * scale)
    if bias:   # sums of 9N terms: tolerance relative to the largest channel sum
        bscale = max(1.0, float(ref.bias.grad.abs().max()))
        np.testing.assert_allclose(hip.bias.grad.cpu().numpy(), ref.bias.grad.numpy(), rtol=1e-4, atol=1e-5 * bscale)


@pytest.mark.parametrize('M,N', [(4096, 27), (131072, 27), (5000, 1), (70001, 256)])
def test_colsum_matches_fp64(cuda, M, N):
    from handyrl_amd.nn import _colsum
    g = torch.Generator(device=cuda).manual_seed(M)
    x = torch.randn(M, N, device=cuda, generator=g)
    got = _colsum(x)
    ref = x.double().sum(0)
    assert torch.allclose(got.double(), ref, rtol=1e-6, atol=1e-4)
    assert torch.equal(_colsum(x), got)      # deterministic


@pytest.mark.gpu
@pytest.mark.parametrize('N', [37, 4096])
@pytest.mark.parametrize('relu_in', [False, True])
def test_conv_bn_chain_matches_layer_by_layer(cuda, N, relu_in):
    """_BoardChain (BN stats in the conv epilogue, BN+ReLU in the next conv's / wgrad's
    prologue, BN-backward sums in the input-gradient epilogue, optional ReLU on the input)
    vs the same layers run one by one (HIP conv, HIP BN): output, every parameter gradient,
    the input gradient and the running statistics.  N = 37 leaves a ragged last tile."""
    from handyrl_amd.envs.tictactoe import SimpleConv2dModel
    from handyrl_amd.nn import accelerate, _ConvBNChain
    torch.manual_seed(0)
    net = accelerate(SimpleConv2dModel()).to(cuda)
    convs = [blk.conv for blk in net.blocks]
    bns = [blk.bn for blk in net.blocks]
    for b in bns:
        b.fused_relu = True
        b.weight.data.uniform_(0.5, 1.5)
        b.bias.data.uniform_(-0.2, 0.2)
    chain = _ConvBNChain(convs, bns, relu_in=relu_in)
    x = torch.randn(N, 32, 3, 3, device=cuda)
    g = torch.randn(N, 32, 3, 3, device=cuda)
    params = [p for c, b in zip(convs, bns) for p in (c.weight, b.weight, b.bias)]
    results = []
    for fused in (False, True):
        for b in bns:
            b.reset_running_stats()
        xi = x.clone().requires_grad_()
        if fused:
            y = chain(xi)
        else:
            y = torch.relu(xi) if relu_in else xi
            for c, b in zip(convs, bns):
                y = b(c(y))
        grads = torch.autograd.grad(y, [xi] + params, g)
        stats = [t.clone() for b in bns for t in (b.running_mean, b.running_var, b.num_batches_tracked)]
        results.append((y.detach(), grads, stats))
    (y0, g0, s0), (y1, g1, s1) = results
    torch.testing.assert_close(y1, y0, rtol=1e-5, atol=1e-5)
    for a, b in zip(g1, g0):
        err = float((a - b).norm() / b.norm().clamp(min=1e-12))
        assert err < 1e-5, err
    for a, b in zip(s1, s0):
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-6)


@pytest.mark.gpu
@pytest.mark.parametrize('shape', [(2048, 32, 6, 6), (37, 8, 6, 6), (5, 1, 6, 6), (64, 32, 3, 3)])
@pytest.mark.parametrize('relu', [False, True])
def test_bn_eval_matches_torch(cuda, shape, relu):
    """Inference BatchNorm (hrl_bn_forward_eval: x*alpha + beta from the running statistics)
    vs torch's eval batch_norm; tolerance 2e-6 relative (alpha/beta rounding)."""
    from handyrl_amd.nn import BatchNorm2d
    torch.manual_seed(shape[0])
    C = shape[1]
    bn = BatchNorm2d(C).to(cuda).eval()
    bn.fused_relu = relu
    bn.running_mean.uniform_(-1, 1)
    bn.running_var.uniform_(0.5, 2)
    bn.weight.data.uniform_(0.5, 1.5)
    bn.bias.data.uniform_(-0.5, 0.5)
    x = torch.randn(*shape, device=cuda) * 3
    with torch.no_grad():
        y = bn(x)
        ref = torch.nn.functional.batch_norm(x, bn.running_mean, bn.running_var, bn.weight, bn.bias, False, 0.0, bn.eps)
        if relu:
            ref = torch.relu(ref)
    torch.testing.assert_close(y, ref, rtol=2e-6, atol=2e-6)


@pytest.mark.parametrize('N', [1, 63, 64, 65, 4099])
def test_fused_heads_match_torch_cpu(cuda, N):
    """csrc/hrl_heads.hip (both TicTacToe heads in one pass, tictactoe.py:35-49) vs the heads on the
    CPU: policy/value outputs, the body-output gradient and every head parameter's gradient, on
    ragged row counts; the inference path (no autograd) gives the same outputs."""
    import copy
    from handyrl_amd.envs.tictactoe import SimpleConv2dModel
    from handyrl_amd.nn import _FusedHeads
    torch.manual_seed(N)
    net = SimpleConv2dModel()
    ref_p, ref_v = net.head_p, net.head_v
    gp, gv = copy.deepcopy(ref_p).to(cuda), copy.deepcopy(ref_v).to(cuda)
    fused = _FusedHeads(gp, gv)
    h = torch.randn(N, 32, 3, 3)
    dp, dv = torch.randn(N, 9), torch.randn(N, 1)
    hc = h.clone().requires_grad_(True)
    (ref_p(hc) * dp).sum().backward()
    (ref_v(hc) * dv).sum().backward()
    hg = h.to(cuda).requires_grad_(True)
    p, v = fused(hg)
    torch.autograd.backward([p, v], [dp.to(cuda), dv.to(cuda)])
    np.testing.assert_allclose(p.detach().cpu().numpy(), ref_p(h).detach().numpy(), rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(v.detach().cpu().numpy(), ref_v(h).detach().numpy(), rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(hg.grad.cpu().numpy(), hc.grad.numpy(), rtol=1e-5, atol=1e-5)
    tol = 2e-5 * max(1.0, (N * 9) ** 0.5)
    for (n, a), b in zip(list(ref_p.named_parameters()) + list(ref_v.named_parameters()),
                         list(gp.parameters()) + list(gv.parameters())):
        np.testing.assert_allclose(b.grad.cpu().numpy(), a.grad.numpy(), rtol=1e-4, atol=tol, err_msg=n)
    with torch.no_grad():
        p2, v2 = fused(h.to(cuda))
    assert torch.equal(p2, p.detach()) and torch.equal(v2, v.detach())


@pytest.mark.parametrize('fwd_form', [2, 1])
@pytest.mark.parametrize('N,cin,bias,binary', [(1, 3, True, True), (17, 3, True, True), (4099, 3, True, True),
                                               (50, 2, False, True), (33, 1, True, True), (4102, 3, True, False),
                                               (7, 2, True, False), (200003, 3, True, False)])
def test_stem_conv_matches_torch_cpu(cuda, N, cin, bias, binary, fwd_form):
    """csrc/hrl_stem.hip (the observation stem, tictactoe.py:57): forward (both forms: 2 = lane per channel,
    1 = fp32 MFMA) and the weight / bias gradients vs torch-CPU conv2d on ragged sample counts (rows past a
    4-row quad), 0/1 observations and real-valued inputs (the input is the observation: no input gradient)."""
    from handyrl_amd import _native
    from handyrl_amd.nn import BoardConv2d
    torch.manual_seed(N + cin)
    ref = nn.Conv2d(cin, 32, 3, padding=1, bias=bias)
    hip = BoardConv2d(cin, 32, 3, padding=1, bias=bias).to(cuda)
    hip.load_state_dict(ref.state_dict())
    x = (torch.rand(N, cin, 3, 3) < 0.5).float() if binary else torch.randn(N, cin, 3, 3)
    dy = torch.randn(N, 32, 3, 3)
    yr = ref(x)
    lib = _native.load()
    prev = lib.hrl_stem_set_fwd_form(fwd_form)
    try:
        yh = hip(x.to(cuda))
        torch.cuda.synchronize()
    finally:
        lib.hrl_stem_set_fwd_form(prev)
    np.testing.assert_allclose(yh.detach().cpu().numpy(), yr.detach().numpy(), rtol=1e-5, atol=1e-5)
    yr.backward(dy)
    yh.backward(dy.to(cuda))
    tol = 2e-5 * max(1.0, (N * 9) ** 0.5)
    np.testing.assert_allclose(hip.weight.grad.cpu().numpy(), ref.weight.grad.numpy(), rtol=1e-5, atol=tol)
    if bias:
        np.testing.assert_allclose(hip.bias.grad.cpu().numpy(), ref.bias.grad.numpy(), rtol=1e-5, atol=tol)


@pytest.mark.parametrize('M', [37, 4099, 20000])
@pytest.mark.parametrize('epi', [0, 2, 3, None])
@pytest.mark.parametrize('pro', [False, True])
@pytest.mark.parametrize('form', [2, 1, 0])
def test_block_backward_matches_unfused_launches(cuda, M, epi, pro, form):
    """hrl_conv3x3_block_backward (BN backward apply + weight gradient + input gradient of one chain block in
    one launch) vs the three launches it replaces on the same inputs: the input gradient is bit-identical
    (same split MFMA order on the same dY) in every kernel form; the weight gradient is bit-identical in the
    per-wave form (form 0) and, in the tile-shared forms (1: 8 waves, 2: two 4-wave workgroups per CU; each tap
    summed over the workgroup's tiles in one accumulator), equal to fp32 reassociation (norm-relative 1e-6); the
    epilogue-2 BatchNorm sums (hrl_conv3x3_block_sum_blocks rows) equal to fp64 rounding of a different fp32
    summation order.  epi None: no input gradient (the per-wave kernel in forms 0/1; form 2's staging and weight
    gradient alone).  M = 37 leaves a ragged last row tile (rows past the batch must contribute nothing);
    M = 20000 gives the tile-shared workgroups several tiles each."""
    from handyrl_amd import _native
    lib = _native.load()
    prev_form = lib.hrl_conv3x3_set_block_form(form)
    P = _native.ptr
    stream = _native.stream_of(cuda)
    g0 = torch.Generator(device=cuda).manual_seed(M + (epi or 7))
    rnd = lambda *s: torch.randn(*s, device=cuda, generator=g0)   # noqa: E731
    g, y, x = rnd(M, 288), rnd(M, 288), rnd(M, 288)
    w = rnd(32, 32, 3, 3) * 0.1
    gamma, beta = rnd(32).abs() + 0.5, rnd(32) * 0.2
    mean, invstd = rnd(32) * 0.1, rnd(32).abs() + 0.5
    kcoef, gmean = rnd(32) * 0.1, rnd(32) * 0.1
    alpha, bet = (rnd(32).abs() + 0.5, rnd(32) * 0.3) if pro else (None, None)
    em, ea, eb = rnd(32) * 0.1, rnd(32).abs() + 0.5, rnd(32) * 0.3
    packed = torch.empty(1, 2, 9216, device=cuda)
    _native.check(lib.hrl_conv3x3_pack_n(_native.ptr_array([w]), 1, P(packed), stream), 'pack')
    ws_bytes = lib.hrl_conv3x3_workspace_bytes(M)
    nblk = lib.hrl_conv3x3_stats_blocks(M)
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=cuda)
    # the three launches
    dy = torch.empty_like(g)
    _native.check(lib.hrl_bn_backward_apply(P(y), P(g), M, 32, 9, P(gamma), P(beta), P(mean), P(invstd), 1,
                                            P(kcoef), P(gmean), P(dy), stream), 'apply')
    dw0 = torch.empty(32, 32, 3, 3, device=cuda)
    _native.check(lib.hrl_conv3x3_wgrad_ex(P(x), P(alpha), P(bet), P(dy), M, P(dw0), P(ws), ws_bytes, stream), 'wg')
    gin0, part0 = torch.empty_like(g), torch.zeros(nblk * 64, dtype=torch.float64, device=cuda)
    if epi is not None:
        _native.check(lib.hrl_conv3x3_forward_ex(P(dy), M, None, None, P(packed[0, 1]), None, 3, P(gin0), epi,
                                                 P(x) if epi else None, P(em), P(ea), P(eb),
                                                 P(part0) if epi == 2 else None, P(ws), ws_bytes, stream), 'dg')
    # one launch
    dw1 = torch.empty_like(dw0)
    nblk1 = lib.hrl_conv3x3_block_sum_blocks(M)   # under the form set above
    gin1, part1 = torch.empty_like(g), torch.zeros(nblk1 * 64, dtype=torch.float64, device=cuda)
    _native.check(lib.hrl_conv3x3_block_backward(
        P(g), P(y), M, P(gamma), P(beta), P(mean), P(invstd), P(kcoef), P(gmean), P(x), P(alpha), P(bet),
        P(packed[0, 1]), P(dw1), P(gin1) if epi is not None else None, epi or 0, P(em), P(ea), P(eb),
        P(part1) if epi == 2 else None, P(ws), ws_bytes, stream), 'block')
    torch.cuda.synchronize(cuda)
    lib.hrl_conv3x3_set_block_form(prev_form)
    if form == 0 or (epi is None and form == 1):
        assert torch.equal(dw1, dw0)
    else:
        err = float((dw1.double() - dw0.double()).norm() / dw0.double().norm())
        assert err < 1e-6, err
    if epi is not None:
        assert torch.equal(gin1, gin0)
    if epi == 2:   # both against the fp64 sums: sum g*m and sum g*m*(x - mean), m = [x*alpha + beta > 0]
        xg, gg = x.double().view(M, 32, 9), gin0.double().view(M, 32, 9)
        m = (x.view(M, 32, 9) * ea.view(1, 32, 1) + eb.view(1, 32, 1) > 0).double()
        ref = torch.stack([(gg * m).sum((0, 2)), (gg * m * (xg - em.double().view(1, 32, 1))).sum((0, 2))], 1)
        scale = float((gg.abs() * (1 + xg.abs())).sum((0, 2)).max())
        err0 = float((part0.view(nblk, 32, 2).sum(0) - ref).abs().max()) / scale
        err1 = float((part1.view(nblk1, 32, 2).sum(0) - ref).abs().max()) / scale
        assert err1 <= max(2 * err0, 1e-7), (err1, err0)


@pytest.mark.parametrize('M', [37, 20000])
@pytest.mark.parametrize('pro', [False, True])
@pytest.mark.parametrize('form', [2, 1])
def test_block_backward_weight_gradient_exact_on_integer_data(cuda, M, pro, form):
    """The tile-shared block backward's weight gradient on small-integer data, where every product and every
    partial sum is exact in fp32: equal to the fp64 reference bit for bit (pins the dY image layout, the
    transposed reads and the x operand's prologue)."""
    from handyrl_amd import _native
    lib = _native.load()
    P = _native.ptr
    stream = _native.stream_of(cuda)
    g0 = torch.Generator(device=cuda).manual_seed(M)
    ri = lambda *s: torch.randint(-3, 4, s, device=cuda, generator=g0).float()   # noqa: E731
    g, y, x = ri(M, 288), ri(M, 288), ri(M, 288)
    one = torch.ones(32, device=cuda)
    zero = torch.zeros(32, device=cuda)
    # BN_i's backward apply is the identity on g where y*1 + 0 > 0: dY = [y > 0] * g (mean 0, k 0, gm 0, invstd 1)
    alpha, beta = (torch.full((32,), 1.0, device=cuda), torch.full((32,), -1.0, device=cuda)) if pro else (None, None)
    w = ri(32, 32, 3, 3)
    packed = torch.empty(1, 2, 9216, device=cuda)
    _native.check(lib.hrl_conv3x3_pack_n(_native.ptr_array([w]), 1, P(packed), stream), 'pack')
    ws_bytes = lib.hrl_conv3x3_workspace_bytes(M)
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=cuda)
    dw = torch.empty(32, 32, 3, 3, device=cuda)
    gin = torch.empty_like(g)
    prev = lib.hrl_conv3x3_set_block_form(form)
    _native.check(lib.hrl_conv3x3_block_backward(
        P(g), P(y), M, P(one), P(zero), P(zero), P(one), P(zero), P(zero), P(x), P(alpha), P(beta),
        P(packed[0, 1]), P(dw), P(gin), 0, None, None, None, None, P(ws), ws_bytes, stream), 'block')
    torch.cuda.synchronize(cuda)
    lib.hrl_conv3x3_set_block_form(prev)
    dy = (g * (y > 0).float()).double().view(M, 32, 3, 3).cpu()
    xin = x.double().view(M, 32, 3, 3).cpu()
    if pro:
        xin = torch.relu(xin - 1.0)
    ref = torch.nn.grad.conv2d_weight(xin, (32, 32, 3, 3), dy, padding=1)
    assert torch.equal(dw.double().cpu(), ref)
    gref = torch.nn.grad.conv2d_input(xin.shape, w.double().cpu(), dy, padding=1)
    assert torch.equal(gin.double().cpu(), gref.reshape(M, 288))


@pytest.mark.gpu
@pytest.mark.parametrize('M', [37, 20000])
@pytest.mark.parametrize('pro', [False, True])
def test_tile_shared_forward_matches_per_wave_conv(cuda, M, pro):
    """The chain's forward conv with BN statistics (hrl_conv3x3_forward_ex, epilogue 1) in the tile-shared form
    (the block backward kernel with x' staged in place of dY), the LDS-DMA ring form (2, conv3x3_fwd_dma_kernel) and
    the ping-pong ring form (3, conv3x3_fwd_pp_kernel: two wave groups alternating MFMAs and staging) vs the
    per-wave conv3x3_kernel: the output is bit-identical (the same split MFMA order on the same x'), the
    per-channel sums sum(y) and sum(y^2) agree
    with the fp64 sums to fp32 rounding of a different per-tile grouping.  Ragged M = 37 (rows past the batch
    contribute nothing) and M = 20000 (several tiles per workgroup); with and without the BN + ReLU prologue."""
    from handyrl_amd import _native
    lib = _native.load()
    P = _native.ptr
    stream = _native.stream_of(cuda)
    g0 = torch.Generator(device=cuda).manual_seed(M + 11)
    rnd = lambda *s: torch.randn(*s, device=cuda, generator=g0)   # noqa: E731
    x = rnd(M, 288)
    w = rnd(32, 32, 3, 3) * 0.1
    alpha, bet = (rnd(32).abs() + 0.5, rnd(32) * 0.3) if pro else (None, None)
    packed = torch.empty(1, 2, 9216, device=cuda)
    _native.check(lib.hrl_conv3x3_pack_n(_native.ptr_array([w]), 1, P(packed), stream), 'pack')
    ws_bytes = lib.hrl_conv3x3_workspace_bytes(M)
    nblk = lib.hrl_conv3x3_stats_blocks(M)
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=cuda)
    outs = []
    for form in (0, 1, 2, 3):
        prev = lib.hrl_conv3x3_set_fwd_form(form)
        y, part = torch.empty_like(x), torch.full((nblk * 64,), float('nan'), dtype=torch.float64, device=cuda)
        try:
            _native.check(lib.hrl_conv3x3_forward_ex(P(x), M, P(alpha), P(bet), P(packed[0, 0]), None, 2, P(y), 1,
                                                     None, None, None, None, P(part), P(ws), ws_bytes, stream), 'fwd')
            torch.cuda.synchronize(cuda)
        finally:
            lib.hrl_conv3x3_set_fwd_form(prev)
        outs.append((y, part))
    (y0, p0), (y1, p1), (y2, p2), (y3, p3) = outs
    assert torch.equal(y1, y0)
    assert torch.equal(y2, y0)
    assert torch.equal(y3, y0)
    yd = y0.double().view(M, 32, 9)
    ref = torch.stack([yd.sum((0, 2)), (yd * yd).sum((0, 2))], 1)
    scale = torch.stack([yd.abs().sum((0, 2)), (yd * yd).sum((0, 2))], 1)
    for p in (p0, p1, p2, p3):
        s = p.view(nblk, 32, 2).sum(0)
        assert bool(torch.isfinite(s).all())
        assert float(((s - ref).abs() / scale).max()) < 1e-6


@pytest.mark.parametrize('G,N,C,HW', [(16, 8, 32, 36), (2, 50, 8, 36), (64, 4, 1, 36), (200, 2, 4, 9)])
def test_grouped_batch_norm_matches_sequential_calls(cuda, G, N, C, HW):
    """nn.batch_norm_train(groups=G) (one launch per direction, the groups' statistics folded in parallel for
    G <= 128 and finalized in group order) vs G sequential calls on the row blocks: outputs, input / weight / bias
    gradients and the running statistics after all G updates, to fp64-level rounding (1e-6 relative)."""
    from handyrl_amd.nn import batch_norm_train
    g0 = torch.Generator(device=cuda).manual_seed(G * 7 + C)
    x = torch.randn(G * N, C, HW, device=cuda, generator=g0) * 2 + 0.5
    dy = torch.randn(G * N, C, HW, device=cuda, generator=g0)
    outs = []
    for grouped in (True, False):
        w = (torch.rand(C, device=cuda, generator=torch.Generator(device=cuda).manual_seed(1)) + 0.5).requires_grad_()
        b = torch.zeros(C, device=cuda, requires_grad=True)
        rm, rv = torch.zeros(C, device=cuda), torch.ones(C, device=cuda)
        xi = x.clone().requires_grad_()
        if grouped:
            y = batch_norm_train(xi, w, b, rm, rv, 0.1, 1e-5, relu=True, groups=G)
        else:
            y = torch.cat([batch_norm_train(xi[k * N:(k + 1) * N], w, b, rm, rv, 0.1, 1e-5, relu=True)
                           for k in range(G)])
        y.backward(dy)
        outs.append((y.detach(), xi.grad, w.grad, b.grad, rm, rv))
    for a, r in zip(*outs):
        scale = max(float(r.abs().max()), 1e-30)
        assert float((a - r).abs().max()) <= 1e-6 * scale


@pytest.mark.parametrize('N', [1, 37, 4099, 20000, 140001])
@pytest.mark.parametrize('bn', [False, True])
def test_heads_backward_forms_agree(cuda, N, bn):
    """hrl_heads_backward's lane-per-channel form (2, the default: accumulators in registers, the fc weight
    gradients in the same pass) against the row-per-lane form (1) on the same inputs: dh bit-identical (the same
    float operations per element), every parameter gradient and the fused BatchNorm's backward sums against the
    fp64 formulas within fp32 reassociation (different fold orders), on ragged row counts with and without the
    body's last BatchNorm + ReLU in front and the value head's tanh folded in.  N = 140001: several 32-row blocks
    per wave (the next block's first 8-row group prefetched across the block boundary)."""
    from handyrl_amd import _native
    lib = _native.load()
    P = _native.ptr
    stream = _native.stream_of(cuda)
    g0 = torch.Generator(device=cuda).manual_seed(N + 7 * bn)
    rnd = lambda *s: torch.randn(*s, device=cuda, generator=g0)   # noqa: E731
    y = rnd(N, 288)
    w1p, w1v, wp, wv = rnd(2, 32), rnd(1, 32), rnd(9, 18), rnd(1, 9)
    a_p, a_v = rnd(N, 18), rnd(N, 9)
    dp, dv = rnd(N, 9), rnd(N, 1)
    vt = torch.tanh(rnd(N, 1))
    al, be, mu = (rnd(32).abs() + 0.5, rnd(32) * 0.3, rnd(32) * 0.1) if bn else (None, None, None)
    res = []
    prev = lib.hrl_heads_set_bwd_form(1)
    try:
        for form in (1, 2):
            lib.hrl_heads_set_bwd_form(form)
            ws_bytes = lib.hrl_heads_workspace_bytes(N)
            ws = torch.empty(ws_bytes, dtype=torch.uint8, device=cuda)
            nparts = lib.hrl_heads_bn_parts(N)
            part = torch.zeros(nparts * 64, dtype=torch.float64, device=cuda)
            dh = torch.empty_like(y)
            outs = [torch.empty(2, 32, device=cuda), torch.empty(2, device=cuda), torch.empty(1, 32, device=cuda),
                    torch.empty(1, device=cuda), torch.empty(9, 18, device=cuda), torch.empty(1, 9, device=cuda)]
            _native.check(lib.hrl_heads_backward(P(y), N, P(w1p), P(w1v), P(wp), P(wv), P(al), P(be), P(mu),
                                                 P(part) if bn else None, P(a_p), P(a_v), P(dp), P(dv), P(vt), P(dh),
                                                 *[P(o) for o in outs], P(ws), ws_bytes, stream), 'heads_backward')
            torch.cuda.synchronize(cuda)
            res.append((dh, outs, part.view(nparts, 32, 2).sum(0) if bn else None))
    finally:
        lib.hrl_heads_set_bwd_form(prev)
    assert torch.equal(res[0][0], res[1][0])
    # fp64 formulas (tictactoe.py:35-49 heads; the tanh backward; bn_bwd_reduce's mask and products)
    d = lambda t: t.double().cpu()   # noqa: E731
    x = d(y).view(N, 32, 9)
    h = torch.relu(x * d(al).view(1, 32, 1) + d(be).view(1, 32, 1)) if bn else x
    gv = d(dv) * (1 - d(vt) ** 2)
    tp = d(dp) @ d(wp)
    zp = torch.where(d(a_p) > 0, tp, tp * 0.1)
    tv = gv * d(wv)
    zv = torch.where(d(a_v) > 0, tv, tv * 0.1)
    dz = torch.cat([zp.view(N, 2, 9), zv.view(N, 1, 9)], 1)              # (N, 3, 9)
    w1 = torch.cat([d(w1p), d(w1v)], 0)                                  # (3, 32)
    ref = [torch.einsum('nmq,ncq->mc', dz, h)[:2], dz[:, :2].sum((0, 2)), torch.einsum('nmq,ncq->mc', dz, h)[2:],
           dz[:, 2].sum((0, 1)).view(1), d(dp).t() @ d(a_p), (gv.t() @ d(a_v))]
    for form, (_, outs, part) in zip((1, 2), res):
        for i, (o, r) in enumerate(zip(outs, ref)):
            err = float((d(o) - r).abs().max()) / max(float(r.abs().max()), 1e-30)
            assert err < 2e-5 * max(1.0, (N / 4096) ** 0.5), (form, i, err)
        if bn:
            dhx = d(res[0][0]).view(N, 32, 9)
            m = (x * d(al).view(1, 32, 1) + d(be).view(1, 32, 1) > 0).double()
            bref = torch.stack([(dhx * m).sum((0, 2)), (dhx * m * (x - d(mu).view(1, 32, 1))).sum((0, 2))], 1)
            scale = float((dhx.abs() * (1 + x.abs())).sum((0, 2)).max())
            assert float((d(part) - bref).abs().max()) / scale < 1e-6, form


@pytest.mark.gpu
@pytest.mark.parametrize('M', [37, 20000, 131072])
@pytest.mark.parametrize('prev_rows', [None, 512])
def test_finalize_folded_into_the_consumer_is_bit_identical(cuda, M, prev_rows):
    """hrl_conv3x3_forward_bnfold / hrl_conv3x3_block_backward_bnfold (the BatchNorm finalize in the consumer kernel's
    prologue, ABI 26) vs hrl_bn_finalize_stats / _backward followed by hrl_conv3x3_forward_ex / block_backward on the
    same inputs: y, the statistics rows, the coefficients, the running statistics, the input gradient, dgamma and
    dbeta, the weight gradient -- all bit-identical.  prev_rows None: the producer's own row count
    (hrl_conv3x3_stats_blocks); 512: as many rows as the fused heads' backward writes (two per folding thread)."""
    from handyrl_amd import _native
    lib = _native.load()
    P = _native.ptr
    stream = _native.stream_of(cuda)
    g0 = torch.Generator(device=cuda).manual_seed(M + 3)
    rnd = lambda *s: torch.randn(*s, device=cuda, generator=g0)   # noqa: E731
    nblk = lib.hrl_conv3x3_stats_blocks(M)
    nprev = prev_rows or nblk
    x, g = rnd(M, 288), rnd(M, 288)
    w = rnd(32, 32, 3, 3) * 0.1
    gamma, beta = rnd(32).abs() + 0.5, rnd(32) * 0.2
    prev = (rnd(nprev, 32, 2).double() * torch.tensor([1.0, 0.0], device=cuda).double()
            + torch.stack([torch.zeros(32, device=cuda), rnd(32).abs() * 3 + 1], 1).double()) * (M * 9 / nprev)
    prev = prev.reshape(-1).contiguous()
    packed = torch.empty(1, 2, 9216, device=cuda)
    _native.check(lib.hrl_conv3x3_pack_n(_native.ptr_array([w]), 1, P(packed), stream), 'pack')
    ws_bytes = lib.hrl_conv3x3_workspace_bytes(M)
    outs = []
    for fused in (False, True):
        ws = torch.empty(ws_bytes, dtype=torch.uint8, device=cuda)
        rm, rv = torch.full((32,), 0.1, device=cuda), torch.full((32,), 0.9, device=cuda)
        coef = torch.empty(4, 32, device=cuda)
        y, part = torch.empty_like(x), torch.zeros(nblk * 64, dtype=torch.float64, device=cuda)
        if fused:
            _native.check(lib.hrl_conv3x3_forward_bnfold(P(x), M, P(prev), nprev, P(gamma), P(beta), P(rm), P(rv),
                                                         0.1, 1e-5, P(coef[0]), P(coef[1]), P(coef[2]), P(coef[3]),
                                                         P(packed[0, 0]), P(y), P(part), P(ws), ws_bytes, stream),
                          'fwd fold')
        else:
            _native.check(lib.hrl_bn_finalize_stats(P(prev), nprev, 32, M * 9, P(gamma), P(beta), P(rm), P(rv), 0.1,
                                                    1e-5, P(coef[0]), P(coef[1]), P(coef[2]), P(coef[3]), stream),
                          'fin')
            _native.check(lib.hrl_conv3x3_forward_ex(P(x), M, P(coef[2]), P(coef[3]), P(packed[0, 0]), None, 2, P(y),
                                                     1, None, None, None, None, P(part), P(ws), ws_bytes, stream),
                          'fwd')
        # the backward of the same block with BN_i's sums = prev (its rows as the consumer's sums)
        kg, dgb = torch.empty(2, 32, device=cuda), torch.empty(2, 32, device=cuda)
        dw, gin = torch.empty(32, 32, 3, 3, device=cuda), torch.empty_like(g)
        epart = torch.zeros(lib.hrl_conv3x3_block_sum_blocks(M) * 64, dtype=torch.float64, device=cuda)
        args = (P(g), P(y), M, P(gamma), P(beta), P(coef[0]), P(coef[1]))
        tail = (P(x), P(coef[2]), P(coef[3]), P(packed[0, 1]), P(dw), P(gin), 2, P(coef[0]), P(coef[2]), P(coef[3]),
                P(epart), P(ws), ws_bytes, stream)
        if fused:
            _native.check(lib.hrl_conv3x3_block_backward_bnfold(*args, P(prev), nprev, P(dgb[0]), P(dgb[1]), P(kg[0]),
                                                                P(kg[1]), *tail), 'bwd fold')
        else:
            _native.check(lib.hrl_bn_finalize_backward(P(prev), nprev, 32, M * 9, P(gamma), P(coef[1]), P(dgb[0]),
                                                       P(dgb[1]), P(kg[0]), P(kg[1]), stream), 'fin bwd')
            _native.check(lib.hrl_conv3x3_block_backward(*args, P(kg[0]), P(kg[1]), *tail), 'bwd')
        torch.cuda.synchronize(cuda)
        outs.append((y, part, coef, rm, rv, kg, dgb, dw, gin, epart))
    for a, b in zip(*outs):
        assert torch.equal(a, b)
    assert bool(torch.isfinite(outs[1][1]).all()) and bool(torch.isfinite(outs[1][8]).all())


@pytest.mark.gpu
@pytest.mark.parametrize('N', [37, 4096])
@pytest.mark.parametrize('relu_in', [False, True])
def test_chain_with_folded_finalizes_is_bit_identical(cuda, N, relu_in):
    """The TicTacToe body chain (_ConvBNChain -> _chain_forward / _chain_backward) with nn.FOLD_BN on (the finalizes
    in the consumers' prologues) and off (their own launches): output, input gradient, every parameter gradient and
    the running statistics bit-identical."""
    from handyrl_amd import nn as hnn
    from handyrl_amd.envs.tictactoe import SimpleConv2dModel
    from handyrl_amd.nn import accelerate, _ConvBNChain
    torch.manual_seed(1)
    net = accelerate(SimpleConv2dModel()).to(cuda)
    convs = [blk.conv for blk in net.blocks]
    bns = [blk.bn for blk in net.blocks]
    for b in bns:
        b.fused_relu = True
        b.weight.data.uniform_(0.5, 1.5)
        b.bias.data.uniform_(-0.2, 0.2)
    chain = _ConvBNChain(convs, bns, relu_in=relu_in)
    x = torch.randn(N, 32, 3, 3, device=cuda)
    g = torch.randn(N, 32, 3, 3, device=cuda)
    params = [p for c, b in zip(convs, bns) for p in (c.weight, b.weight, b.bias)]
    results = []
    prev = hnn.FOLD_BN
    try:
        for fold in (False, True):
            hnn.FOLD_BN = fold
            for b in bns:
                b.reset_running_stats()
            xi = x.clone().requires_grad_()
            y = chain(xi)
            grads = torch.autograd.grad(y, [xi] + params, g)
            stats = [t.clone() for b in bns for t in (b.running_mean, b.running_var)]
            results.append([y.detach()] + list(grads) + stats)
    finally:
        hnn.FOLD_BN = prev
    for a, b in zip(*results):
        assert torch.equal(a, b)
