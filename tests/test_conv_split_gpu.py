"""Split-bf16 arithmetic of the board and torus convs (csrc/hrl_conv.hip, csrc/hrl_torus.hip; *_set_split).

The forward / input-gradient kernel splits both fp32 operands exactly into three bf16 parts and
runs six partial products on v_mfma_f32_16x16x32_bf16 with fp32 accumulation.  Checked here:
  * integer data (every product and partial sum exact in fp32) gives exactly the fp64 result,
    so the bf16 fragment layouts (k order of A and B, both column tiles, every tap) are right;
  * on random data the error against an fp64 reference is no larger than torch's own fp32
    conv's error (tolerance: 2x torch-CPU fp32's max error, measured on the same data);
  * the fp32-MFMA form (split off) gives the same results within the same bound.
"""

import pytest
import torch

from handyrl_amd import _native

pytestmark = pytest.mark.gpu


@pytest.fixture
def cuda():
    if not torch.cuda.is_available():
        pytest.skip('no GPU')
    return torch.device('cuda', 0)


def _run(lib, dev, x, w, b, flip, split):
    M = x.shape[0]
    y = torch.empty_like(x)
    ws_bytes = lib.hrl_conv3x3_workspace_bytes(M)
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
    prev = lib.hrl_conv3x3_set_split(split)
    try:
        P = _native.ptr
        _native.check(lib.hrl_conv3x3_forward(P(x), M, 32, 32, P(w), P(b) if b is not None else None, flip, P(y),
                                              P(ws), ws_bytes, _native.stream_of(dev)), 'conv')
        torch.cuda.synchronize(dev)
    finally:
        lib.hrl_conv3x3_set_split(prev)
    return y


def _ref64(x, w, b, flip):
    M = x.shape[0]
    x64, w64 = x.double().cpu().view(M, 32, 3, 3), w.double().cpu()
    if flip:   # input gradient: the adjoint of the 'same' conv
        return torch.nn.grad.conv2d_input((M, 32, 3, 3), w64, x64, padding=1).view(M, 288)
    return torch.nn.functional.conv2d(x64, w64, None if b is None else b.double().cpu(), padding=1).view(M, 288)


@pytest.mark.parametrize('flip', [0, 1])
@pytest.mark.parametrize('split', [1, 0])
def test_integer_data_is_exact(cuda, flip, split):
    lib = _native.load()
    g = torch.Generator().manual_seed(3 + flip)
    M = 1000
    x = torch.randint(-8, 9, (M, 288), generator=g).float()
    w = torch.randint(-8, 9, (32, 32, 3, 3), generator=g).float()
    b = None if flip else torch.randint(-8, 9, (32,), generator=g).float()
    y = _run(lib, cuda, x.to(cuda), w.to(cuda), None if b is None else b.to(cuda), flip, split)
    assert torch.equal(y.cpu().double(), _ref64(x, w, b, flip))


@pytest.mark.parametrize('flip', [0, 1])
@pytest.mark.parametrize('M', [17, 4099])
def test_error_within_fp32_conv_error(cuda, flip, M):
    lib = _native.load()
    g = torch.Generator().manual_seed(M + flip)
    # wide dynamic range: per-row scales over 2^-20 .. 2^20, a few exact zeros and negative zeros
    x = torch.randn(M, 288, generator=g) * torch.exp2(torch.randint(-20, 21, (M, 1), generator=g).float())
    x[::7, ::5] = 0.0
    x[1::7, ::11] = -0.0
    w = torch.randn(32, 32, 3, 3, generator=g) * 0.1
    b = None if flip else torch.randn(32, generator=g)
    ref = _ref64(x, w, b, flip)
    M_ = x.shape[0]
    if flip:
        t32 = torch.nn.grad.conv2d_input((M_, 32, 3, 3), w, x.view(M_, 32, 3, 3), padding=1).view(M_, 288)
    else:
        t32 = torch.nn.functional.conv2d(x.view(M_, 32, 3, 3), w, b, padding=1).view(M_, 288)
    # per-row error relative to the row's largest output (rows span 40 binades)
    rowmax = ref.abs().amax(dim=1, keepdim=True).clamp_min(1e-300)
    bound = 2.0 * float(((t32.double() - ref).abs() / rowmax).max()) + 1e-7
    for split in (1, 0):
        y = _run(lib, cuda, x.to(cuda), w.to(cuda), None if b is None else b.to(cuda), flip, split).cpu().double()
        err = float(((y - ref).abs() / rowmax).max())
        assert err <= bound, (split, err, bound)


def _torus64(x, w, b):
    """GeeseNet's TorusConv2d (hungry_geese.py:30-35: wrap with two cats, 'valid' conv) in fp64."""
    xp = torch.cat([x[:, :, -1:], x, x[:, :, :1]], dim=2)
    xp = torch.cat([xp[:, :, :, -1:], xp, xp[:, :, :, :1]], dim=3)
    return torch.nn.functional.conv2d(xp, w, b)


@pytest.mark.parametrize('cin', [32, 17])
@pytest.mark.parametrize('integer', [True, False])
def test_torus_split_matches_fp64(cuda, cin, integer):
    """csrc/hrl_torus.hip's split forward: exact on integer data (fragment layouts, the 17-channel stem's zero
    padding to one 32-deep k-step), and within 2x torch fp32's error on random data; both arithmetics."""
    lib = _native.load()
    g = torch.Generator().manual_seed(cin + integer)
    N, H, W = 300, 7, 11
    if integer:
        x = torch.randint(-8, 9, (N, cin, H, W), generator=g).float()
        w = torch.randint(-8, 9, (32, cin, 3, 3), generator=g).float()
        b = torch.randint(-8, 9, (32,), generator=g).float()
    else:
        x = torch.randn(N, cin, H, W, generator=g) * torch.exp2(torch.randint(-20, 21, (N, 1, 1, 1), generator=g).float())
        w = torch.randn(32, cin, 3, 3, generator=g) * 0.1
        b = torch.randn(32, generator=g)
    ref = _torus64(x.double(), w.double(), b.double())
    t32 = _torus64(x, w, b).double()
    rowmax = ref.abs().flatten(1).amax(dim=1).clamp_min(1e-300).view(N, 1, 1, 1)
    bound = 2.0 * float(((t32 - ref).abs() / rowmax).max()) + 1e-7
    ws_bytes = lib.hrl_torus_workspace_bytes(N)
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=cuda)
    P = _native.ptr
    for split in (1, 0):
        xg, wg, bg = x.to(cuda), w.to(cuda), b.to(cuda)
        y = torch.empty(N, 32, H, W, device=cuda)
        prev = lib.hrl_torus_set_split(split)
        try:
            _native.check(lib.hrl_torus_conv_forward(P(xg), N, cin, 32, H, W, P(wg), P(bg), 0, P(y), None, None,
                                                     None, P(ws), ws_bytes, _native.stream_of(cuda)), 'torus')
            torch.cuda.synchronize(cuda)
        finally:
            lib.hrl_torus_set_split(prev)
        yd = y.cpu().double()
        if integer:
            assert torch.equal(yd, ref), split
        else:
            err = float(((yd - ref).abs() / rowmax).max())
            assert err <= bound, (split, err, bound)


def _wgrad(lib, dev, x, dy, split, alpha=None, beta=None):
    M = x.shape[0]
    dw = torch.empty(32, 32, 3, 3, device=dev)
    ws_bytes = lib.hrl_conv3x3_workspace_bytes(M)
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
    prev = lib.hrl_conv3x3_set_split(split)
    try:
        P = _native.ptr
        _native.check(lib.hrl_conv3x3_wgrad_ex(P(x), P(alpha) if alpha is not None else None,
                                               P(beta) if beta is not None else None, P(dy), M, P(dw), P(ws),
                                               ws_bytes, _native.stream_of(dev)), 'wgrad')
        torch.cuda.synchronize(dev)
    finally:
        lib.hrl_conv3x3_set_split(prev)
    return dw


def _wgrad_ref64(x, dy, alpha=None, beta=None):
    M = x.shape[0]
    x64 = x.double().cpu().view(M, 32, 3, 3)
    if alpha is not None:   # the fused prologue: relu(x*alpha + beta) per input channel
        x64 = torch.relu(x64 * alpha.double().cpu().view(1, 32, 1, 1) + beta.double().cpu().view(1, 32, 1, 1))
    return torch.nn.grad.conv2d_weight(x64, (32, 32, 3, 3), dy.double().cpu().view(M, 32, 3, 3), padding=1)


@pytest.mark.parametrize('pro', [False, True])
@pytest.mark.parametrize('split', [1, 0])
@pytest.mark.parametrize('M', [1000, 4099])
def test_wgrad_integer_data_is_exact(cuda, pro, split, M):
    """conv3x3_wgrad_split_kernel (32x32x16 bf16 MFMA, one tap = one tile): exact on integer data, so the
    A/B/C fragment layouts, every tap and the ragged last row tile are right; the fp32 form likewise."""
    lib = _native.load()
    g = torch.Generator().manual_seed(11 + M)
    x = torch.randint(-4, 5, (M, 288), generator=g).float()
    dy = torch.randint(-4, 5, (M, 288), generator=g).float()
    alpha = beta = None
    if pro:
        alpha = torch.randint(1, 3, (32,), generator=g).float()
        beta = torch.randint(-2, 3, (32,), generator=g).float()
    dw = _wgrad(lib, cuda, x.to(cuda), dy.to(cuda), split, None if alpha is None else alpha.to(cuda),
                None if beta is None else beta.to(cuda))
    assert torch.equal(dw.cpu().double(), _wgrad_ref64(x, dy, alpha, beta))


def test_wgrad_error_within_fp32_error(cuda):
    """On random data the split weight gradient's error against fp64 is within 2x torch-CPU fp32's."""
    lib = _native.load()
    g = torch.Generator().manual_seed(5)
    M = 8192
    x = torch.randn(M, 288, generator=g)
    dy = torch.randn(M, 288, generator=g) * torch.exp(torch.randn(M, 1, generator=g) * 3)
    ref = _wgrad_ref64(x, dy)
    t32 = torch.nn.grad.conv2d_weight(x.view(M, 32, 3, 3), (32, 32, 3, 3), dy.view(M, 32, 3, 3), padding=1)
    scale = ref.abs().max()
    bound = 2 * float((t32.double() - ref).abs().max() / scale)
    for split in (1, 0):
        dw = _wgrad(lib, cuda, x.to(cuda), dy.to(cuda), split).cpu().double()
        err = float((dw - ref).abs().max() / scale)
        assert err <= bound, (split, err, bound)


@pytest.mark.parametrize('split', [1, 0])
@pytest.mark.parametrize('N,H,W', [(300, 7, 11), (57, 4, 5), (33, 8, 10)])
def test_torus_wgrad_integer_data_is_exact(cuda, split, N, H, W):
    """torus_wgrad_split_kernel (32x32x16 bf16, X split once per sample into LDS, one tap = one tile) and the
    fp32 form: exact on integer data against fp64, so the fragment layouts, the neighbour gathers, the cells
    past the board and the bias sum are right."""
    lib = _native.load()
    g = torch.Generator().manual_seed(N + H)
    x = torch.randint(-4, 5, (N, 32, H, W), generator=g).float()
    dy = torch.randint(-4, 5, (N, 32, H, W), generator=g).float()
    xr = x.double().requires_grad_(False)
    w64 = torch.zeros(32, 32, 3, 3, dtype=torch.float64, requires_grad=True)
    b64 = torch.zeros(32, dtype=torch.float64, requires_grad=True)
    _torus64(xr, w64, b64).backward(dy.double())
    ws_bytes = lib.hrl_torus_workspace_bytes(N)
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=cuda)
    dw = torch.empty(32, 32, 3, 3, device=cuda)
    db = torch.empty(32, device=cuda)
    P = _native.ptr
    xg, dyg = x.to(cuda), dy.to(cuda)   # held: a temporary's block could be reused by the next copy
    prev = lib.hrl_torus_set_split(split)
    try:
        _native.check(lib.hrl_torus_conv_wgrad(P(xg), P(dyg), N, 32, 32, H, W, P(dw), P(db), P(ws),
                                               ws_bytes, _native.stream_of(cuda)), 'torus wgrad')
        torch.cuda.synchronize(cuda)
    finally:
        lib.hrl_torus_set_split(prev)
    assert torch.equal(dw.cpu().double(), w64.grad)
    assert torch.equal(db.cpu().double(), b64.grad)


@pytest.mark.parametrize('split', [1, 0])
@pytest.mark.parametrize('N,H,W,Cout,cin_total,ci0', [(37, 6, 6, 128, 64, 32), (300, 6, 6, 384, 32, 0),
                                                      (5, 3, 5, 32, 32, 0), (9, 8, 10, 64, 96, 64),
                                                      (2, 2, 2, 32, 32, 0)])
def test_board_conv_integer_data_is_exact(cuda, split, N, H, W, Cout, cin_total, ci0):
    """hrl_board_conv_forward (the torus kernel with zero padding, 3 or 5 cell tiles, 32-channel output chunks,
    a channel slice of the weight): exact against fp64 on integer data, both arithmetics."""
    from handyrl_amd.nn import board_conv_forward
    lib = _native.load()
    g = torch.Generator().manual_seed(N + Cout + ci0)
    x = torch.randint(-4, 5, (N, 32, H, W), generator=g).float()
    w = torch.randint(-4, 5, (Cout, cin_total, 3, 3), generator=g).float()
    b = torch.randint(-4, 5, (Cout,), generator=g).float()
    ref = torch.nn.functional.conv2d(x.double(), w[:, ci0:ci0 + 32].double(), b.double(), padding=1)
    prev = lib.hrl_torus_set_split(split)
    try:
        y = board_conv_forward(x.to(cuda), w.to(cuda), b.to(cuda), ci0)
        torch.cuda.synchronize(cuda)
    finally:
        lib.hrl_torus_set_split(prev)
    assert torch.equal(y.cpu().double(), ref)


def test_board_conv_error_within_fp32_error(cuda):
    """Random data, 6x6 (GeisterNet's h half): within 2x torch-CPU fp32's error against fp64."""
    from handyrl_amd.nn import board_conv_forward
    g = torch.Generator().manual_seed(7)
    x = torch.randn(257, 32, 6, 6, generator=g)
    w = torch.randn(128, 64, 3, 3, generator=g) * 0.1
    ref = torch.nn.functional.conv2d(x.double(), w[:, 32:].double(), None, padding=1)
    t32 = torch.nn.functional.conv2d(x, w[:, 32:], None, padding=1).double()
    scale = ref.abs().max()
    bound = 2 * float((t32 - ref).abs().max() / scale) + 1e-7
    y = board_conv_forward(x.to(cuda), w.to(cuda), None, 32).cpu().double()
    assert float((y - ref).abs().max() / scale) <= bound
