"""GeisterNet's board convolutions on csrc/hrl_gboard.hip (games as MFMA rows, exact bf16 split).

Checked against the fp64 convolution of the same inputs (torch CPU, double):
  * integer data (every product and partial sum exact in fp32) gives exactly the fp64 result, which pins the
    split fragment layouts, every tap of every cell, the zero padding and the channel / group addressing;
  * random data: max error within 4x the larger of torch-CPU fp32's and the vendor GPU convolution's (the
    F.conv2d it replaces) max errors on the same data: fp32-accurate.  The split products accumulate into one
    fp32 accumulator per output in (cell, k-step, part) order (6 adds per (cell, tap) pair, up to 108 for the
    64-channel head), measured at 1.4-2.8x torch-CPU's error and 1.5-2.3x the vendor convolution's;
  * the remaining checks bound the error by 4e-6 of the output's scale (max |y|, about 32 ulps);
  * every shape GeisterNet uses (stem 25 -> 32 + BatchNorm/ReLU epilogue, x halves 32 -> 384, grouped h halves
    96 -> 384 in 3 groups from a channel slice, move head [h_e, h_last] 64 -> 8 from two sources), a ragged
    game count, and the packed buffer refreshed in place.
"""

import pytest
import torch
import torch.nn.functional as F

from handyrl_amd import nn as hnn

pytestmark = pytest.mark.gpu


@pytest.fixture
def cuda():
    if not torch.cuda.is_available():
        pytest.skip('no GPU')
    return torch.device('cuda', 0)


def _close(y, ref):
    return (y - ref).abs().max().item() <= 4e-6 * ref.abs().max().item()


def _ref(x, w, groups, bias=None, alpha=None, beta=None, relu=False):
    y = F.conv2d(x.double().cpu(), w.double().cpu(), None if bias is None else bias.double().cpu(), padding=1,
                 groups=groups)
    if alpha is not None:
        y = y * alpha.double().cpu()[None, :, None, None] + beta.double().cpu()[None, :, None, None]
    if relu:
        y = y.clamp_min(0)
    return y


CASES = [  # (N, Cin_g, Cout, groups)
    (37, 25, 32, 1),     # stem (ragged channel k-step, ragged games)
    (64, 32, 384, 1),    # the cells' x halves
    (48, 32, 384, 3),    # grouped h halves
    (16, 32, 16, 1),
    (33, 64, 8, 1),      # move head (two k-steps, 8 of 16 channels stored)
]


@pytest.mark.parametrize('N,cin,cout,groups', CASES)
def test_gboard_integer_data_is_exact(cuda, N, cin, cout, groups):
    g = torch.Generator().manual_seed(N + cout)
    x = torch.randint(-8, 9, (N, cin * groups, 6, 6), generator=g).float()
    w = torch.randint(-8, 9, (cout, cin, 3, 3), generator=g).float()
    b = torch.randint(-4, 5, (cout,), generator=g).float()
    pk = hnn.gboard_pack(w.to(cuda))
    y = hnn.gboard_conv(x.to(cuda), pk, cout, cin, groups, bias=b.to(cuda))
    ref = _ref(x, w, groups, b)
    assert torch.equal(y.cpu().double(), ref)


@pytest.mark.parametrize('N,cin,cout,groups', CASES)
def test_gboard_random_data_fp32_accurate(cuda, N, cin, cout, groups):
    g = torch.Generator().manual_seed(7 * N + cout)
    x = torch.randn(N, cin * groups, 6, 6, generator=g)
    w = torch.randn(cout, cin, 3, 3, generator=g) * 0.2
    pk = hnn.gboard_pack(w.to(cuda))
    y = hnn.gboard_conv(x.to(cuda), pk, cout, cin, groups).cpu().double()
    ref = _ref(x, w, groups)
    err = (y - ref).abs().max().item()
    err32 = (F.conv2d(x, w, padding=1, groups=groups).double() - ref).abs().max().item()
    err_dev = (F.conv2d(x.to(cuda), w.to(cuda), padding=1, groups=groups).cpu().double() - ref).abs().max().item()
    assert err <= 4 * max(err32, err_dev) + 1e-7, (err, err32, err_dev)


def test_gboard_epilogue_slices_and_two_sources(cuda):
    """The stem's BatchNorm + ReLU epilogue, the h halves read from a channel slice of the stacked state
    (game stride 96*36) and the move head's two-source input, all against the fp64 reference."""
    g = torch.Generator().manual_seed(3)
    N = 50
    # stem + BN/ReLU
    x = torch.randn(N, 25, 6, 6, generator=g)
    w = torch.randn(32, 25, 3, 3, generator=g) * 0.2
    al, be = torch.rand(32, generator=g) + 0.5, torch.randn(32, generator=g)
    y = hnn.gboard_conv(x.to(cuda), hnn.gboard_pack(w.to(cuda)), 32, 25, alpha=al.to(cuda), beta=be.to(cuda),
                        relu=True).cpu().double()
    ref = _ref(x, w, 1, alpha=al, beta=be, relu=True)
    assert _close(y, ref)
    # the move head: [h_e, h_last] with h_last a channel slice of the (N, 96, 6, 6) stacked state
    he = torch.randn(N, 32, 6, 6, generator=g)
    st = torch.randn(N, 96, 6, 6, generator=g)
    wh = torch.randn(8, 64, 3, 3, generator=g) * 0.2
    st_d = st.to(cuda)
    y = hnn.gboard_conv(he.to(cuda), hnn.gboard_pack(wh.to(cuda)), 8, 64, x2=st_d[:, 64:96]).cpu().double()
    ref = _ref(torch.cat([he, st[:, 64:96]], 1), wh, 1)
    assert _close(y, ref)
    # grouped conv on the slice st[:, 0:96] of a wider tensor (game stride 128*36)
    wide = torch.randn(N, 128, 6, 6, generator=g)
    wg = torch.randn(384, 32, 3, 3, generator=g) * 0.2
    y = hnn.gboard_conv(wide.to(cuda)[:, :96], hnn.gboard_pack(wg.to(cuda)), 384, 32, 3).cpu().double()
    ref = _ref(wide[:, :96], wg, 3)
    assert _close(y, ref)


def test_gboard_pack_refreshes_in_place(cuda):
    g = torch.Generator().manual_seed(5)
    x = torch.randn(20, 32, 6, 6, generator=g).to(cuda)
    w1, w2 = (torch.randn(64, 32, 3, 3, generator=g).to(cuda) for _ in range(2))
    pk = hnn.gboard_pack(w1)
    ptr = pk.data_ptr()
    hnn.gboard_pack(w2, out=pk)
    assert pk.data_ptr() == ptr
    y = hnn.gboard_conv(x, pk, 64, 32).cpu().double()
    assert _close(y, _ref(x.cpu(), w2.cpu(), 1))


def test_gboard_rejects_bad_shapes(cuda):
    from handyrl_amd import _native
    lib = _native.load()
    assert lib.hrl_gboard_pack_bytes(32, 65) < 0
    x = torch.zeros(4, 96, 6, 6, device=cuda)
    pk = hnn.gboard_pack(torch.zeros(40, 32, 3, 3, device=cuda))
    with pytest.raises(ValueError):   # 40 / 2 groups = 20 channels per group: not a multiple of 16
        hnn.gboard_conv(x[:, :64], pk, 40, 32, groups=2)


@pytest.mark.parametrize('O,C1,C2', [(4, 8, 0), (2, 32, 32), (1, 25, 0), (8, 64, 64)])
def test_gboard_pointwise_matches_conv1x1(cuda, O, C1, C2):
    """hrl_gboard_pointwise == F.conv2d(cat([x1, x2]), w) (1x1, fp32 on the CPU) with the optional BatchNorm apply
    and ReLU; x2 a channel slice of a wider tensor, as the heads read h_last from the stacked state."""
    g = torch.Generator().manual_seed(O * 100 + C1 + C2)
    N = 37
    x1 = torch.randn(N, C1, 6, 6, generator=g)
    wide = torch.randn(N, C2 + 16, 6, 6, generator=g)
    x2 = wide[:, 8:8 + C2]
    w = torch.randn(O, C1 + C2, 1, 1, generator=g)
    al, be = torch.rand(O, generator=g) + 0.5, torch.randn(O, generator=g)
    ref = F.conv2d(torch.cat([x1, x2], 1) if C2 else x1, w).double()
    y = hnn.gboard_pointwise(x1.to(cuda), w.to(cuda), x2=wide.to(cuda)[:, 8:8 + C2] if C2 else None).cpu().double()
    assert _close(y, ref)
    y = hnn.gboard_pointwise(x1.to(cuda), w.to(cuda), x2=wide.to(cuda)[:, 8:8 + C2] if C2 else None,
                             alpha=al.to(cuda), beta=be.to(cuda), relu=True).cpu().double()
    ref = (ref * al.double()[None, :, None, None] + be.double()[None, :, None, None]).clamp_min(0)
    assert _close(y, ref)


@pytest.mark.parametrize('N,cout_fwd,ci0,cin', [(37, 128, 32, 32), (64, 128, 0, 32), (20, 32, 0, 25), (33, 8, 0, 64)])
def test_gboard_adjoint_matches_conv_input_gradient(cuda, N, cout_fwd, ci0, cin):
    """hrl_gboard_pack_adjoint + hrl_gboard_forward == the input gradient of F.conv2d(x, w[:, ci0:ci0+cin], padding=1)
    (fp64 reference): the ConvLSTM cells' h-half input gradient (128 -> 32, four k-steps), a stem-like ragged slice
    and the move head's 8 -> 64."""
    g = torch.Generator().manual_seed(N + cout_fwd + ci0)
    w = torch.randn(cout_fwd, ci0 + cin + 3, 3, 3, generator=g) * 0.2
    dy = torch.randn(N, cout_fwd, 6, 6, generator=g)
    wv = w[:, ci0:ci0 + cin].double()
    x = torch.zeros(N, cin, 6, 6, dtype=torch.float64, requires_grad=True)
    F.conv2d(x, wv, padding=1).backward(dy.double())
    ref = x.grad
    pk = hnn.gboard_pack_adjoint(w.to(cuda), ci0, cin)
    y = hnn.gboard_conv(dy.to(cuda), pk, cin, cout_fwd).cpu().double()
    assert _close(y, ref)


@pytest.mark.parametrize('cout,cin_total,ci0,cin,ns,bias', [
    (128, 64, 32, 32, (37, 256, 5), True),      # a ConvLSTM cell's h half: three recorded uses, ragged
    (128, 64, 0, 32, (4096,), True),            # its x half over a whole unroll (T*N games at once)
    (32, 25, 0, 25, (300,), False),             # the stem: 25 input planes (a padded channel tile)
    (8, 64, 0, 64, (17, 100), False),           # the move head's 64 -> 8 (a padded output tile)
    (128, 64, 32, 32, (2,) * 24 + (5,), True),  # many tiny records (the learner's liveness probe): one partial
                                                # per record tile, far more than sum(ns) / 16
    (128, 64, 32, 32, (300,) * 20, True),       # 380 tiles over 256 workgroups: accumulators carried across
                                                # tiles, the segment search restarting inside a workgroup's range
    (128, 64, 32, 32, (512,) * 40, True),       # 1,280 tiles in 40 segments (the bench learner's h halves: 48 x 16)
    (32, 25, 0, 25, (4100, 3000), False),       # the stem over a whole unroll and more: 445 ragged tiles
])
@pytest.mark.parametrize('integer', [True, False])
def test_gboard_wgrad_matches_conv_weight_gradient(cuda, cout, cin_total, ci0, cin, ns, bias, integer):
    """hrl_gboard_wgrad (games as the MFMA K, every recorded use in one launch, no concatenation) ADDS the weight
    (and bias) gradient of F.conv2d(x_i, w[:, ci0:ci0+cin], padding=1) summed over the records into the slice of
    an existing gradient: exactly the fp64 sum on integer data (pins the image layouts, every (cell, tap) pair,
    the padded channel tiles, ragged game counts and the segment table), within 4e-6 of the gradient's scale on
    random data; the rest of the gradient tensor is untouched."""
    g = torch.Generator().manual_seed(cout * 7 + cin + len(ns) + int(integer))
    mk = ((lambda *s: torch.randint(-3, 4, s, generator=g).float()) if integer else
          (lambda *s: torch.randn(*s, generator=g)))
    w = torch.nn.Parameter(torch.zeros(cout, cin_total, 3, 3, device=cuda))
    b = torch.nn.Parameter(torch.zeros(cout, device=cuda)) if bias else None
    w.grad = mk(cout, cin_total, 3, 3).to(cuda)          # an existing gradient: the kernel adds into its slice
    before = w.grad.clone()
    if b is not None:
        b.grad = mk(cout).to(cuda)
        bbefore = b.grad.clone()
    rec = [(mk(n, cin, 6, 6).to(cuda), mk(n, cout, 6, 6).to(cuda)) for n in ns]
    sl = None if (ci0 == 0 and cin == cin_total) else (ci0, ci0 + cin)
    hnn.gboard_wgrad(rec, w, b, sl)
    torch.cuda.synchronize(cuda)
    X = torch.cat([r[0] for r in rec]).double().cpu()
    DY = torch.cat([r[1] for r in rec]).double().cpu()
    dw = torch.nn.grad.conv2d_weight(X, (cout, cin, 3, 3), DY, padding=1)
    ref = before.double().cpu()
    ref[:, ci0:ci0 + cin] += dw
    got = w.grad.double().cpu()
    if integer:
        assert torch.equal(got, ref)
    else:
        assert (got - ref).abs().max().item() <= 4e-6 * dw.abs().max().item()
        outside = torch.ones(cin_total, dtype=torch.bool)
        outside[ci0:ci0 + cin] = False
        assert torch.equal(got[:, outside], before.double().cpu()[:, outside])
    if b is not None:
        bref = bbefore.double().cpu() + DY.sum((0, 2, 3))
        if integer:
            assert torch.equal(b.grad.double().cpu(), bref)
        else:
            assert (b.grad.double().cpu() - bref).abs().max().item() <= 4e-6 * DY.abs().sum((0, 2, 3)).max().item()


@pytest.mark.parametrize('N,cout_fwd,ci0,cin', [(37, 128, 32, 32), (256, 128, 32, 32), (20, 64, 0, 32),
                                                (9, 96, 16, 48)])
def test_gboard_adjoint_split_matches_conv_input_gradient(cuda, N, cout_fwd, ci0, cin):
    """The K-split input gradient (nn.gboard_adjoint_split: S = Cout / 32 partial adjoint convs as one grouped
    hrl_gboard launch, then their sum) == the input gradient of F.conv2d(x, w[:, ci0:ci0+cin], padding=1): exactly
    the fp64 result on integer data, within 4e-6 of its scale on random data."""
    for integer in (True, False):
        g = torch.Generator().manual_seed(N + cout_fwd + ci0 + int(integer))
        mk = ((lambda *s: torch.randint(-3, 4, s, generator=g).float()) if integer else
              (lambda *s: torch.randn(*s, generator=g)))
        w = mk(cout_fwd, ci0 + cin + 3, 3, 3)
        dy = mk(N, cout_fwd, 6, 6)
        x = torch.zeros(N, cin, 6, 6, dtype=torch.float64, requires_grad=True)
        F.conv2d(x, w[:, ci0:ci0 + cin].double(), padding=1).backward(dy.double())
        ref = x.grad
        rec = hnn.DeferredGrads()
        y = hnn.gboard_adjoint_split(dy.to(cuda), w.to(cuda), ci0, cin, rec).cpu().double()
        if integer:
            assert torch.equal(y, ref)
        else:
            assert _close(y, ref)


def test_gboard_forward_groups_and_grouped_gates(cuda):
    """hrl_gboard_forward_groups (each group reads its own input tensor) == the grouped conv of the stacked inputs,
    bit for bit; hrl_lstm_gates_forward_grouped == one lstm_gates per layer on the conv's channel slices, bit for
    bit (zx a channel slice of a wider tensor, ragged game count)."""
    from handyrl_amd import _native
    lib = _native.load()
    g = torch.Generator().manual_seed(11)
    N, H, L = 45, 32, 3
    hs = [torch.randn(N, H, 6, 6, generator=g).to(cuda) for _ in range(L)]
    cs = [torch.randn(N, H, 6, 6, generator=g).to(cuda) for _ in range(L)]
    wide = torch.randn(N, 4 * H * L + 32, 6, 6, generator=g).to(cuda)
    zx = [wide[:, 4 * H * i:4 * H * (i + 1)] for i in range(L)]
    w = (torch.randn(4 * H * L, H, 3, 3, generator=g) * 0.2).to(cuda)
    pk = hnn.gboard_pack(w)
    ref = hnn.gboard_conv(torch.cat(hs, 1), pk, 4 * H * L, H, groups=L)
    zh = torch.empty_like(ref)
    P = _native.ptr
    stream = _native.stream_of(cuda)
    _native.check(lib.hrl_gboard_forward_groups(_native.ptr_array(hs), _native.i64_array([h.stride(0) for h in hs]),
                                                N, H, L, P(pk), pk.numel(), 4 * H * L, P(zh), zh.stride(0), stream),
                  'groups')
    assert torch.equal(zh, ref)
    h_out = [torch.empty_like(c) for c in cs]
    c_out = [torch.empty_like(c) for c in cs]
    gates = [torch.empty(N, 4 * H, 6, 6, device=cuda) for _ in range(L)]
    _native.check(lib.hrl_lstm_gates_forward_grouped(
        L, P(zh), zh.stride(0), _native.ptr_array(zx), _native.i64_array([z.stride(0) for z in zx]),
        _native.ptr_array(cs), N, H, 36, _native.ptr_array(h_out), _native.ptr_array(c_out), _native.ptr_array(gates),
        stream), 'gates')
    for i in range(L):
        hn, cn = hnn.lstm_gates(zx[i], zh[:, 4 * H * i:4 * H * (i + 1)], cs[i])
        assert torch.equal(h_out[i], hn) and torch.equal(c_out[i], cn), i


@pytest.mark.parametrize('O,C,ns', [(1, 64, (300,)), (4, 8, (37, 5)), (8, 256, (64,))])
def test_gboard_pointwise_wgrad_matches_conv1x1_weight_gradient(cuda, O, C, ns):
    """hrl_gboard_pointwise_wgrad ADDS the 1x1 conv's weight gradient sum_{n,q} dy[n,o,q] x[n,c,q] over the records
    into an existing gradient: exactly the fp64 sum on integer data, within 4e-6 of its scale on random data."""
    for integer in (True, False):
        g = torch.Generator().manual_seed(O * 31 + C + int(integer))
        mk = ((lambda *s: torch.randint(-3, 4, s, generator=g).float()) if integer else
              (lambda *s: torch.randn(*s, generator=g)))
        w = torch.nn.Parameter(torch.zeros(O, C, 1, 1, device=cuda))
        w.grad = mk(O, C, 1, 1).to(cuda)
        before = w.grad.double().cpu()
        rec = [(mk(n, C, 6, 6).to(cuda), mk(n, O, 6, 6).to(cuda)) for n in ns]
        hnn.gboard_pointwise_wgrad(rec, w, None)
        X = torch.cat([r[0] for r in rec]).double().cpu()
        DY = torch.cat([r[1] for r in rec]).double().cpu()
        dw = torch.einsum('noq,ncq->oc', DY.reshape(DY.shape[0], O, 36), X.reshape(X.shape[0], C, 36))
        ref = before + dw.view(O, C, 1, 1)
        got = w.grad.double().cpu()
        if integer:
            assert torch.equal(got, ref)
        else:
            assert (got - ref).abs().max().item() <= 4e-6 * dw.abs().max().item()
