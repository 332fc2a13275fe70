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
