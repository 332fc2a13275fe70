"""libhrl.so loads on a CPU-only host and exports exactly the C ABI of include/*.h.

No compute call is made here (no GPU): only the argument-validation paths,
which return before any HIP call.
"""

import ctypes
import glob
import os
import re
import subprocess

import pytest

from handyrl_amd import _native

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    syms = set()
    for h in glob.glob(os.path.join(ROOT, 'include', '*.h')):
        text = open(h).read()
        text = re.sub(r'/\*.*?\*/', '', text, flags=re.S)
        syms |= set(re.findall(r'\b(hrl_[a-z0-9_]+)\s*\(', text))
    return syms


def test_header_symbols_bound():
    syms = declared_symbols()
    assert 'hrl_compute_target' in syms and 'hrl_compute_targets_fused' in syms
    assert syms == set(_native.SIGNATURES), 'ctypes signatures out of sync with include/*.h'


def test_library_exports_every_declared_symbol():
    lib = _native.load()
    for s in declared_symbols():
        assert hasattr(lib, s), s
    out = subprocess.run(['nm', '-D', '--defined-only', _native.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r' T (hrl_[a-z0-9_]+)', out))
    assert declared_symbols() <= exported


def test_abi_version_and_errors():
    lib = _native.load()
    assert lib.hrl_abi_version() == _native.ABI_VERSION
    assert b'invalid' in lib.hrl_strerror(_native.HRL_EINVAL)
    assert lib.hrl_strerror(0) == b'success'


@pytest.mark.parametrize('alg,kw', [
    (7, {}),                                  # unknown algorithm
    (1, {'T': 0}),                            # empty time axis
    (1, {'C': 65}),                           # more columns than a wave
    (1, {'ret_T': 3}),                        # returns time extent not in {1, T}
    (3, {'rho_C': 2, 'rho_div': 2, 'C': 2}),  # rho columns do not tile value columns
    (3, {'null_rho': True}),                  # V-trace without rhos
    (0, {'targets': True}),                   # MC writes no targets
])
def test_invalid_arguments_rejected_without_gpu(alg, kw):
    lib = _native.load()
    dummy = ctypes.c_void_p(16)
    B, T, C = 4, kw.get('T', 8), kw.get('C', 2)
    rho_C, rho_div = kw.get('rho_C', 1), kw.get('rho_div', C)
    rho = None if kw.get('null_rho') else dummy
    tgt = dummy if kw.get('targets') else None
    code = lib.hrl_compute_target(alg, dummy, dummy, None, rho, rho, B, T, C, kw.get('ret_T', 1),
                                  rho_C, rho_div, 0.7, 1.0, tgt, dummy, None)
    assert code == _native.HRL_EINVAL


def test_missing_library_fails_loudly(monkeypatch, tmp_path):
    monkeypatch.setattr(_native, '_lib', None)
    monkeypatch.setattr(_native, 'LIB_PATH', str(tmp_path / 'nope.so'))
    with pytest.raises(RuntimeError, match='no CPU fallback'):
        _native.load()


def test_gboard_wgrad_rejects_workspace_sized_by_games_not_tiles():
    """hrl_gboard_wgrad runs one workgroup partial per 16-game tile of each record, so 24 records of 2 games need
    24 partials, not ceil(48 / 16) = 3: a workspace sized from the game total is rejected before any launch."""
    lib = _native.load()
    n = 24
    ptrs = (ctypes.c_void_p * n)(*[4096 * (i + 1) for i in range(n)])
    strides = (ctypes.c_int64 * n)(*[32 * 36] * n)
    dstrides = (ctypes.c_int64 * n)(*[128 * 36] * n)
    ns = (ctypes.c_int64 * n)(*[2] * n)
    cast = lambda a: ctypes.cast(a, ctypes.c_void_p)   # noqa: E731
    small = lib.hrl_gboard_wgrad_workspace_bytes(128, 32, 2 * n)
    enough = lib.hrl_gboard_wgrad_workspace_bytes(128, 32, 16 * n)
    assert 0 < small < enough
    code = lib.hrl_gboard_wgrad(cast(ptrs), cast(strides), cast(ptrs), cast(dstrides), cast(ns), n, 128, 32,
                                ctypes.c_void_p(16), 64, 32, None, ctypes.c_void_p(16), small, None)
    assert code == _native.HRL_EINVAL


def test_gboard_forward_rejects_undersized_packed_buffer():
    """hrl_gboard_forward / hrl_gboard_forward_groups take the packed buffer's size (ABI 19) and return HRL_EINVAL,
    before any launch, when it is below hrl_gboard_pack_bytes(Cout, Cin_g): a C caller binding the ABI directly
     cannot make the kernel read past the fragments.  Only argument validation runs here."""
    lib = _native.load()
    dummy = ctypes.c_void_p(4096)
    N, Cout, cin = 8, 64, 32
    need = lib.hrl_gboard_pack_bytes(Cout, cin)
    assert need > 0
    for size in (need - 16, need // 2, 0):
        code = lib.hrl_gboard_forward(dummy, cin * 36, None, 0, N, cin, 1, dummy, size, Cout, None, None, None, 0,
                                      dummy, Cout * 36, None)
        assert code == _native.HRL_EINVAL
    # the adjoint packing of the move head's 64 <- 8 input gradient (K = 8): Cout 64, Cin_g 8
    need_adj = lib.hrl_gboard_pack_bytes(64, 8)
    code = lib.hrl_gboard_forward(dummy, 8 * 36, None, 0, N, 8, 1, dummy, need_adj - 1, 64, None, None, None, 0,
                                  dummy, 64 * 36, None)
    assert code == _native.HRL_EINVAL
    L, H = 3, 32
    xs = (ctypes.c_void_p * L)(*[4096 * (i + 1) for i in range(L)])
    strides = (ctypes.c_int64 * L)(*[H * 36] * L)
    cast = lambda a: ctypes.cast(a, ctypes.c_void_p)   # noqa: E731
    need_g = lib.hrl_gboard_pack_bytes(4 * H * L, H)
    code = lib.hrl_gboard_forward_groups(cast(xs), cast(strides), N, H, L, dummy, need_g - 16, 4 * H * L, dummy,
                                         4 * H * L * 36, None)
    assert code == _native.HRL_EINVAL


def test_gboard_conv_refuses_packed_weights_of_another_shape():
    """The Python boundary refuses a packed buffer smaller than hrl_gboard_pack_bytes(Cout, Cin_g) (or of another
    dtype) before any launch (no GPU needed); the C entry checks the size again."""
    import torch
    from handyrl_amd import nn as hnn
    lib = _native.load()
    need = lib.hrl_gboard_pack_bytes(64, 32)
    x = torch.zeros(1, 32, 6, 6)
    with pytest.raises(ValueError):
        hnn.gboard_conv(x, torch.zeros(need - 16, dtype=torch.uint8), 64, 32)
    with pytest.raises(ValueError):
        hnn.gboard_conv(x, torch.zeros(need // 4, dtype=torch.float32), 64, 32)
