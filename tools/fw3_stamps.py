"""Per-wave phase timeline of the LDS-DMA ring forward conv (conv3x3_fwd_dma_kernel, hrl_conv3x3_set_fwd_form(2)).

    python tools/stamps.py --build        # here (CPU): tools/micro/libhrl_stamps.so with -DHRL_STAMPS
    python tools/fw3_stamps.py            # on the GPU box

Lane 0 of every wave writes s_memtime (no drain) at the phase boundaries of iterations 2 and 3 (BB2_STAMP in
csrc/hrl_conv.hip): 0 loop head, 1 LDS-DMA issued and the next tile staged, 2 MFMAs issued, 3 stores issued and
the ring's counted vmcnt wait passed; the rest of the period is the barrier.  Prints per-wave medians over the
workgroups and the iteration period.
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, 'tools', 'micro', 'libhrl_stamps.so')


def main():
    os.environ['HRL_LIB_PATH'] = LIB
    sys.path.insert(0, ROOT)
    import numpy as np
    import torch
    from handyrl_amd import _native
    dev = torch.device('cuda', 0)
    lib = _native.load()
    P = _native.ptr
    stream = _native.stream_of(dev)
    M = 131072
    g0 = torch.Generator(device=dev).manual_seed(1)
    x = torch.randn(M, 288, device=dev, generator=g0)
    w = torch.randn(32, 32, 3, 3, device=dev, generator=g0) * 0.1
    al, be = torch.rand(32, device=dev, generator=g0) + 0.5, torch.randn(32, device=dev, generator=g0) * 0.3
    packed = torch.empty(1, 2, 9216, device=dev)
    _native.check(lib.hrl_conv3x3_pack_n(_native.ptr_array([w]), 1, P(packed), stream), 'pack')
    ws_bytes = lib.hrl_conv3x3_workspace_bytes(M)
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
    nblk = lib.hrl_conv3x3_stats_blocks(M)
    part = torch.empty(nblk * 64, dtype=torch.float64, device=dev)
    y = torch.empty_like(x)
    buf = torch.zeros(nblk * 8 * 2 * 8, dtype=torch.int64, device=dev)
    lib.hrl_debug_set_stamps_conv(ctypes.c_void_p(buf.data_ptr()))
    lib.hrl_conv3x3_set_fwd_form(2)
    for _ in range(20):
        _native.check(lib.hrl_conv3x3_forward_ex(P(x), M, P(al), P(be), P(packed[0, 0]), None, 2, P(y), 1, None, None,
                                                 None, None, P(part), P(ws), ws_bytes, stream), 'fwd')
    torch.cuda.synchronize(dev)
    st = buf.view(nblk, 8, 2, 8).cpu().numpy().astype(np.int64)
    for wv in range(8):
        d = st[:, wv, :, 1:4] - st[:, wv, :, 0:3]
        period = np.median(st[:, wv, 1, 0] - st[:, wv, 0, 0])
        med = np.median(d.reshape(-1, 3), axis=0)
        print('wave %d: period %6.0f cycles; dma+stage %6.0f, mfma %6.0f, epilogue+wait %6.0f, barrier %6.0f' % (
            wv, period, med[0], med[1], med[2], period - med.sum()))


if __name__ == '__main__':
    main()
