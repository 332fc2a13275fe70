"""Per-wave phase timeline of the LDS-DMA ring forward conv (conv3x3_fwd_dma_kernel, hrl_conv3x3_set_fwd_form(2)).

    python tools/stamps.py --build        # here (CPU): tools/micro/libhrl_stamps.so with -DHRL_STAMPS
    python tools/fw3_stamps.py            # on the GPU box

Lane 0 of every wave writes s_memtime (no drain) at the phase boundaries of iterations 2 and 3 (BB2_STAMP in
csrc/hrl_conv.hip).  MFMA waves 0-3: 0 loop head, 1 MFMAs issued, 2 epilogue issued, 3 past the barrier.  Stagers
4-7: 0 loop head, 1 LDS-DMA issued, 2 stage written, 3 past the counted vmcnt wait, 4 past the barrier.  Prints
per-wave medians over the workgroups and the iteration period.
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
        npts = 4 if wv < 4 else 5
        d = st[:, wv, :, 1:npts] - st[:, wv, :, 0:npts - 1]
        period = np.median(st[:, wv, 1, 0] - st[:, wv, 0, 0])
        med = np.median(d.reshape(-1, npts - 1), axis=0)
        print('wave %d (%s): period %6.0f cycles; phases %s' % (
            wv, 'mfma' if wv < 4 else 'stager', period, ' '.join('%6.0f' % v for v in med)))


if __name__ == '__main__':
    main()
