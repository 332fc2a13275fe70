"""Per-wave phase timeline of the tile-shared chain block backward (conv3x3_block_bwd2_kernel).

    python tools/bb2_stamps.py --build     # here (CPU): tools/diag/libhrl_stamps.so with -DHRL_STAMPS
    python tools/bb2_stamps.py             # on the GPU box

Lane 0 of every wave writes s_memtime, without draining its memory operations, at the phase boundaries of
iterations 2 and 3 (BB2_STAMP in csrc/hrl_conv.hip): the wave's issue timeline, with the compiler's own waits
for loaded registers where the product has them.  Prints per-wave-role medians over the workgroups.
"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, 'tools', 'diag', 'libhrl_stamps.so')


def main():
    if '--build' in sys.argv:
        subprocess.check_call([sys.executable, os.path.join(ROOT, 'tools', 'stamps.py'), '--build'])
        return
    os.environ['HRL_LIB_PATH'] = LIB
    sys.path.insert(0, ROOT)
    import numpy as np
    import torch
    from handyrl_amd import _native
    dev = torch.device('cuda', 0)
    lib = _native.load()
    import ctypes
    raw = lib
    P = _native.ptr
    stream = _native.stream_of(dev)
    M = 131072
    g0 = torch.Generator(device=dev).manual_seed(1)
    rnd = lambda *s: torch.randn(*s, device=dev, generator=g0)   # noqa: E731
    g, y, x = rnd(M, 288), rnd(M, 288), rnd(M, 288)
    w = rnd(32, 32, 3, 3) * 0.1
    c = [rnd(32).abs() + 0.5 for _ in range(11)]
    packed = torch.empty(1, 2, 9216, device=dev)
    _native.check(lib.hrl_conv3x3_pack_n(_native.ptr_array([w]), 1, P(packed), stream), 'pack')
    ws_bytes = lib.hrl_conv3x3_workspace_bytes(M)
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
    part = torch.empty(lib.hrl_conv3x3_stats_blocks(M) * 64, dtype=torch.float64, device=dev)
    dw, gin = torch.empty(32, 32, 3, 3, device=dev), torch.empty_like(g)
    nblk = lib.hrl_conv3x3_stats_blocks(M)
    buf = torch.zeros(nblk * 8 * 2 * 8, dtype=torch.int64, device=dev)
    raw.hrl_debug_set_stamps_conv(ctypes.c_void_p(buf.data_ptr()))
    for _ in range(5):
        _native.check(lib.hrl_conv3x3_block_backward(
            P(g), P(y), M, *[P(t) for t in c[:6]], P(x), P(c[6]), P(c[7]), P(packed[0, 1]), P(dw), P(gin), 2,
            P(c[8]), P(c[9]), P(c[10]), P(part), P(ws), ws_bytes, stream), 'block')
    torch.cuda.synchronize(dev)
    st = buf.view(nblk, 8, 2, 8).cpu().numpy().astype(np.int64)
    labels = ['first part', 'second part', 'barrier']
    print('points: 0 loop head, 1 after the first part, 2 after the second part, 3 after the barrier; the first '
          'part is compute + gin store for compute-first waves (kCFirst: 0, 1, 6, 7), stage + issue for the others')
    for wv in range(8):
        d = st[:, wv, :, 1:4] - st[:, wv, :, 0:3]
        it_total = np.median(st[:, wv, 1, 0] - st[:, wv, 0, 0])
        med = np.median(d.reshape(-1, 3), axis=0)
        print('wave %d: ' % wv + '  '.join('%s %6.0f' % (l, m) for l, m in zip(labels, med))
              + '  | iteration %6.0f cyc' % it_total)

if __name__ == '__main__':
    main()
