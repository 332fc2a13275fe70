"""Per-phase wave timelines of the scan and fused-loss kernels from in-kernel clock stamps.

    python tools/stamps.py --build     # here (CPU): tools/diag/libhrl_stamps.so with -DHRL_STAMPS
    python tools/stamps.py             # on the GPU box

The diagnostic library is the product sources built with -DHRL_STAMPS (hrl_scan.h): lane 0 of each
workgroup drains its memory operations and writes s_memtime at phase boundaries (slots 0..13) and
s_memrealtime (100 MHz) at entry and exit (slots 14, 15).  The drains serialise what the product
overlaps, so phase sums exceed the product's wave time; the split is what this is for.
"""
import ctypes
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, 'tools', 'diag', 'libhrl_stamps.so')   # not gpurun-ignored: it travels to the box
SRCS = sorted(f for f in os.listdir(os.path.join(ROOT, 'handyrl_amd', 'csrc')) if f.endswith('.hip'))   # all: _native binds every symbol


def build():
    flags = ['--offload-arch=gfx950', '-O3', '-std=c++17', '-fPIC', '-ffp-contract=off', '-DHRL_STAMPS',
             '-I', os.path.join(ROOT, 'include')]
    objs = ['/tmp/stamps_' + s + '.o' for s in SRCS]
    procs = [subprocess.Popen(['hipcc'] + flags + ['-c', os.path.join(ROOT, 'handyrl_amd', 'csrc', s), '-o', o])
             for s, o in zip(SRCS, objs)]
    if any(p.wait() for p in procs):
        raise RuntimeError('stamps build failed')
    subprocess.check_call(['hipcc', '--offload-arch=gfx950', '-shared', '-fPIC', '-o', LIB] + objs)
    print('built', LIB)


def summarize(name, st, nslots, labels):
    import numpy as np
    st = st.astype(np.int64)
    wall = (st[:, 15] - st[:, 14]) * 10.0   # ns
    span = (st[:, 15].max() - st[:, 14].min()) * 10.0
    first = (st[:, 14] - st[:, 14].min()) * 10.0
    print('%s: %d waves, entry spread %.2f us (median entry %.2f us after the first), wave wall median %.2f us, '
          'max %.2f us, first entry -> last exit %.2f us'
          % (name, len(st), first.max() / 1e3, np.median(first) / 1e3, np.median(wall) / 1e3, wall.max() / 1e3,
             span / 1e3))
    for k in range(1, nslots):
        d = st[:, k] - st[:, k - 1]
        print('   %-34s median %7.0f cyc  p90 %7.0f' % (labels[k - 1], np.median(d), np.percentile(d, 90)))
    tot = st[:, nslots - 1] - st[:, 0]
    print('   %-34s median %7.0f cyc' % ('total (stamped, drained)', np.median(tot)))


def main():
    if '--build' in sys.argv:
        build()
        return
    import numpy as np
    import torch
    dev = torch.device('cuda', 0)
    lib = ctypes.CDLL(LIB)
    vp, i64, dbl = ctypes.c_void_p, ctypes.c_int64, ctypes.c_double
    lib.hrl_compute_targets_fused.argtypes = [ctypes.c_int, ctypes.c_int, vp, vp, vp, vp, vp, i64, i64, i64, i64,
                                              i64, i64, dbl, dbl, vp, vp, vp]
    lib.hrl_loss_workspace_bytes.restype = i64
    lib.hrl_loss_workspace_bytes.argtypes = [i64, i64, i64, i64]
    lib.hrl_loss_forward.argtypes = [vp, vp, vp, i64, i64, i64, i64, i64, vp, vp, vp, vp, vp, vp, vp, vp, vp,
                                     ctypes.c_int, ctypes.c_int, ctypes.c_int, dbl, dbl, dbl, dbl, vp, i64, vp, vp]
    p = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None  # noqa: E731
    stream = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    g = torch.Generator(device=dev).manual_seed(0)

    def run_scan(B, T):
        v = torch.tanh(torch.randn(B, T, 2, 1, device=dev, generator=g))
        ret = torch.randint(-1, 2, (B, 1, 2, 1), device=dev, generator=g).float()
        rho = torch.rand(B, T, 1, 1, device=dev, generator=g)
        cs = torch.rand(B, T, 1, 1, device=dev, generator=g)
        tgt, adv = torch.empty_like(v), torch.empty_like(v)
        waves = max(1, B // 4)
        buf = torch.zeros(waves * 16 + 16, dtype=torch.int64, device=dev)
        for it in range(3):
            buf.zero_()
            lib.hrl_debug_set_stamps_targets(p(buf))
            rc = lib.hrl_compute_targets_fused(3, 2, p(v), p(ret), None, p(rho), p(cs), B, T, 2, 1, 1, 2, 0.7, 1.0,
                                               p(tgt), p(adv), stream)
            assert rc == 0, rc
            torch.cuda.synchronize(dev)
        st = buf.view(-1, 16).cpu().numpy()
        st = st[st[:, 15] != 0]
        nch = (T + 15) // 16
        labels = ['boot + first loads landed']
        for c in range(nch):
            labels += ['chunk %d: to LDS + barrier' % c, 'chunk %d: recurrence' % c, 'chunk %d: stores' % c]
        summarize('scan B=%d T=%d' % (B, T), st, 2 + 3 * nch, labels)

    def run_loss(B, T, A=9):
        tpol = torch.randn(B, T, 1, A, device=dev, generator=g)
        bpol = torch.randn(B, T, 1, A, device=dev, generator=g)
        action = torch.randint(0, A, (B, T, 1), device=dev, generator=g)
        emask = torch.ones(B, T, 1, device=dev)
        turn = torch.arange(T, device=dev) % 2
        tmask = torch.stack([1 - turn, turn], -1).float().view(1, T, 2, 1).expand(B, T, 2, 1).contiguous()
        omask = torch.ones(B, T, 2, 1, device=dev)
        progress = torch.rand(B, T, 1, device=dev, generator=g)
        value = torch.tanh(torch.randn(B, T, 2, 1, device=dev, generator=g))
        outcome = torch.randint(-1, 2, (B, 1, 2, 1), device=dev, generator=g).float()
        ws = torch.empty(lib.hrl_loss_workspace_bytes(B, T, 2, 1), dtype=torch.uint8, device=dev)
        losses = torch.empty(6, device=dev)
        waves = B
        buf = torch.zeros(waves * 16 + 16, dtype=torch.int64, device=dev)
        for it in range(3):
            buf.zero_()
            lib.hrl_debug_set_stamps_loss(p(buf))
            rc = lib.hrl_loss_forward(p(tpol), p(bpol), p(action), B, T, 2, 1, A, p(emask), p(tmask), p(omask),
                                      p(progress), p(value), p(outcome), None, None, None, 3, 2, 1, 0.7, 1.0, 0.1,
                                      0.3, p(ws), ws.numel(), p(losses), stream)
            assert rc == 0, rc
            torch.cuda.synchronize(dev)
        st = buf.view(-1, 16).cpu().numpy()
        st = st[st[:, 15] != 0]
        summarize('fused loss B=%d T=%d' % (B, T), st, 6,
                  ['prep: policy rows', 'prep: values + barrier', 'scans + barrier', 'terms + barrier',
                   'wave fold + partial store'])

    def run_block(M=131072):
        lib.hrl_conv3x3_workspace_bytes.restype = i64
        lib.hrl_conv3x3_workspace_bytes.argtypes = [i64]
        lib.hrl_conv3x3_stats_blocks.restype = i64
        lib.hrl_conv3x3_stats_blocks.argtypes = [i64]
        lib.hrl_conv3x3_pack_n.argtypes = [vp, ctypes.c_int, vp, vp]
        lib.hrl_conv3x3_block_backward.argtypes = [vp, vp, i64] + [vp] * 12 + [ctypes.c_int, vp, vp, vp, vp, vp,
                                                                            i64, vp]
        r = lambda *sh: torch.randn(*sh, device=dev, generator=g)   # noqa: E731
        gg, y, x = r(M, 288), r(M, 288), r(M, 288)
        w = r(32, 32, 3, 3) * 0.1
        c = [r(32).abs() + 0.5 for _ in range(11)]
        packed = torch.empty(1, 2, 9216, device=dev)
        wp = (ctypes.c_void_p * 1)(w.data_ptr())
        assert lib.hrl_conv3x3_pack_n(wp, 1, p(packed), stream) == 0
        wsb = lib.hrl_conv3x3_workspace_bytes(M)
        ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
        part = torch.empty(lib.hrl_conv3x3_stats_blocks(M) * 64, dtype=torch.float64, device=dev)
        dw, gin = torch.empty(32, 32, 3, 3, device=dev), torch.empty_like(gg)
        buf = torch.zeros(256 * 16 + 16, dtype=torch.int64, device=dev)
        for it in range(3):
            buf.zero_()
            lib.hrl_debug_set_stamps_conv(p(buf))
            rc = lib.hrl_conv3x3_block_backward(p(gg), p(y), M, *[p(t) for t in c[:6]], p(x), p(c[6]), p(c[7]),
                                                p(packed[0, 1]), p(dw), p(gin), 2, p(c[8]), p(c[9]), p(c[10]),
                                                p(part), p(ws), wsb, stream)
            assert rc == 0, rc
            torch.cuda.synchronize(dev)
        st = buf.view(-1, 16).cpu().numpy()
        st = st[st[:, 15] != 0]
        import numpy as np
        st = st.astype(np.int64)
        labels = ['loads + BN apply (dY)', 'weight gradient (dY split, 294 MFMA32)', 'dY to LDS wait + input-grad MFMA',
                  'epilogue: stage, sums, stores']
        wall = (st[:, 15] - st[:, 14]) * 10.0
        print('block backward M=%d: %d workgroups, wave-0 wall median %.1f us' % (M, len(st), np.median(wall) / 1e3))
        for t in range(2):
            for k in range(4):
                d = st[:, 6 * t + k + 1] - st[:, 6 * t + k]
                print('   tile %d %-42s median %7.0f cyc  p90 %7.0f' % (t, labels[k], np.median(d), np.percentile(d, 90)))
        d = st[:, 12] - st[:, 0]
        print('   all tiles (stamped, drained)                      median %7.0f cyc' % np.median(d))
        d = st[:, 13] - st[:, 12]
        print('   final folds                                       median %7.0f cyc' % np.median(d))

    which = sys.argv[1:] or ['scan', 'loss', 'block']
    if 'scan' in which:
        run_scan(4096, 32)
        run_scan(4096, 9)
        run_scan(1 << 18, 9)
    if 'loss' in which:
        run_loss(4096, 32)
        run_loss(4096, 9)
    if 'block' in which:
        run_block()


if __name__ == '__main__':
    main()
