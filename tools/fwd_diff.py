"""Compare the chain forward's forms at M rows (random data): max |y2 - y0|, the first differing rows and cells."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from handyrl_amd import _native  # noqa: E402


def main():
    dev = torch.device('cuda', 0)
    lib = _native.load()
    P = _native.ptr
    stream = _native.stream_of(dev)
    for M in (20000, 40000, 131072):
        g0 = torch.Generator(device=dev).manual_seed(M)
        x = torch.randn(M, 288, device=dev, generator=g0)
        w = torch.randn(32, 32, 3, 3, device=dev, generator=g0) * 0.1
        al, be = torch.rand(32, device=dev, generator=g0) + 0.5, torch.randn(32, device=dev, generator=g0) * 0.3
        packed = torch.empty(1, 2, 9216, device=dev)
        _native.check(lib.hrl_conv3x3_pack_n(_native.ptr_array([w]), 1, P(packed), stream), 'pack')
        ws_bytes = lib.hrl_conv3x3_workspace_bytes(M)
        ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
        nblk = lib.hrl_conv3x3_stats_blocks(M)
        ys = []
        for form in (0, 2):
            lib.hrl_conv3x3_set_fwd_form(form)
            y = torch.full_like(x, float('nan'))
            part = torch.empty(nblk * 64, dtype=torch.float64, device=dev)
            _native.check(lib.hrl_conv3x3_forward_ex(P(x), M, P(al), P(be), P(packed[0, 0]), None, 2, P(y), 1, None,
                                                     None, None, None, P(part), P(ws), ws_bytes, stream), 'fwd')
            torch.cuda.synchronize(dev)
            ys.append(y)
        lib.hrl_conv3x3_set_fwd_form(1)
        d = (ys[1] - ys[0]).abs()
        bad = (d > 0) | torch.isnan(d)
        rows = bad.any(1).nonzero().flatten()
        print('M', M, 'max diff', float(d.nan_to_num(1e30).max()), 'bad rows', rows.numel(), 'first', rows[:8].tolist(),
              'tiles', sorted(set((rows // 16).tolist()))[:10], flush=True)
        if rows.numel():
            r = int(rows[0])
            cells = bad[r].view(32, 9).any(0).nonzero().flatten().tolist()
            chans = bad[r].view(32, 9).any(1).nonzero().flatten().tolist()
            print('   row', r, 'cells', cells, 'channels', chans[:32], flush=True)


if __name__ == '__main__':
    main()
