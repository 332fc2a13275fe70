"""dW = X^T @ dY over M = B*T rows: plain vs chunked batched GEMM + sum."""
import torch
dev = torch.device('cuda', 0)
M = 4096 * 32


def t(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s = torch.cuda.Event(enable_timing=True); e = torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record(); e.synchronize()
    return s.elapsed_time(e) / iters * 1e3


for K, N in ((288, 288), (27, 288), (288, 18), (288, 9)):
    x = torch.randn(M, K, device=dev)
    dy = torch.randn(M, N, device=dev)
    fl = 2 * M * K * N / 1e12
    ref = x.t() @ dy
    print('K=%3d N=%3d plain       %8.1f us %6.1f TF' % (K, N, t(lambda: x.t() @ dy), fl / (t(lambda: x.t() @ dy) * 1e-6)), flush=True)
    for S in (16, 64, 256, 1024):
        f = lambda: torch.bmm(x.view(S, M // S, K).transpose(1, 2), dy.view(S, M // S, N)).sum(0)
        err = (f() - ref).abs().max().item() / ref.abs().max().item()
        us = t(f)
        print('K=%3d N=%3d chunks=%4d %8.1f us %6.1f TF  relerr %.1e' % (K, N, S, us, fl / (us * 1e-6), err), flush=True)
