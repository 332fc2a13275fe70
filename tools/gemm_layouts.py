"""fp32 GEMM layout variants for the board-conv shapes (M = B*T rows)."""
import time, torch
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


for K, N in ((288, 288), (27, 288), (288, 18)):
    x = torch.randn(M, K, device=dev)
    dy = torch.randn(M, N, device=dev)
    W = torch.randn(K, N, device=dev)
    Wt = W.t().contiguous()
    b = torch.randn(N, device=dev)
    fl = 2 * M * K * N / 1e12
    res = {
        'fwd x@W': t(lambda: torch.addmm(b, x, W)),
        'fwd x@Wt.t()': t(lambda: torch.addmm(b, x, Wt.t())),
        'dX dy@W.t()': t(lambda: dy @ W.t()),
        'dX dy@Wt': t(lambda: dy @ Wt),
        'dW x.t()@dy': t(lambda: x.t() @ dy),
        'dW (dy.t()@x).t()': t(lambda: (dy.t() @ x)),
    }
    for k, us in res.items():
        print('K=%3d N=%3d %-20s %8.1f us %6.1f TF' % (K, N, k, us, fl / (us * 1e-6)), flush=True)
