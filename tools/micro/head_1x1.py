"""Geister self-play heads at E=2048: the 1x1 convs (64->2 value/return, 8->4 policy) as MIOpen convs vs
broadcast matmuls, fp32.  us per call and max abs difference."""
import time
import torch
import torch.nn.functional as F

dev = torch.device('cuda', 0)
E = 2048
torch.manual_seed(0)
h = torch.randn(E, 64, 6, 6, device=dev)
z = torch.randn(E, 8, 6, 6, device=dev)
w2 = torch.randn(2, 64, 1, 1, device=dev)
w4 = torch.randn(4, 8, 1, 1, device=dev)


def bench(fn, n=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return round((time.perf_counter() - t0) / n * 1e6, 1)


res = {
    'conv_64to2': bench(lambda: F.conv2d(h, w2)),
    'matmul_64to2': bench(lambda: torch.matmul(w2.view(2, 64), h.view(E, 64, 36))),
    'conv_8to4': bench(lambda: F.conv2d(z, w4)),
    'matmul_8to4': bench(lambda: torch.matmul(w4.view(4, 8), z.view(E, 8, 36))),
}
res['diff_64to2'] = float((F.conv2d(h, w2).view(E, 2, 36) - torch.matmul(w2.view(2, 64), h.view(E, 64, 36))).abs().max())
res['diff_8to4'] = float((F.conv2d(z, w4).view(E, 4, 36) - torch.matmul(w4.view(4, 8), z.view(E, 8, 36))).abs().max())
print(res)
