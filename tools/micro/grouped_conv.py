"""MIOpen: three 32->128 3x3 convs on a 6x6 board vs one grouped (groups=3) 96->384 conv, E=2048 (fp32)."""
import time
import torch
import torch.nn.functional as F

dev = torch.device('cuda', 0)
E = 2048
xs = [torch.randn(E, 32, 6, 6, device=dev) for _ in range(3)]
ws = [torch.randn(128, 32, 3, 3, device=dev) * 0.05 for _ in range(3)]
xg = torch.cat(xs, 1)
wg = torch.cat(ws, 0)


def bench(fn, n=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n * 1e6


sep = bench(lambda: [F.conv2d(x, w, padding=1) for x, w in zip(xs, ws)])
grp = bench(lambda: F.conv2d(xg, wg, padding=1, groups=3))
ys = torch.cat([F.conv2d(x, w, padding=1) for x, w in zip(xs, ws)], 1)
yg = F.conv2d(xg, wg, padding=1, groups=3)
print({'three_convs_us': round(sep, 1), 'grouped_us': round(grp, 1),
       'max_abs_diff': float((ys - yg).abs().max()), 'bit_equal': bool(torch.equal(ys, yg))})
