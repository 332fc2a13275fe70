"""Geister self-play convs at E=2048 on a 6x6 board: MIOpen NCHW (grouped h conv 96->384 g3, x half 32->384)
vs channels_last vs unfold + GEMM, fp32.  Times in us per call."""
import time
import torch
import torch.nn.functional as F

dev = torch.device('cuda', 0)
E = 2048
torch.manual_seed(0)
h = torch.randn(E, 96, 6, 6, device=dev)
wg = torch.randn(384, 32, 3, 3, device=dev) * 0.05
x = torch.randn(E, 32, 6, 6, device=dev)
wx = torch.randn(384, 32, 3, 3, device=dev) * 0.05


def bench(fn, n=30):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return round((time.perf_counter() - t0) / n * 1e6, 1)


def gemm_conv(inp, w, groups):
    n, c = inp.shape[:2]
    cols = F.unfold(inp, 3, padding=1)                                   # (E, c*9, 36)
    cg = c // groups
    cols = cols.view(n, groups, cg * 9, 36).permute(1, 0, 3, 2).reshape(groups, n * 36, cg * 9)
    wm = w.view(groups, -1, cg * 9).transpose(1, 2)                      # (g, cg*9, co/g)
    y = torch.bmm(cols, wm)                                              # (g, E*36, co/g)
    return y.view(groups, n, 36, -1).permute(1, 0, 3, 2).reshape(n, -1, 6, 6)


res = {}
res['h_nchw'] = bench(lambda: F.conv2d(h, wg, padding=1, groups=3))
res['x_nchw'] = bench(lambda: F.conv2d(x, wx, padding=1))
hl, xl = h.to(memory_format=torch.channels_last), x.to(memory_format=torch.channels_last)
wgl, wxl = wg.to(memory_format=torch.channels_last), wx.to(memory_format=torch.channels_last)
res['h_nhwc'] = bench(lambda: F.conv2d(hl, wgl, padding=1, groups=3))
res['x_nhwc'] = bench(lambda: F.conv2d(xl, wxl, padding=1))
res['h_gemm'] = bench(lambda: gemm_conv(h, wg, 3))
res['x_gemm'] = bench(lambda: gemm_conv(x, wx, 1))
ref = F.conv2d(h.double(), wg.double(), padding=1, groups=3)
for name, y in (('nchw', F.conv2d(h, wg, padding=1, groups=3)), ('nhwc', F.conv2d(hl, wgl, padding=1, groups=3)),
                ('gemm', gemm_conv(h, wg, 3))):
    res['err_' + name] = float((y.double() - ref).abs().max())
print(res)
