"""Does a hipEventRecordExternal event captured in a HIP graph order a later hipStreamWaitEvent on another stream?
(torch refuses external events on ROCm, so this calls HIP directly.)"""
import ctypes
import torch
hip = ctypes.CDLL('libamdhip64.so.7')
dev = torch.device('cuda', 0)
x = torch.zeros(1 << 22, device=dev)
y = torch.zeros(1, device=dev)
ev = ctypes.c_void_p()
assert hip.hipEventCreateWithFlags(ctypes.byref(ev), 0x2) == 0     # hipEventDisableTiming
g = torch.cuda.CUDAGraph()
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    x.add_(1)
torch.cuda.current_stream().wait_stream(s)
with torch.cuda.graph(g):
    for _ in range(50):
        x.add_(1)
    cur = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    rc = hip.hipEventRecordWithFlags(ev, cur, 0x1)                  # hipEventRecordExternal
    for _ in range(400):
        x.mul_(1.0)
print('record rc', rc)
side = torch.cuda.Stream()
ok = True
for it in range(5):
    g.replay()
    assert hip.hipStreamWaitEvent(ctypes.c_void_p(side.cuda_stream), ev, 0) == 0
    with torch.cuda.stream(side):
        y.copy_(x[:1])
    torch.cuda.synchronize()
    expect = 1 + 50 * (it + 1)
    print(it, y.item(), expect)
    ok &= y.item() == expect
print('EXTERNAL_EVENT_OK' if ok else 'EXTERNAL_EVENT_BAD')
