"""Time the torus-conv kernels (csrc/hrl_torus.hip) at the Geese learner size: python tools/torus_bench.py [N] [split]."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from handyrl_amd import _native

N = int(sys.argv[1]) if len(sys.argv) > 1 else 131072
dev = torch.device('cuda', 0)
lib = _native.load()
lib.hrl_torus_set_split(int(sys.argv[2]) if len(sys.argv) > 2 else 1)
P = _native.ptr
g = torch.Generator(device=dev).manual_seed(0)
x = torch.randn(N, 32, 7, 11, device=dev, generator=g)
w = torch.randn(32, 32, 3, 3, device=dev, generator=g) * 0.1
b = torch.randn(32, device=dev, generator=g)
y = torch.empty_like(x)
add = torch.randn_like(x)
dw = torch.empty_like(w)
db = torch.empty_like(b)
ws_bytes = lib.hrl_torus_workspace_bytes(N)
ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
part = torch.empty(lib.hrl_torus_stats_blocks(N) * 64, dtype=torch.float64, device=dev)
s = _native.stream_of(dev)
flops = 2.0 * N * 77 * 288 * 32
cases = {
    'fwd': lambda: lib.hrl_torus_conv_forward(P(x), N, 32, 32, 7, 11, P(w), P(b), 0, P(y), None, None, None, P(ws), ws_bytes, s),
    'fwd+stats': lambda: lib.hrl_torus_conv_forward(P(x), N, 32, 32, 7, 11, P(w), P(b), 0, P(y), P(part), None, None, P(ws), ws_bytes, s),
    'dgrad': lambda: lib.hrl_torus_conv_forward(P(x), N, 32, 32, 7, 11, P(w), None, 1, P(y), None, None, None, P(ws), ws_bytes, s),
    'dgrad+res': lambda: lib.hrl_torus_conv_forward(P(x), N, 32, 32, 7, 11, P(w), None, 1, P(y), None, P(add), P(x), P(ws), ws_bytes, s),
    'wgrad': lambda: lib.hrl_torus_conv_wgrad(P(x), P(add), N, 32, 32, 7, 11, P(dw), P(db), P(ws), ws_bytes, s),
}
for name, fn in cases.items():
    for _ in range(2):
        _native.check(fn(), name)
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    st.record()
    for _ in range(10):
        fn()
    en.record()
    en.synchronize()
    us = st.elapsed_time(en) * 1e3 / 10
    print('%-10s %9.1f us  %6.1f TFLOP/s  %.3f of 157.3' % (name, us, flops / us / 1e6, flops / us / 1e6 / 157.3), flush=True)
