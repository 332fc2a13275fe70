"""Time the TicTacToe net forward+backward at the bench size under layout variants."""
import sys, os, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from handyrl_amd.envs.tictactoe import SimpleConv2dModel

dev = torch.device('cuda', 0)
N = 4096 * 32


def run(name, cl=False, bench=False, cudnn=True, iters=10, hip=False):
    torch.backends.cudnn.benchmark = bench
    torch.backends.cudnn.enabled = cudnn
    torch.manual_seed(0)
    net = SimpleConv2dModel().to(dev)
    if hip:
        from handyrl_amd.nn import accelerate
        accelerate(net)
    x = (torch.rand(N, 3, 3, 3, device=dev) < 0.5).float()
    if cl:
        net = net.to(memory_format=torch.channels_last)
        x = x.contiguous(memory_format=torch.channels_last)
    def step():
        out = net(x)
        (out['policy'].sum() + out['value'].sum()).backward()
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        step()
    torch.cuda.synchronize()
    print('%-28s %.3f ms' % (name, (time.perf_counter() - t0) / iters * 1e3), flush=True)



if __name__ == '__main__':
    which = sys.argv[1]
    t0 = time.perf_counter()
    {'nchw': lambda: run('nchw'),
     'cl': lambda: run('channels_last', cl=True),
     'hip': lambda: run('nchw + HIP BatchNorm', hip=True),
     'nchw_bench': lambda: run('nchw benchmark', bench=True),
     'cl_bench': lambda: run('channels_last benchmark', cl=True, bench=True)}[which]()
    print('  (%s total %.1f s incl. warm-up)' % (which, time.perf_counter() - t0), flush=True)
