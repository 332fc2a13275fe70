"""List the framework reductions/copies of one eager learner step with their input shapes."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from torch.profiler import profile, ProfilerActivity
from handyrl_amd.envs.tictactoe import SimpleConv2dModel
from handyrl_amd.synthetic import tictactoe_batch, default_args
from handyrl_amd.trainer import LearnerStep

dev = torch.device('cuda', 0)
B, T = 4096, 32
args = default_args(T, B)
torch.manual_seed(0)
net = SimpleConv2dModel().to(dev)
step = LearnerStep(net, args, dev, graph=False)
batch = tictactoe_batch(B, T, dev, seed=1)
for _ in range(3):
    step.step(batch)
torch.cuda.synchronize()
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True) as prof:
    step.step(batch)
    torch.cuda.synchronize()
rows = prof.key_averages(group_by_input_shape=True)
for r in sorted(rows, key=lambda r: -r.device_time_total)[:40]:
    print('%-40s %10.1f us  x%-3d %s' % (r.key[:40], r.device_time_total, r.count, str(r.input_shapes)[:110]))
