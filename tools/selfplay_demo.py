"""Train TicTacToe from scratch with the device-resident loop; print win rate vs random."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from handyrl_amd.envs.tictactoe import SimpleConv2dModel
from handyrl_amd.loop import SelfPlayTrainer, evaluate_vs_random
from handyrl_amd.synthetic import default_args

dev = torch.device('cuda', 0)
rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 30
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
torch.manual_seed(0)
net = SimpleConv2dModel().to(dev)
args = default_args(9, 1024)
args['maximum_episodes'] = 32768
tr = SelfPlayTrainer(net, args, dev, games_per_round=4096, capacity=32768)
print('before', evaluate_vs_random(net, dev), flush=True)
t0 = time.perf_counter()
for r in range(rounds):
    tr.run(1, steps, log=print if r % 5 == 0 else None)
    if r % 10 == 9:
        print('eval', r, evaluate_vs_random(net, dev), flush=True)
torch.cuda.synchronize()
print('after', evaluate_vs_random(net, dev), 'time %.1fs episodes %d steps %d' % (time.perf_counter() - t0, tr.episodes, tr.steps), flush=True)
