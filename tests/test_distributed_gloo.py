"""Data-parallel learner step on CPU with gloo, world_size 2.

Two ranks each train half of a batch; the bucketed, hook-launched SUM
all-reduce (handyrl_amd/distributed.py) must reproduce the single-process
full-batch update exactly as the reference defines it (losses are sums over
the batch, train.py:202-213, so gradients add).  The loss here is the CPU
oracle's (the HIP scans need a GPU); the distributed machinery is the
product's.
"""

import os
import socket
import tempfile

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp
import torch.nn as nn
import torch.nn.functional as F


class SmallNet(nn.Module):
    """BatchNorm-free TicTacToe-shaped net (BN statistics are per replica, so excluded)."""

    def __init__(self):
        super().__init__()
        self.conv = nn.Conv2d(3, 8, 3, padding=1)
        self.conv2 = nn.Conv2d(8, 8, 3, padding=1)
        self.fc_p = nn.Linear(72, 9)
        self.fc_v = nn.Linear(72, 1)

    def forward(self, x, hidden=None):
        h = F.relu(self.conv2(F.relu(self.conv(x)))).flatten(1)
        return {'policy': self.fc_p(h), 'value': torch.tanh(self.fc_v(h))}


class HeadsFirstNet(SmallNet):
    """The same net with its heads registered before its convs: registration order is not backward
    order, so the first gradient hook lands in a later bucket than the first backward-order one."""

    def __init__(self):
        nn.Module.__init__(self)
        self.fc_p = nn.Linear(72, 9)
        self.fc_v = nn.Linear(72, 1)
        self.conv = nn.Conv2d(3, 8, 3, padding=1)
        self.conv2 = nn.Conv2d(8, 8, 3, padding=1)


NETS = {'SmallNet': SmallNet, 'HeadsFirstNet': HeadsFirstNet}


def oracle_loss(outputs, batch, args):
    from oracle.learner import loss_from_outputs
    losses, dcnt = loss_from_outputs(outputs, batch, args)
    return losses, torch.tensor(dcnt)


def make_batch_and_args(B=8, T=9):
    from handyrl_amd.synthetic import tictactoe_batch, default_args
    return tictactoe_batch(B, T, torch.device('cpu'), seed=42), default_args(T, B)


pytestmark = []


def _free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def _rank_main(rank, world, port, out_path, steps, bucket_bytes, net_name='SmallNet'):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    from handyrl_amd import distributed as hdist
    from handyrl_amd.trainer import LearnerStep
    hdist.init_process_group('cpu')
    batch, args = make_batch_and_args()
    B = batch['value'].size(0)
    shard = {k: v[rank * B // world:(rank + 1) * B // world] for k, v in batch.items()}
    torch.manual_seed(0)
    net = NETS[net_name]()
    step = LearnerStep(net, args, torch.device('cpu'), world_size=world, loss_fn=oracle_loss,
                       bucket_bytes=bucket_bytes, lr=1e-3)
    assert len(step.reducer.buckets) >= 1
    for _ in range(steps):
        step.step(shard)
    sums, n = step.pop_stats()           # all-reduced loss sums
    flat = torch.cat([p.detach().reshape(-1) for p in net.parameters()])
    gathered = [torch.zeros_like(flat) for _ in range(world)]
    dist.all_gather(gathered, flat)
    if rank == 0:
        torch.save({'params': [g.clone() for g in gathered], 'sums': sums, 'buckets': len(step.reducer.buckets)},
                   out_path)
    dist.barrier()
    dist.destroy_process_group()


def _single_process(steps, net_name='SmallNet'):
    from handyrl_amd.trainer import LearnerStep
    batch, args = make_batch_and_args()
    torch.manual_seed(0)
    net = NETS[net_name]()
    step = LearnerStep(net, args, torch.device('cpu'), loss_fn=oracle_loss, lr=1e-3)
    for _ in range(steps):
        step.step(batch)
    sums, _ = step.pop_stats()
    return torch.cat([p.detach().reshape(-1) for p in net.parameters()]).numpy(), sums


@pytest.mark.parametrize('bucket_bytes,net_name', [(256 * 1024, 'SmallNet'),   # one bucket
                                                    (1024, 'SmallNet'),         # several hook-launched buckets
                                                    (1024, 'HeadsFirstNet')])   # registration != backward order
def test_two_rank_sum_allreduce_matches_full_batch(bucket_bytes, net_name):
    steps = 3
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, 'r0.pt')
        mp.spawn(_rank_main, args=(2, _free_port(), out, steps, bucket_bytes, net_name), nprocs=2, join=True)
        res = torch.load(out, weights_only=True)
    ref_params, ref_sums = _single_process(steps, net_name)
    p0, p1 = (p.numpy() for p in res['params'])
    np.testing.assert_array_equal(p0, p1)                        # replicas stay identical
    np.testing.assert_allclose(p0, ref_params, rtol=1e-5, atol=1e-7)
    for k in ('p', 'v', 'ent', 'total', 'dcnt'):
        assert abs(res['sums'][k] - ref_sums[k]) <= 1e-4 * max(1.0, abs(ref_sums[k])), k
    if bucket_bytes == 1024:
        assert res['buckets'] > 1


def test_data_parallel_lr_is_the_global_batch_lr():
    """args['batch_size'] is the per-rank shard; one update SUMs the gradients of world_size shards,
    so the lr is the reference's for the global batch: 3e-8 * world_size * B * T (train.py:318-322)."""
    from handyrl_amd.trainer import LearnerStep, Trainer
    _, args = make_batch_and_args(B=8, T=9)
    step = LearnerStep(SmallNet(), args, torch.device('cpu'), world_size=4)
    assert step.current_lr() == pytest.approx(3e-8 * 4 * 8 * 9, rel=1e-12)
    tr = Trainer(args, SmallNet(), batcher=None, device=torch.device('cpu'), world_size=4)
    assert tr.data_cnt_ema == 4 * 8 * 9
    assert tr.learner.current_lr() == pytest.approx(3e-8 * 4 * 8 * 9, rel=1e-12)


def test_bucket_layout_covers_flat_buffer():
    from handyrl_amd.distributed import FlatGrads
    net = SmallNet()
    fg = FlatGrads(list(net.parameters()))
    for p in net.parameters():
        assert p.grad.data_ptr() >= fg.flat.data_ptr()
        assert p.grad.shape == p.shape
    assert fg.flat.numel() == sum(p.numel() for p in net.parameters())


class _Deferred(torch.autograd.Function):
    """y = x @ w.T whose weight gradient is held back (returned as None, so w's accumulate hook fires with
    nothing added) and written later by a flush -- nn.DeferredGrads' pattern for a recurrent unroll."""

    @staticmethod
    def forward(ctx, x, w, store):
        ctx.save_for_backward(x, w)
        ctx.store = store
        return x @ w.t()

    @staticmethod
    def backward(ctx, g):
        x, w = ctx.saved_tensors
        ctx.store.append(g.t() @ x)
        return g @ w, None, None


def _deferred_rank_main(rank, world, port, out_path, steps, slow):
    """Each rank: two unrolled uses of a deferred weight and a plain head; after the backward the flush
    adds the held-back weight gradients and marks them ready.  ``slow`` delays the flush, so a bucket
    launched at the weight's hook (before its gradient is complete) would all-reduce a partial sum."""
    import time
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    from handyrl_amd.distributed import FlatGrads, GradAllReduce
    dist.init_process_group('gloo', rank=rank, world_size=world)
    torch.manual_seed(0)
    w = nn.Parameter(torch.randn(6, 6))
    head = nn.Linear(6, 1)
    fg = FlatGrads([w, head.weight, head.bias])
    red = GradAllReduce(fg, bucket_bytes=64)         # a bucket per parameter
    g = torch.Generator().manual_seed(10 + rank)
    out = []
    for _ in range(steps):
        fg.zero()
        x = torch.randn(5, 6, generator=g)
        store = []
        h = torch.tanh(_Deferred.apply(torch.tanh(_Deferred.apply(x, w, store)), w, store))
        head(h).square().sum().backward()
        if slow:
            time.sleep(0.2)
        w.grad.add_(sum(store))
        red.mark_ready([w, w])
        red.finish()
        out.append(fg.flat.clone())
    gathered = [torch.zeros_like(torch.stack(out)) for _ in range(world)]
    dist.all_gather(gathered, torch.stack(out))
    if rank == 0:
        torch.save({'flat': gathered, 'expected': red.expected}, out_path)
    dist.destroy_process_group()


def test_deferred_gradient_bucket_waits_for_the_flush():
    """A parameter whose gradient arrives in two events (its accumulate hook, then mark_ready after a flush)
    counts for its bucket only at the second from the second step on: both ranks end every step with the
    same summed gradient, equal to the sum of the ranks' own full gradients."""
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, 'r0.pt')
        mp.spawn(_deferred_rank_main, args=(2, _free_port(), out, 3, True), nprocs=2, join=True)
        res = torch.load(out, weights_only=True)
    assert res['expected'] == [2, 1, 1]
    a, b = res['flat']
    assert torch.equal(a, b)
    # each rank's own (un-reduced) gradient, recomputed in-process
    torch.manual_seed(0)
    w = nn.Parameter(torch.randn(6, 6))
    head = nn.Linear(6, 1)
    tot = None
    for r in range(2):
        g = torch.Generator().manual_seed(10 + r)
        rows = []
        for _ in range(3):
            w.grad = None
            head.zero_grad(set_to_none=True)
            x = torch.randn(5, 6, generator=g)
            h = torch.tanh(torch.tanh(x @ w.t()) @ w.t())
            head(h).square().sum().backward()
            rows.append(torch.cat([w.grad.reshape(-1), head.weight.grad.reshape(-1), head.bias.grad]))
        tot = torch.stack(rows) if tot is None else tot + torch.stack(rows)
    torch.testing.assert_close(a, tot, rtol=1e-5, atol=1e-6)


def _gpu_rank_main(rank, world, port, out_path, steps, graph=False):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK='0')
    from handyrl_amd.trainer import LearnerStep
    dev = torch.device('cuda', 0)
    torch.cuda.set_device(dev)
    # gloo over device tensors: exercises the product's bucketed hook-launched all-reduce and the HIP
    # learner step with two ranks on one GPU (RCCL itself needs one GPU per rank)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    batch, args = make_batch_and_args(B=64, T=9)
    batch = {k: v.to(dev) for k, v in batch.items()}
    B = batch['value'].size(0)
    shard = {k: v[rank * B // world:(rank + 1) * B // world].contiguous() for k, v in batch.items()}
    args = dict(args, batch_size=B // world)   # per-rank shard; LearnerStep's lr is the global batch's
    torch.manual_seed(0)
    net = SmallNet()
    step = LearnerStep(net, args, dev, world_size=world, bucket_bytes=1024, graph=graph)
    for _ in range(steps):
        step.step(shard)
    sums, _ = step.pop_stats()
    flat = torch.cat([p.detach().reshape(-1) for p in net.parameters()]).cpu()
    gathered = [torch.zeros_like(flat) for _ in range(world)]
    dist.all_gather(gathered, flat)
    if rank == 0:
        torch.save({'params': gathered, 'sums': sums}, out_path)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize('graph', [False, True])
def test_two_rank_gpu_step_matches_full_batch(cuda, graph):
    """Eager (hook-launched buckets) and graph-captured (backward graph, flat all-reduce, update graph)
    data-parallel steps both reproduce the full-batch single-process update."""
    from handyrl_amd.trainer import LearnerStep
    steps = 3
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, 'r0.pt')
        mp.spawn(_gpu_rank_main, args=(2, _free_port(), out, steps, graph), nprocs=2, join=True)
        res = torch.load(out, weights_only=True)
    batch, args = make_batch_and_args(B=64, T=9)
    batch = {k: v.to(cuda) for k, v in batch.items()}
    torch.manual_seed(0)
    net = SmallNet()
    step = LearnerStep(net, args, cuda)
    for _ in range(steps):
        step.step(batch)
    ref_sums, _ = step.pop_stats()
    ref = torch.cat([p.detach().reshape(-1) for p in net.parameters()]).cpu()
    p0, p1 = res['params']
    assert torch.equal(p0, p1)
    assert torch.allclose(p0, ref, rtol=1e-5, atol=1e-6), (p0 - ref).abs().max()
    for k in ('p', 'v', 'ent', 'total', 'dcnt'):
        assert abs(res['sums'][k] - ref_sums[k]) <= 1e-4 * max(1.0, abs(ref_sums[k])), k


def _rccl_rank_main(rank, world, port, out_path, steps):
    """One rank over the real RCCL backend: LearnerStep with a reducer (world_size forced to 2 so the
    data-parallel path is built) in HIP-graph mode -- backward graph, eager RCCL all-reduce, update graph --
    on a one-rank communicator, where the SUM all-reduce is the identity."""
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK='0')
    from handyrl_amd.envs.tictactoe import SimpleConv2dModel
    from handyrl_amd.synthetic import tictactoe_batch, default_args
    from handyrl_amd.trainer import LearnerStep
    dev = torch.device('cuda', 0)
    torch.cuda.set_device(dev)
    dist.init_process_group('nccl', rank=rank, world_size=world, device_id=dev)
    B, T = 64, 9
    args = default_args(T, B)
    batch = tictactoe_batch(B, T, dev, seed=4)
    torch.manual_seed(0)
    # world_size 2 on a one-rank communicator: pin the lr to the single-GPU step's (train.py:318)
    step = LearnerStep(SimpleConv2dModel(), args, dev, graph=True, world_size=2, lr=3e-8 * B * T)
    assert step.reducer is not None
    for _ in range(steps):
        step.step(batch)
    sums, _ = step.pop_stats()
    flat = torch.cat([p.detach().reshape(-1) for p in step.net.parameters()]).cpu()
    torch.save({'params': flat, 'sums': sums, 'split': step._graph_update is not None}, out_path)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.gpu
def test_rccl_graph_step_matches_single_gpu_step(cuda):
    """The graph-captured data-parallel step over RCCL (the bench's N > 1 path) on a one-rank
    communicator equals the plain single-GPU graph step."""
    from handyrl_amd.envs.tictactoe import SimpleConv2dModel
    from handyrl_amd.synthetic import tictactoe_batch, default_args
    from handyrl_amd.trainer import LearnerStep
    steps = 3
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, 'r0.pt')
        mp.spawn(_rccl_rank_main, args=(1, _free_port(), out, steps), nprocs=1, join=True)
        res = torch.load(out, weights_only=True)
    assert res['split']
    B, T = 64, 9
    batch = tictactoe_batch(B, T, cuda, seed=4)
    torch.manual_seed(0)
    step = LearnerStep(SimpleConv2dModel(), default_args(T, B), cuda, graph=True)
    for _ in range(steps):
        step.step(batch)
    ref_sums, _ = step.pop_stats()
    ref = torch.cat([p.detach().reshape(-1) for p in step.net.parameters()]).cpu()
    torch.testing.assert_close(res['params'], ref, rtol=1e-5, atol=1e-6)
    for k in ('p', 'v', 'ent', 'total', 'dcnt'):
        assert abs(res['sums'][k] - ref_sums[k]) <= 1e-4 * max(1.0, abs(ref_sums[k])), k


def _segmented_rank_main(rank, world, port, out_path, steps, segment=True, name='TicTacToe'):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK='0')
    from handyrl_amd.trainer import LearnerStep, split_torus_tower
    dev = torch.device('cuda', 0)
    torch.cuda.set_device(dev)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    cls, batch, args, rec = _net_case(name, dev)
    B = batch['value'].size(0)
    shard = {k: (v[rank * B // world:(rank + 1) * B // world].contiguous() if isinstance(v, torch.Tensor) else
                 {kk: vv[rank * B // world:(rank + 1) * B // world].contiguous() for kk, vv in v.items()})
             for k, v in batch.items()}
    args = dict(args, batch_size=B // world)   # per-rank shard; LearnerStep's lr is the global batch's
    torch.manual_seed(0)
    net = cls()
    if not segment:
        split_torus_tower(net)   # the reference run: the same split tower (a segmented capture sets it itself)
    step = LearnerStep(net, args, dev, graph=True, world_size=world, segment_backward=segment)
    hidden = _hidden(net, B // world, batch['value'].size(2), dev) if rec else None
    for _ in range(steps):
        step.step(shard, hidden)
    sums, _ = step.pop_stats()
    names = {id(p): n for n, p in step.net.named_parameters()}
    sched = [([tuple(r) for r in ranges], [names[id(p)] for p in ps]) for ranges, ps in (step.segments or [])]
    flat = torch.cat([p.detach().reshape(-1) for p in step.net.parameters()]).cpu()
    gathered = [torch.zeros_like(flat) for _ in range(world)]
    dist.all_gather(gathered, flat)
    if rank == 0:
        torch.save({'params': gathered, 'sums': sums, 'sched': sched, 'numel': step.grads.flat.numel(),
                    'names': [(n, p.numel()) for n, p in step.net.named_parameters()],
                    'grads': step.grads.flat.detach().cpu(),
                    'seg2': step._graph_seg2 is not None, 'why': step.segment_error}, out_path)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.gpu
def test_segmented_graph_step_matches_one_segment_step(cuda):
    """Data-parallel graph step in two backward segments (the fused chain's input as the cut): the upper
    segment's gradients (loss, heads, conv chain) are all-reduced while the lower segment (the stem)
    replays.  The schedule: two segments, the stem's parameters alone below the cut, the two buckets'
    ranges disjoint and covering the flat buffer.  Two ranks (gloo, one GPU) give exactly the parameters
    and loss sums of the same two-rank step captured as one backward graph with one flat all-reduce (the
    TicTacToe net has BatchNorm, whose statistics are per replica, so the single-process full batch is not
    the reference here; SmallNet's test above covers that)."""
    steps = 3
    res = {}
    with tempfile.TemporaryDirectory() as d:
        for seg in (True, False):
            out = os.path.join(d, 'r0_%d.pt' % seg)
            mp.spawn(_segmented_rank_main, args=(2, _free_port(), out, steps, seg), nprocs=2, join=True)
            res[seg] = torch.load(out, weights_only=True)
    r, ref = res[True], res[False]
    assert r['seg2'] and len(r['sched']) == 2, r['why']
    assert not ref['seg2']
    (up_ranges, up_names), (low_ranges, low_names) = r['sched']
    assert sorted(low_names) == ['conv.bias', 'conv.weight'], low_names      # the stem (tictactoe.py:55)
    assert any(n.startswith('blocks.') for n in up_names) and any(n.startswith('head') for n in up_names)
    _check_same_step(r, ref, up_ranges, low_ranges)


def _check_same_step(r, ref, up_ranges, low_ranges):
    covered = sorted(up_ranges + low_ranges)
    assert covered[0][0] == 0 and covered[-1][1] == r['numel']
    assert all(a[1] <= b[0] for a, b in zip(covered, covered[1:]))           # disjoint
    p0, p1 = r['params']
    assert torch.equal(p0, p1)
    diff, off = {}, 0
    for n, k in r['names']:
        d = float((p0[off:off + k] - ref['params'][0][off:off + k]).abs().max())
        if d > 0:
            diff[n] = d
        off += k
    assert not diff, diff
    for k in ('p', 'v', 'ent', 'total', 'dcnt'):
        assert r['sums'][k] == ref['sums'][k], k


@pytest.mark.gpu
def test_segmented_geese_tower_step_matches_one_segment_step(cuda):
    """GeeseNet's data-parallel graph step in two backward segments: the torus tower runs as two Functions
    (units [0, 7) and [7, 13), hungry_geese.py:48-51), the cut is the tensor between them, and the upper segment's
    gradients (blocks 6-11 and the heads) are all-reduced while the lower segment (conv0 and blocks 0-5) replays.
    The schedule: two segments with exactly that parameter split, the buckets' ranges disjoint and covering the
    flat buffer.  Two ranks (gloo, one GPU) give exactly the parameters and loss sums of the same two-rank step
    captured as one backward graph (the same split tower) with one flat all-reduce."""
    steps = 2
    res = {}
    with tempfile.TemporaryDirectory() as d:
        for seg in (True, False):
            out = os.path.join(d, 'g_%d.pt' % seg)
            mp.spawn(_segmented_rank_main, args=(2, _free_port(), out, steps, seg, 'Geese'), nprocs=2, join=True)
            res[seg] = torch.load(out, weights_only=True)
    r, ref = res[True], res[False]
    assert r['seg2'] and len(r['sched']) == 2, r['why']
    assert not ref['seg2']
    (up_ranges, up_names), (low_ranges, low_names) = r['sched']
    lower_units = {'conv0'} | {'blocks.%d' % i for i in range(6)}
    assert {n.rsplit('.', 2)[0] if n.startswith('blocks.') else n.split('.')[0] for n in low_names} == lower_units, \
        low_names
    assert all(n.startswith(('blocks.', 'head_')) for n in up_names)
    assert {'blocks.%d' % i for i in range(6, 12)} <= {'.'.join(n.split('.')[:2]) for n in up_names}
    assert any(n.startswith('head_') for n in up_names)
    _check_same_step(r, ref, up_ranges, low_ranges)


@pytest.mark.gpu
def test_segmented_geister_flush_step_matches_one_segment_step(cuda):
    """GeisterNet's data-parallel graph step in two segments: the backward and the first flush phase (every
    weight outside the DRC cells: stem, heads, the grouped BatchNorms) in the first graph, whose bucket is
    all-reduced while the second graph flushes the cells' deferred weight gradients (nn.DeferredGrads late
    records, the DRC step's h-half convolutions).  The schedule: the cells' conv weights alone in the second
    segment, the ranges disjoint and covering the flat buffer.  Two ranks (gloo, one GPU) give exactly the
    parameters and loss sums of the same step captured as one backward graph with one flat all-reduce."""
    steps = 2
    res = {}
    with tempfile.TemporaryDirectory() as d:
        for seg in (True, False):
            out = os.path.join(d, 'q_%d.pt' % seg)
            mp.spawn(_segmented_rank_main, args=(2, _free_port(), out, steps, seg, 'Geister'), nprocs=2, join=True)
            res[seg] = torch.load(out, weights_only=True)
    r, ref = res[True], res[False]
    assert r['seg2'] and len(r['sched']) == 2, r['why']
    assert not ref['seg2']
    (early_ranges, early_names), (late_ranges, late_names) = r['sched']
    assert late_names and all(n.startswith('body.blocks.') for n in late_names), late_names   # weights + biases
    assert any(n.endswith('conv.weight') for n in late_names), late_names
    assert any(n.startswith('head') for n in early_names) and not any(n.startswith('body.blocks.')
                                                                     for n in early_names), early_names
    _check_same_step(r, ref, early_ranges, late_ranges)


def _net_case(name, dev):
    """(net class, batch, args, hidden maker) of a BatchNorm net the learner trains: the TicTacToe net,
    GeeseNet (configs[3], torus tower) or GeisterNet (recurrent: DeferredGrads -> mark_ready)."""
    from handyrl_amd.synthetic import tictactoe_batch, default_args, geese_batch, geese_args, geister_batch
    if name == 'TicTacToe':
        from handyrl_amd.envs.tictactoe import SimpleConv2dModel
        return SimpleConv2dModel, tictactoe_batch(64, 9, dev, seed=4), default_args(9, 64), None
    if name == 'Geese':
        from handyrl_amd.envs.hungry_geese import GeeseNet
        return GeeseNet, geese_batch(16, 8, dev, seed=4), geese_args(8, 16), None
    from handyrl_amd.envs.geister import GeisterNet
    return GeisterNet, geister_batch(16, 6, dev, seed=4), default_args(6, 16), True


def _hidden(net, B, P, dev):
    return tuple([h.to(dev) for h in hs] for hs in net.init_hidden([B, P]))


def _dp_rank_main(rank, world, port, out_path, name, graph):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK='0')
    from handyrl_amd.trainer import LearnerStep
    import handyrl_amd.distributed as hd
    dev = torch.device('cuda', 0)
    torch.cuda.set_device(dev)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    cls, batch, args, rec = _net_case(name, dev)
    B = batch['value'].size(0)
    shard = {k: (v[rank * B // world:(rank + 1) * B // world].contiguous() if isinstance(v, torch.Tensor) else
                 {kk: vv[rank * B // world:(rank + 1) * B // world].contiguous() for kk, vv in v.items()})
             for k, v in batch.items()}
    args = dict(args, batch_size=B // world)
    torch.manual_seed(0)
    net = cls()
    step = LearnerStep(net, args, dev, world_size=world, bucket_bytes=16 * 1024, graph=graph)
    launched = []
    real_finish = hd.GradAllReduce.finish

    def finish(self):
        launched.append(self._next)           # buckets launched during the backward, before finish()
        return real_finish(self)
    hd.GradAllReduce.finish = finish
    hidden = _hidden(net, B // world, batch['value'].size(2), dev) if rec else None
    for _ in range(2):
        step.step(shard, hidden)
    torch.cuda.synchronize()
    sums, _ = step.pop_stats()
    flat = torch.cat([p.detach().reshape(-1) for p in net.parameters()]).cpu()
    bufs = torch.cat([b.detach().double().reshape(-1) for b in net.buffers()]).cpu()
    gathered = [torch.zeros_like(flat) for _ in range(world)]
    dist.all_gather(gathered, flat)
    gb = [torch.zeros_like(bufs) for _ in range(world)]
    dist.all_gather(gb, bufs)
    if rank == 0:
        torch.save({'params': gathered, 'buffers': gb, 'sums': sums, 'launched': launched,
                    'nbuckets': len(step.reducer.buckets),
                    'expected': step.reducer.expected}, out_path)
    dist.barrier()
    dist.destroy_process_group()


def _simulated_dp(name, dev, steps=2, world=2, split=True):
    """The data-parallel update without any collective: one replica per shard (its own BatchNorm statistics,
    as under the reference's nn.DataParallel), each computing its shard's gradients with LearnerStep's own
    backward; the SUM of the replicas' gradients is clipped and applied by Adam with the global batch's lr
    (3e-8 * world * B_shard * T, train.py:318) on every replica."""
    from handyrl_amd.trainer import LearnerStep, split_torus_tower
    cls, batch, args, rec = _net_case(name, dev)
    B = batch['value'].size(0)
    args = dict(args, batch_size=B // world)
    lr = 3e-8 * B * args['forward_steps']
    shards = [{k: (v[r * B // world:(r + 1) * B // world].contiguous() if isinstance(v, torch.Tensor) else
                   {kk: vv[r * B // world:(r + 1) * B // world].contiguous() for kk, vv in v.items()})
               for k, v in batch.items()} for r in range(world)]
    reps = []
    for r in range(world):
        torch.manual_seed(0)
        net = cls()
        if split:                   # as a data-parallel graph LearnerStep runs GeeseNet's tower
            split_torus_tower(net)
        st = LearnerStep(net, args, dev, lr=lr)
        st.fold_deferral = False    # the shard's gradient complete in the flat buffer after _grads
        reps.append((net, st))
    for _ in range(steps):
        grads = []
        for (net, st), sh in zip(reps, shards):
            hidden = _hidden(net, B // world, batch['value'].size(2), dev) if rec else None
            st._grads(sh, hidden)
            grads.append(st.grads.flat.clone())
        total = sum(grads[1:], grads[0].clone())
        for net, st in reps:
            st.grads.flat.copy_(total)
            if st.tail is not None:      # clip + Adam as the step tail's two launches
                st.tail(None)
            else:
                st.grads.clip_(4.0)
                st.optimizer.step()
    torch.cuda.synchronize()
    params = torch.cat([p.detach().reshape(-1) for p in reps[0][0].parameters()]).cpu()
    bufs = [torch.cat([b.detach().double().reshape(-1) for b in net.buffers()]).cpu() for net, _ in reps]
    return params, bufs


@pytest.mark.gpu
@pytest.mark.parametrize('name', ['TicTacToe', 'Geese', 'Geister'])
@pytest.mark.parametrize('graph', [False, True])
def test_two_rank_bn_nets_match_simulated_replicas(cuda, name, graph):
    """Two ranks (gloo over device tensors, one GPU) train the TicTacToe net, GeeseNet (torus tower) and
    GeisterNet (recurrent unroll, batched weight gradients marked ready at their flush) for two steps,
    eager (hook-launched buckets) and HIP-graph (flat all-reduce between the backward and
    update graphs): parameters equal on both ranks and equal to the collective-free simulation of the same
    update (per-replica BatchNorm, summed gradients, clip, Adam at the global lr); each rank's BatchNorm
    statistics are its replica's.  Eager: from the second step on buckets launch during the backward, each
    when its parameters' last gradient event (accumulate hook, or mark_ready after DeferredGrads.flush) has
    come, as the first step counted them."""
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, 'r0.pt')
        mp.spawn(_dp_rank_main, args=(2, _free_port(), out, name, graph), nprocs=2, join=True)
        res = torch.load(out, weights_only=True)
    ref, ref_bufs = _simulated_dp(name, cuda, split=graph)   # eager data-parallel steps keep one tower
    p0, p1 = res['params']
    assert torch.equal(p0, p1)
    torch.testing.assert_close(p0, ref, rtol=1e-5, atol=2e-6)
    for r in range(2):
        torch.testing.assert_close(res['buffers'][r], ref_bufs[r], rtol=1e-5, atol=1e-6)
    if not graph:
        assert res['launched'][0] == 0                     # the learning step launches at finish()
        assert res['launched'][-1] > 0, res['launched']   # second step: buckets launched before finish()
        if name == 'Geister':   # deferred weights: the accumulate hook, then mark_ready after the flush
            assert 2 in res['expected'], res['expected']


def _schedule_rank_main(rank, world, port, out_path):
    """One rank of the segmented graph step's replay schedule (LearnerStep.step, the path bench.py --gpus N
    takes every timed step), with recording stand-ins for the three captured graphs: each stand-in logs its
    replay and writes this rank's values into its segment's range of the flat gradient buffer, as the real
    graph's kernels would; the all-reduce calls are the product's (GradAllReduce.all_reduce_ranges over gloo),
    wrapped to log their issue and their waits."""
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    from handyrl_amd import distributed as hdist
    from handyrl_amd.trainer import LearnerStep
    hdist.init_process_group('cpu')
    batch, args = make_batch_and_args()
    step = LearnerStep(SmallNet(), args, torch.device('cpu'), world_size=world, loss_fn=oracle_loss)
    flat = step.grads.flat
    n = flat.numel()
    log = []

    class Graph:
        def __init__(self, name, lo=0, hi=0):
            self.name, self.lo, self.hi = name, lo, hi

        def replay(self):
            log.append('replay:' + self.name)
            if self.hi > self.lo:     # this rank's gradients of the segment: rank + 1 + element index
                flat[self.lo:self.hi] = torch.arange(self.lo, self.hi, dtype=torch.float32) + (rank + 1)

    cut = n // 3
    upper, lower = [(cut, n)], [(0, cut)]
    step.graph = True
    step.segments = [(upper, []), (lower, [])]
    step._graph = Graph('upper', cut, n)
    step._graph_seg2 = Graph('lower', 0, cut)
    step._graph_update = Graph('update')
    step._static, step._static_hidden = batch, None
    step._static_out = {'total': torch.zeros(())}
    real = step.reducer.all_reduce_ranges

    class Work:
        def __init__(self, w, tag):
            self.w, self.tag = w, tag

        def wait(self):
            log.append('wait:' + self.tag)
            return self.w.wait()

    def all_reduce_ranges(ranges):
        tag = 'upper' if ranges == upper else ('lower' if ranges == lower else repr(ranges))
        log.append('issue:' + tag)
        return [Work(w, tag) for w in real(ranges)]
    step.reducer.all_reduce_ranges = all_reduce_ranges
    for _ in range(2):
        log.append('step')
        step.step(batch)
    ref = torch.arange(n, dtype=torch.float32) * world + sum(r + 1 for r in range(world))
    if rank == 0:
        torch.save({'log': log, 'flat': flat.clone(), 'ref': ref}, out_path)
    dist.barrier()
    dist.destroy_process_group()


def test_segmented_graph_replay_schedule_two_ranks():
    """The per-step order of the data-parallel graph step (bench.py --gpus N), two gloo ranks on the
    CPU: upper graph (loss, heads, chain) -> the upper segment's all-reduce issued -> lower graph (stem) replays
    while it runs -> the lower segment's all-reduce -> both waited for -> update graph (clip, Adam); and each
    segment's range of the flat buffer is the SUM over the ranks of what that rank's graph wrote (the upper
    range all-reduced only after the upper graph wrote it, the lower only after the lower one)."""
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, 'sched.pt')
        mp.spawn(_schedule_rank_main, args=(2, _free_port(), out), nprocs=2, join=True)
        res = torch.load(out, weights_only=True)
    one = ['replay:upper', 'issue:upper', 'replay:lower', 'issue:lower', 'wait:upper', 'wait:lower',
           'replay:update']
    assert res['log'] == ['step'] + one + ['step'] + one, res['log']
    assert torch.equal(res['flat'], res['ref'])
