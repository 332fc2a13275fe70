"""Data parallelism for the learner: one process per GPU, SUM all-reduce over RCCL.

Replaces the reference's single-process ``nn.DataParallel`` (train.py:364-367).
The trajectory batch shards along B: every rank runs the full learner step on
its own (B_local, T, P) batch, and the ONLY exchange is the gradient
all-reduce.  It is a SUM, not a mean: the reference losses are sums over the
batch (train.py:202-213) and the learning rate is scaled by the data count
(train.py:318-322), so averaging would shrink the update by 1/world_size.

Gradients live in one flat fp32 buffer (each ``p.grad`` is a view into it),
cut into a few buckets in backward order.  A post-accumulate-grad hook on each
parameter launches its bucket's asynchronous all-reduce the moment the
bucket's last gradient is ready, so the collectives run on RCCL's stream while
autograd is still computing the earlier layers' gradients; ``finish()`` makes
the compute stream wait for them before clipping and Adam.  The model
gradients are 116 KB (TicTacToe) to 935 KB (Geister): latency-bound messages
on xGMI, so buckets are few and large.

BatchNorm keeps per-replica batch statistics, as under DataParallel.
"""

import os

import torch
import torch.distributed as dist


def world_from_env():
    """(rank, world_size, local_rank) from the torchrun environment (defaults 0, 1, 0)."""
    rank = int(os.environ.get('RANK', '0'))
    world = int(os.environ.get('WORLD_SIZE', '1'))
    local = int(os.environ.get('LOCAL_RANK', str(rank)))
    return rank, world, local


def init_process_group(device_type):
    """Initialise torch.distributed when launched with WORLD_SIZE > 1.

    Backend ``nccl`` (RCCL on ROCm) for GPUs, ``gloo`` for CPU tests.
    """
    rank, world, local = world_from_env()
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
        os.environ.setdefault('MASTER_PORT', '29533')
        backend = 'nccl' if device_type == 'cuda' else 'gloo'
        # HRL_DIST_BACKEND=gloo: several ranks on ONE GPU (RCCL refuses two ranks on one device), the
        # one-GPU box's rehearsal of the multi-rank bench; gloo all-reduces device tensors via the host
        backend = os.environ.get('HRL_DIST_BACKEND', backend)
        kwargs = {}
        if device_type == 'cuda' and backend == 'nccl':
            kwargs['device_id'] = torch.device('cuda', local)
        dist.init_process_group(backend, rank=rank, world_size=world, **kwargs)
    return rank, world, local


class FlatGrads:
    """One contiguous gradient buffer; every ``p.grad`` is a view into it."""

    def __init__(self, params):
        self.params = [p for p in params if p.requires_grad]
        numel = sum(p.numel() for p in self.params)
        dev = self.params[0].device
        self.flat = torch.zeros(numel, dtype=torch.float32, device=dev)
        self._total = None
        self.slices = []
        off = 0
        for p in self.params:
            n = p.numel()
            p.grad = self.flat[off:off + n].view_as(p)
            self.slices.append((off, n))
            off += n

    def zero(self):
        self.flat.zero_()

    def norm(self):
        return torch.linalg.vector_norm(self.flat, 2)

    def clip_(self, max_norm):
        """clip_grad_norm_(params, max_norm) on the flat buffer, without a host sync (train.py:384);
        on the GPU one csrc/hrl_optim.hip launch instead of six torch ops."""
        if self.flat.is_cuda:
            from . import _native
            lib = _native.load()
            if self._total is None:
                self._total = torch.empty((), dtype=torch.float32, device=self.flat.device)
                self._clip_ws = torch.empty(max(lib.hrl_clip_workspace_bytes(self.flat.numel()), 8),
                                            dtype=torch.uint8, device=self.flat.device)
            _native.check(lib.hrl_clip_grad_norm_ws(_native.ptr(self.flat), self.flat.numel(), float(max_norm),
                                                    _native.ptr(self._total), _native.ptr(self._clip_ws),
                                                    self._clip_ws.numel(), _native.stream_of(self.flat.device)),
                          'hrl_clip_grad_norm')
            return self._total
        total = self.norm()
        coef = torch.clamp(max_norm / (total + 1e-6), max=1.0)
        self.flat.mul_(coef)
        return total


class GradAllReduce:
    """Bucketed, backward-overlapped SUM all-reduce of a FlatGrads buffer.

    A bucket's all-reduce is launched as soon as every gradient in it is final.  When that is, the first
    step learns: a parameter's gradient can arrive in several events -- its autograd accumulate hook (which
    also fires when a HIP Function wrote the gradient in place and returned None, nn.direct_grads), and
    mark_ready() after nn.DeferredGrads.flush has added the batched weight gradients of a recurrent unroll,
    i.e. after that parameter's hook already fired.  The first step counts each parameter's events and
    launches every bucket at finish(); later steps count a parameter for its bucket at its last event.  A
    parameter that gets no gradient (expected 0 events) never holds its bucket back."""

    def __init__(self, flat_grads, group=None, bucket_bytes=256 * 1024):
        self.fg = flat_grads
        self.group = group
        params = flat_grads.params
        # buckets over params in reverse registration order (≈ backward order);
        # each bucket is a contiguous range of the flat buffer.
        self.buckets = []           # (start, end) element ranges, launch order
        self.param_bucket = {}
        cur, cur_lo, cur_hi = [], None, None
        for i in reversed(range(len(params))):
            off, n = flat_grads.slices[i]
            cur.append(i)
            cur_lo = off if cur_lo is None else min(cur_lo, off)
            cur_hi = off + n if cur_hi is None else max(cur_hi, off + n)
            if (cur_hi - cur_lo) * 4 >= bucket_bytes or i == 0:
                bid = len(self.buckets)
                self.buckets.append((cur_lo, cur_hi))
                for j in cur:
                    self.param_bucket[j] = bid
                cur, cur_lo, cur_hi = [], None, None
        self._index = {id(p): i for i, p in enumerate(params)}
        self.expected = None        # per parameter: gradient events per step (learned in the first step)
        self._seen = [0] * len(params)
        self.bucket_size = [0] * len(self.buckets)
        self._pending = list(self.bucket_size)
        self._works = [None] * len(self.buckets)
        self._next = 0
        self._hooks = [p.register_post_accumulate_grad_hook(self._make_hook(i)) for i, p in enumerate(params)]

    def _make_hook(self, i):
        def hook(_param):
            self._event(i)
        return hook

    enabled = True

    def _event(self, i):
        if not self.enabled:
            return      # a probe or capture pass: nothing is counted (and nothing launched)
        self._seen[i] += 1
        if self.expected is None:
            return      # the learning step: every bucket launches at finish()
        if self._seen[i] > self.expected[i]:
            raise RuntimeError('parameter %d got %d gradient events this step, %d in the first: its bucket was '
                               'already all-reduced' % (i, self._seen[i], self.expected[i]))
        if self._seen[i] == self.expected[i]:
            self._pending[self.param_bucket[i]] -= 1
            self._launch_ready()

    def mark_ready(self, params):
        """Params whose gradient was written outside autograd (nn.DeferredGrads.flush): one more gradient
        event each, however often a parameter appears in ``params``."""
        if not self.enabled:
            return
        for i in sorted({self._index[id(p)] for p in params if id(p) in self._index}):
            self._event(i)

    def _launch_ready(self):
        if not self.enabled:
            return
        # launch strictly in bucket order so every rank issues the same sequence
        while self._next < len(self.buckets) and self._pending[self._next] == 0:
            lo, hi = self.buckets[self._next]
            self._works[self._next] = dist.all_reduce(self.fg.flat[lo:hi], op=dist.ReduceOp.SUM,
                                                      group=self.group, async_op=True)
            self._next += 1

    def finish(self):
        """Launch the buckets not launched yet (all of them in the learning step), then wait for all."""
        if self.expected is None and any(self._seen):
            self.expected = list(self._seen)
            self.bucket_size = [0] * len(self.buckets)
            for j, b in self.param_bucket.items():
                if self.expected[j] > 0:
                    self.bucket_size[b] += 1
        for b in range(self._next, len(self.buckets)):
            self._pending[b] = 0
        self._launch_ready()
        for w in self._works:
            if w is not None:
                w.wait()
        self.reset()

    def reset(self):
        """Forget a partially counted step (after a probe or a capture, whose hooks counted nothing)."""
        self._pending = list(self.bucket_size)
        self._works = [None] * len(self.buckets)
        self._next = 0
        self._seen = [0] * len(self._seen)

    def all_reduce_flat(self):
        """SUM all-reduce of the whole flat buffer as one message, ordered on the current stream
        (the graph-captured step: between the backward graph and the clip/Adam graph)."""
        dist.all_reduce(self.fg.flat, op=dist.ReduceOp.SUM, group=self.group)

    def all_reduce_ranges(self, ranges):
        """Asynchronous SUM all-reduce of element ranges of the flat buffer (one message each), ordered
        after the work already enqueued on the current stream; returns the work handles."""
        return [dist.all_reduce(self.fg.flat[lo:hi], op=dist.ReduceOp.SUM, group=self.group, async_op=True)
                for lo, hi in ranges]

    def remove(self):
        for h in self._hooks:
            h.remove()


def all_reduce_sum_(tensors, group=None):
    """SUM-reduce a list of small tensors (loss sums, dcnt) in one flat message."""
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return tensors
    flat = torch.cat([t.reshape(-1) for t in tensors])
    dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=group)
    out, off = [], 0
    for t in tensors:
        out.append(flat[off:off + t.numel()].view_as(t))
        off += t.numel()
    return out
