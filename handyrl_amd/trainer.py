"""The learner update on MI355X (handyrl/train.py:312-414, Trainer).

``LearnerStep`` is one iteration of the reference's training loop body
(train.py:372-392) on a device-resident batch:

    forward_prediction -> IS ratios -> fused HIP target scans -> losses
    -> backward (+ bucketed RCCL SUM all-reduce, overlapped) -> clip 4.0
    -> Adam(lr = 3e-8 * data_cnt_ema, weight_decay = 1e-5)

differences from the reference that do not change the arithmetic:
* no ``.item()`` in the step: loss sums and ``dcnt`` accumulate on the device
  and are read once per epoch (train.py:199, :390 sync every step);
* gradients sit in one flat buffer (zeroed by one kernel, clipped by one
  norm, all-reduced in a few buckets);
* optionally the whole step is captured once in a HIP graph and replayed
  (``graph=True``): the batch tensors are then static buffers that the caller
  refills (``load_batch``), exactly like a graph's input slots.

``Trainer`` keeps the reference class's epoch API (``train()`` returns a CPU
copy of the model, lr schedule at epoch end, train.py:357-401) over any batch
source with a ``batch()`` method.
"""

import contextlib
import copy

import torch
import torch.nn as nn

from . import distributed as hdist
from .nn import accelerate, fuse_bn_relu, deferred_weight_grads, deferred_folds, direct_grads
from .train import backward_total, forward_prediction, loss_terms
from .util import map_r, bimap_r

DEFAULT_LR = 3e-8  # train.py:318


class StepTail:
    """clip_grad_norm_(4.0) + torch.optim.Adam(lr, weight_decay=1e-5) (train.py:322, 384-385) over the learner's
    flat gradient buffer as two HIP launches (csrc/hrl_optim.hip): hrl_grad_fold_norm (the deferred weight-gradient
    folds of the step's HIP Functions, the norm's per-block sums of squares, the step count and the BatchNorm
    batch counters) and hrl_adam_clip (the clip coefficient from those sums, the in-place scaling -- p.grad holds
    the clipped gradient afterwards, as in the reference -- and torch's fused Adam arithmetic on the parameters
    that receive a gradient).  Replaces the clip launch, torch's step-count / counter increments, its fused Adam
    and the Functions' reduce launches.  lr and the step count are device scalars, so a captured graph replays
    with their current values."""

    def __init__(self, grads, lr, weight_decay=1e-5, betas=(0.9, 0.999), eps=1e-8, max_norm=4.0):
        from . import _native
        self.lib = _native.load()
        self.grads = grads
        flat = grads.flat
        dev = flat.device
        n = flat.numel()
        self.n = n
        self.m = torch.zeros(n, dtype=torch.float32, device=dev)
        self.v = torch.zeros(n, dtype=torch.float32, device=dev)
        self.step_t = torch.zeros((), dtype=torch.float32, device=dev)
        self.lr_t = torch.tensor(float(lr), dtype=torch.float32, device=dev)
        self.norm_part = torch.empty(self.lib.hrl_grad_fold_norm_blocks(n), dtype=torch.float64, device=dev)
        self.total = torch.empty((), dtype=torch.float32, device=dev)
        self.wd, self.betas, self.eps, self.max_norm = weight_decay, betas, eps, max_norm
        params = grads.params
        self.ptrs = _native.ptr_array(params)
        self.offsets = _native.i64_array([off for off, _ in grads.slices] + [n])
        self.set_live([True] * len(params))

    @staticmethod
    def supports(params):
        return (0 < len(params) <= 64 and all(p.is_cuda and p.dtype == torch.float32 and p.is_contiguous()
                                             for p in params))

    def set_live(self, live):
        import ctypes
        self.live = (ctypes.c_int * len(live))(*[int(x) for x in live])

    def set_lr(self, lr):
        self.lr_t.fill_(lr)

    def state_tensors(self):
        return [self.m, self.v, self.step_t]

    def __call__(self, folds=None, acc=None):
        """Fold, clip and update; folds: a finished nn.deferred_folds (or None); acc: (sources, dst) -- dst[k] +=
        sources[k] (0-dim float32 device tensors, self.total for the norm) in the same launch.  Returns the norm
        (device)."""
        from . import _native
        lib, P = self.lib, _native.ptr
        flat = self.grads.flat
        base = flat.data_ptr()
        fl = folds.folds if folds is not None else []
        counters = folds.counters if folds is not None else []
        incs = folds.increments if folds is not None else []
        if len(fl) > 16 or len(counters) > 8:
            raise ValueError('step tail: %d folds / %d counters (at most 16 / 8)' % (len(fl), len(counters)))
        dst = []
        for f in fl:
            off = (f[4].data_ptr() - base) // 4
            if f[4].data_ptr() % 4 or off < 0 or off + f[5] > self.n:
                raise ValueError('step tail: a fold destination outside the flat gradient buffer')
            dst.append(off)
        i64 = _native.i64_array
        import ctypes
        stream = _native.stream_of(flat.device)
        _native.check(lib.hrl_grad_fold_norm(
            P(flat), self.n, _native.ptr_array([f[0] for f in fl]), i64([f[1] for f in fl]),
            i64([f[2] for f in fl]), i64([f[3] for f in fl]), i64(dst), i64([f[5] for f in fl]),
            (ctypes.c_int * max(len(fl), 1))(*[f[6] for f in fl]), len(fl), P(self.step_t),
            _native.ptr_array(counters), i64(incs) if incs else None, len(counters), P(self.norm_part),
            self.norm_part.numel() * 8, stream),
            'hrl_grad_fold_norm')
        srcs, acc_dst = acc if acc is not None else ([], None)
        acc_src = (ctypes.c_void_p * max(len(srcs), 1))(*[None if t is self.total else t.data_ptr() for t in srcs])
        _native.check(lib.hrl_adam_clip(
            P(flat), self.n, P(self.norm_part), float(self.max_norm), P(self.total), self.ptrs, self.offsets,
            self.live, len(self.live), P(self.m), P(self.v), P(self.lr_t), P(self.step_t), float(self.betas[0]),
            float(self.betas[1]), float(self.eps), float(self.wd), acc_src, len(srcs), P(acc_dst), stream),
            'hrl_adam_clip')
        return self.total


def split_torus_tower(net, on=True):
    """Run a torus-conv tower (GeeseNet) as two Functions split after its middle unit (nn.torus_tower), so a
    data-parallel segmented capture can all-reduce the upper half's gradients while the lower half's backward
    replays (hungry_geese.py:48-51: conv0 and 12 blocks -> units [0, 7) and [7, 13)).  Same values as the one
    Function up to the order of the BatchNorm sums at the split.  on=False removes the split again."""
    from .envs.hungry_geese import TorusConv2d
    torus = [m for m in net.modules() if isinstance(m, TorusConv2d)]
    if len(torus) >= 2:
        torus[0].tower_split = (len(torus) + 1) // 2 if on else None


class LearnerStep:
    def __init__(self, net, args, device, lr=None, graph=False, reduce_group=None, world_size=1,
                 bucket_bytes=256 * 1024, hip_layers=True, loss_fn=None, segment_backward=True):
        self.net = net.to(device)
        self._fuse_pending = False
        if hip_layers and device.type == 'cuda':
            accelerate(self.net)  # HIP BatchNorm etc.; same parameters and state_dict
            self._fuse_pending = True  # BN->ReLU fusion, checked on the first batch
        self.args = args
        self.device = device
        # loss_fn(outputs, batch, args) -> (losses, dcnt tensor); the HIP path by default
        self.loss_fn = loss_fn or loss_terms
        self.graph = graph and device.type == 'cuda'
        self.params = [p for p in self.net.parameters() if p.requires_grad]
        self.grads = hdist.FlatGrads(self.params)
        self.reducer = None
        if world_size > 1:
            self.reducer = hdist.GradAllReduce(self.grads, group=reduce_group, bucket_bytes=bucket_bytes)
            if self.graph and segment_backward:
                split_torus_tower(self.net)   # only a segmented capture uses the cut (eager: one Function)
        if lr is None:
            # train.py:318-321: lr = 3e-8 * batch_size * forward_steps for the batch ONE update sees.
            # Here args['batch_size'] is the per-rank shard and the gradients are SUMmed over the ranks,
            # so one update sees world_size * batch_size windows (nn.DataParallel's global batch).
            lr = DEFAULT_LR * args['batch_size'] * world_size * args['forward_steps']
        # one fused multi-tensor Adam kernel on the GPU (train.py:322: Adam, weight_decay 1e-5)
        fused = device.type == 'cuda'
        if self.graph:
            self._opt_kwargs = dict(lr=torch.tensor(lr, device=device), weight_decay=1e-5, capturable=True,
                                    fused=True)
        else:
            self._opt_kwargs = dict(lr=lr, weight_decay=1e-5, fused=fused, foreach=None if fused else True)
        # the step tail (clip + Adam, and on one GPU the Functions' deferred gradient folds) as two HIP launches;
        # torch's Adam where it does not apply (CPU, more than 64 parameter tensors)
        self.tail = StepTail(self.grads, lr) if (fused and StepTail.supports(self.params)) else None
        self.optimizer = None if self.tail is not None else torch.optim.Adam(self.params, **self._opt_kwargs)
        self.fold_deferral = self.tail is not None and world_size == 1
        self._folds = None
        self.live = None        # params that receive a gradient (set on the first batch)
        self.defer = hip_layers and device.type == 'cuda'   # batched weight gradients for recurrent steps
        self._graph = None
        self._graph_seg2 = None     # data parallel: the backward below the cut (second segment)
        self._graph_update = None
        self.segments = None        # data parallel: [(flat-buffer ranges, params)] per backward segment
        self.segment_error = None   # why the step stayed one backward graph
        self._late_ids = set()      # recurrent nets: the weights whose deferred gradients are flushed last
        self.segment_backward = segment_backward
        self._cut = None            # forward pre-hook state: the fused chain's input (the segment cut)
        self._static = None
        self._static_out = None
        self.stats = None
        self._tail_stats = False

    # -- learning rate (train.py:396-398) ---------------------------------
    def current_lr(self):
        """The lr the next update uses (a float; the step tail's and a capturable Adam's live on the device)."""
        lr = self.tail.lr_t if self.tail is not None else self.optimizer.param_groups[0]['lr']
        return float(lr)

    def set_lr(self, lr):
        if self.tail is not None:
            self.tail.set_lr(lr)
            return
        for group in self.optimizer.param_groups:
            if isinstance(group['lr'], torch.Tensor):
                group['lr'].fill_(lr)
            else:
                group['lr'] = lr

    # -- one update ----------------------------------------------------------
    def _probe_live(self, batch, hidden):
        """Which parameters receive a gradient at all (reference semantics: torch.optim.Adam skips a
        parameter whose .grad stays None -- no update, no weight decay; e.g. GeisterNet's first two DRC
        blocks never reach an output, geister.py:91-94).  One forward/backward on a 2-trajectory slice
        of the first batch with every .grad set to None; BatchNorm buffers are restored afterwards."""
        def head(x):
            return x[:2] if isinstance(x, torch.Tensor) and x.dim() > 0 else x
        small = map_r(batch, head)
        small_hidden = None if hidden is None else map_r(hidden, head)
        buffers = [b.detach().clone() for b in self.net.buffers()]
        views = [p.grad for p in self.params]
        for p in self.params:
            p.grad = None
        if self.reducer is not None:
            self.reducer.enabled = False    # its hooks neither count nor launch during the probe
        try:
            if hidden is not None and self.defer:
                # the step's own kernels (deferred weight gradients, flushed into .grad): no vendor-conv path
                # runs just for the probe
                with deferred_weight_grads() as deferred:
                    outputs = forward_prediction(self.net, small_hidden, small, self.args)
                    losses, _ = self.loss_fn(outputs, small, self.args)
                    backward_total(losses)
                deferred.flush()
            else:
                outputs = forward_prediction(self.net, small_hidden, small, self.args)
                losses, _ = self.loss_fn(outputs, small, self.args)
                backward_total(losses)
            live = [p.grad is not None for p in self.params]
        finally:
            for p, v in zip(self.params, views):
                p.grad = v
            for b, saved in zip(self.net.buffers(), buffers):
                b.copy_(saved)
            if self.reducer is not None:
                self.reducer.enabled = True
                self.reducer.reset()
        self.live = live
        if self.tail is not None:
            self.tail.set_live(live)   # a parameter with no gradient: no update, no weight decay
        elif not all(live):
            kw = dict(self._opt_kwargs)
            kw['lr'] = self.optimizer.param_groups[0]['lr']   # keep a set_lr() made before the first step
            self.optimizer = torch.optim.Adam([p for p, l in zip(self.params, live) if l], **kw)

    def _grads(self, batch, hidden):
        """zero -> forward_prediction -> losses -> backward; returns (losses, dcnt)."""
        if self.live is None:
            self._probe_live(batch, hidden)
        if self._fuse_pending:
            self._fuse_pending = False
            obs = batch['observation']
            if hidden is None and isinstance(obs, torch.Tensor):
                self.fused_pairs = fuse_bn_relu(self.net, obs[:2].reshape(-1, *obs.shape[3:]))
        self.grads.zero()
        if hidden is not None and self.defer:
            # recurrent unroll: every weight is used T times; batch its weight gradients (nn.DeferredGrads).  On
            # one GPU the single-use parameters' gradients are written in place (direct_grads: the grouped
            # BatchNorms) and the BatchNorm batch counters ride on the step tail (deferred_folds)
            single = self.reducer is None
            with deferred_weight_grads() as deferred, (direct_grads() if single else contextlib.nullcontext()), \
                    deferred_folds(enabled=self.fold_deferral) as df:
                outputs = forward_prediction(self.net, hidden, batch, self.args)
                losses, dcnt = self.loss_fn(outputs, batch, self.args)
                backward_total(losses)
            self._folds = df if self.fold_deferral else None
            self._late_ids = deferred.late_ids()
            if self.reducer is None:
                deferred.flush()
            else:
                # data parallel: the weights outside the recurrent cells first, so their buckets can launch
                # while the cells' (late) weight gradients are formed
                self.reducer.mark_ready(deferred.flush(phase=1))
                self.reducer.mark_ready(deferred.flush(phase=2))
        else:
            # the HIP Functions write single-use parameter gradients straight into the flat buffer
            # (zeroed above) instead of autograd's per-parameter accumulate-adds (nn.direct_grads); on one GPU
            # they leave them as partial rows that the step tail folds (nn.deferred_folds)
            with direct_grads(), deferred_folds(enabled=self.fold_deferral) as df:
                outputs = forward_prediction(self.net, hidden, batch, self.args)
                losses, dcnt = self.loss_fn(outputs, batch, self.args)
                backward_total(losses)
            self._folds = df if self.fold_deferral else None
        return losses, dcnt

    def _update(self, losses, dcnt):
        """clip_grad_norm_(4.0) on the (all-reduced) gradients, then Adam (train.py:384-385)."""
        out = {k: v.detach() for k, v in losses.items()}
        out['dcnt'] = dcnt
        if self.tail is not None:
            folds, self._folds = self._folds, None
            out['grad_norm'] = self.tail.total
            self._tail_stats = self._tail_accumulable(out)
            acc = None
            if self._tail_stats:
                # the running statistics are summed by the tail's second launch (no stack + add per step)
                if self.stats is None:
                    self.stats_keys = sorted(out)
                    self.stats = torch.zeros(len(out), dtype=torch.float32, device=self.device)
                    self.batches = 0
                acc = ([out[k] for k in self.stats_keys], self.stats)
            self.tail(folds, acc)
        else:
            out['grad_norm'] = self.grads.clip_(4.0)
            self.optimizer.step()
        return out

    def _tail_accumulable(self, out):
        keys = sorted(out)
        return (len(keys) <= 8 and (self.stats is None or self.stats_keys == keys) and
                all(isinstance(v, torch.Tensor) and v.numel() == 1 and v.dtype == torch.float32 and v.is_cuda
                    for v in out.values()))

    def snapshot(self):
        """A copy of the training state (parameters, buffers, Adam's state tensors) that restore() puts back in
        place, so captured graphs keep pointing at the same tensors."""
        with torch.no_grad():
            return ([p.detach().clone() for p in self.net.parameters()],
                    [b.detach().clone() for b in self.net.buffers()],
                    [(v, v.detach().clone()) for v in self._opt_state()])

    def restore(self, snap):
        params, buffers, opt = snap
        with torch.no_grad():
            for p, v in zip(self.net.parameters(), params):
                p.copy_(v)
            for b, v in zip(self.net.buffers(), buffers):
                b.copy_(v)
            for t, v in opt:
                t.copy_(v)

    def _opt_state(self):
        if self.tail is not None:
            # with the running statistics, which the tail accumulates (zeroed after a capture's warm-up too)
            return self.tail.state_tensors() + ([self.stats] if self._tail_stats else [])
        return [v for st in self.optimizer.state.values() for v in st.values() if isinstance(v, torch.Tensor)]

    def _body(self, batch, hidden):
        losses, dcnt = self._grads(batch, hidden)
        if self.reducer is not None:
            self.reducer.finish()
        return self._update(losses, dcnt)

    def _accumulate(self, out):
        if self._tail_stats:          # summed on the device by the step tail
            self.batches += 1
            return
        vec = torch.stack([out[k].reshape(()) for k in sorted(out)])
        if self.stats is None:
            self.stats_keys = sorted(out)
            self.stats = torch.zeros_like(vec)
            self.batches = 0
        self.stats += vec
        self.batches += 1

    def step(self, batch, hidden=None):
        """Run one update; returns the step's losses / dcnt as device tensors (no sync)."""
        if self.graph:
            if self._graph is None:
                self._capture(batch, hidden)
            else:
                if batch is not self._static:
                    self.load_batch(batch)
                if hidden is not None and hidden is not self._static_hidden:
                    bimap_r(self._static_hidden, hidden, lambda dst, src: dst.copy_(src, non_blocking=True))
            self._graph.replay()
            if self._graph_update is not None:
                if self._graph_seg2 is not None:
                    # data parallel, two backward segments: the upper segment's gradients are complete
                    # when its graph has run, so their all-reduce is enqueued (RCCL stream, eager) before
                    # the lower segment's graph and runs while it does; then the lower segment's bucket
                    works = [self.reducer.all_reduce_ranges(self.segments[0][0])]
                    self._graph_seg2.replay()
                    works.append(self.reducer.all_reduce_ranges(self.segments[1][0]))
                    for w in works:
                        for x in w:
                            x.wait()
                else:
                    # data parallel: the gradient exchange runs between the two graphs (eager RCCL
                    # all-reduce of the flat buffer, one message), then clip + Adam replay
                    self.reducer.all_reduce_flat()
                self._graph_update.replay()
            out = self._static_out
        else:
            out = self._body(batch, hidden)
        self._accumulate(out)
        return out

    def _capture(self, batch, hidden):
        """Capture the step in HIP graphs.

        One GPU: the whole step is one graph.  Data parallel: two graphs -- (zero, forward, loss,
        backward) and (clip, Adam) -- with the SUM all-reduce of the flat gradient buffer issued
        eagerly between their replays, so no collective is captured.
        """
        self._static = batch
        self._static_hidden = hidden  # recurrent nets: the window's initial state (zeros, train.py:375)
        # Warm up on a side stream (allocator pools, MIOpen kernel selection, lazy optimizer state),
        # then put the training state back so the first replay is the first update: parameters and
        # buffers restored in place, Adam's moments and step counts zeroed in place (the graph keeps
        # pointing at the same tensors).  Every rank runs the same warm-up (its collectives included).
        params = list(self.net.parameters())
        saved_p = [p.detach().clone() for p in params]
        saved_b = [b.detach().clone() for b in self.net.buffers()]
        side = torch.cuda.Stream(self.device)
        side.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(side):
            for _ in range(3):
                self._body(batch, hidden)
            if self.reducer is not None and hidden is None and self.segment_backward:
                self._try_plan_segments(batch)   # its forward's BatchNorm updates are undone below
            elif self.reducer is not None and hidden is not None and self.defer and self.segment_backward:
                self._plan_flush_segments()
        torch.cuda.current_stream(self.device).wait_stream(side)
        with torch.no_grad():
            for p, v in zip(params, saved_p):
                p.copy_(v)
            for b, v in zip(self.net.buffers(), saved_b):
                b.copy_(v)
            for v in self._opt_state():
                v.zero_()
        if self.reducer is None:
            self._graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self._graph):
                self._static_out = self._body(batch, hidden)
            return
        torch.cuda.synchronize(self.device)
        self.reducer.enabled = False     # no collective inside a capture
        seg2 = None
        try:
            grads_graph, update_graph = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
            # thread-local capture: the process group's watchdog thread may query its events meanwhile
            if self.segments is not None and hidden is not None:
                # recurrent net: the backward and the first flush phase, then the cells' flush
                seg2 = torch.cuda.CUDAGraph()
                with torch.cuda.graph(grads_graph, capture_error_mode='thread_local'):
                    self.grads.zero()
                    with deferred_weight_grads() as deferred:
                        outputs = forward_prediction(self.net, hidden, batch, self.args)
                        losses, dcnt = self.loss_fn(outputs, batch, self.args)
                        backward_total(losses)
                    deferred.flush(phase=1)
                with torch.cuda.graph(seg2, capture_error_mode='thread_local'):
                    deferred.flush(phase=2)
            elif self.segments is not None:
                seg2 = torch.cuda.CUDAGraph()
                with self._cut_hook():
                    with direct_grads():
                        with torch.cuda.graph(grads_graph, capture_error_mode='thread_local'):
                            self.grads.zero()
                            outputs = forward_prediction(self.net, hidden, batch, self.args)
                            losses, dcnt = self.loss_fn(outputs, batch, self.args)
                            cut, upper, lower = self._cut, self.segments[0][1], self.segments[1][1]
                            backward_total(losses, inputs=[cut] + upper, retain_graph=True)
                        with torch.cuda.graph(seg2, capture_error_mode='thread_local'):
                            torch.autograd.backward(cut, grad_tensors=cut.grad, inputs=lower)
            else:
                with torch.cuda.graph(grads_graph, capture_error_mode='thread_local'):
                    losses, dcnt = self._grads(batch, hidden)
            with torch.cuda.graph(update_graph, capture_error_mode='thread_local'):
                self._static_out = self._update(losses, dcnt)
        finally:
            self.reducer.enabled = True
            self.reducer.reset()
        self._graph, self._graph_update, self._graph_seg2 = grads_graph, update_graph, seg2

    # -- data parallel: two backward segments ------------------------------------------------------
    @contextlib.contextmanager
    def _cut_hook(self):
        """Inside: the step's forward records the segment cut in self._cut -- the fused conv chain's input (a
        forward pre-hook on it) or the tensor between a split torus tower's two parts (nn._CUT_FN)."""
        from . import nn as hnn
        mod = self._cut_module()
        handle = mod.register_forward_pre_hook(self._grab_cut) if mod is not None else None
        prev = hnn._CUT_FN
        if mod is None:
            hnn._CUT_FN = self._grab_cut_tensor
        try:
            yield
        finally:
            if handle is not None:
                handle.remove()
            hnn._CUT_FN = prev
            self._cut = None

    def _has_cut_site(self):
        if self._cut_module() is not None:
            return True
        return any(getattr(m, 'tower_split', None) for m in self.net.modules())

    def _grab_cut_tensor(self, t):
        cut = t.view_as(t)
        self._cut = cut
        return cut

    def _cut_module(self):
        """The fused conv chain (nn._ChainHeads / nn._ConvBNChain): the backward is cut at its input,
        the upper segment (loss, heads, chain) holds nearly all of the step's backward, the lower one
        the layers in front of the chain (the stem).  None: the step stays one backward graph."""
        from .nn import _ChainHeads, _ConvBNChain
        gm = getattr(self.net, '_hrl_graph', None)   # fuse_bn_relu's rewritten forward holds the chain
        if gm is None:
            return None
        for node in gm.graph.nodes:                  # the first one the forward CALLS (a chain merged into
            if node.op == 'call_module':             # _ChainHeads stays registered but is not called)
                m = gm.get_submodule(node.target)
                if isinstance(m, (_ChainHeads, _ConvBNChain)):
                    return m
        return None

    def _grab_cut(self, _module, args):
        """The chain gets a view of its input, and that view is the cut: for a non-leaf `inputs=` tensor
        the autograd engine still runs the tensor's own grad_fn in the first segment, which must not be
        the stem's HIP Function (its backward writes the stem's weight gradient in place; the second
        segment would then add it again)."""
        cut = args[0].view_as(args[0])
        self._cut = cut
        return (cut,) + tuple(args[1:])

    def _try_plan_segments(self, batch):
        """Eager dry run (forward + loss) that finds the segment cut and splits the parameters; leaves
        self.segments None when the net has no fused chain or its parameters do not split cleanly."""
        if not self._has_cut_site():
            self.segment_error = 'no fused conv chain or split torus tower in the net'
            return
        try:
            with self._cut_hook(), direct_grads():
                outputs = forward_prediction(self.net, None, batch, self.args)
                losses, _ = self.loss_fn(outputs, batch, self.args)
                self._plan_segments(losses['total'])
        except RuntimeError as e:
            self.segments = None
            self.segment_error = str(e)
            split_torus_tower(self.net, False)   # no segmented capture: the tower runs as one Function again

    def _plan_flush_segments(self):
        """Recurrent net, data parallel: segment 1 = the live parameters completed by the backward and the first
        flush phase, segment 2 = the recurrent cells' weights (late records, nn.DeferredGrads.flush(phase=2)), as
        flat-buffer ranges.  None when the unroll records nothing late."""
        late = [p for p, l in zip(self.params, self.live) if l and id(p) in self._late_ids]
        early = [p for p, l in zip(self.params, self.live) if l and id(p) not in self._late_ids]
        if not late or not early:
            self.segments = None
            self.segment_error = 'no late (recurrent-cell) weight records in the unroll'
            return
        self.segments = [(self._ranges(early), early), (self._ranges(late), late)]

    def _ranges(self, ps):
        index = {id(p): i for i, p in enumerate(self.params)}
        out = []
        for off, n in sorted(self.grads.slices[index[id(p)]] for p in ps):
            if out and out[-1][1] == off:
                out[-1][1] = off + n
            else:
                out.append([off, off + n])
        return [tuple(r) for r in out]

    def _plan_segments(self, loss):
        """Split the live parameters at the cut tensor by walking the autograd graph: `upper` are reached
        from the loss without passing the cut's node, `lower` from the cut.  Both sets disjoint and each a
        few contiguous ranges of the flat buffer, one bucket per segment (self.segments)."""
        cut = self._cut
        if cut is None or not cut.requires_grad or cut.grad_fn is None:
            raise RuntimeError('segmented capture: the chain input was not seen or does not require grad')

        def reach(root, stop):
            seen, params, todo = set(), set(), [root]
            while todo:
                fn = todo.pop()
                if fn is None or fn in seen or fn is stop:
                    continue
                seen.add(fn)
                var = getattr(fn, 'variable', None)
                if var is not None:
                    params.add(id(var))
                todo.extend(f for f, _ in fn.next_functions)
            return params
        up = reach(loss.grad_fn, cut.grad_fn)
        low = reach(cut.grad_fn, None)
        live = self.live or [True] * len(self.params)
        upper = [p for p, l in zip(self.params, live) if l and id(p) in up]
        lower = [p for p, l in zip(self.params, live) if l and id(p) in low]
        if set(map(id, upper)) & set(map(id, lower)) or len(upper) + len(lower) != sum(live):
            raise RuntimeError('segmented capture: parameters shared across the cut')
        self.segments = [(self._ranges(upper), upper), (self._ranges(lower), lower)]
        return cut, upper, lower

    def load_batch(self, batch):
        """Copy a new batch into the captured graph's static input tensors."""
        for k, v in batch.items():
            dst = self._static[k]
            if isinstance(v, dict):
                for kk, vv in v.items():
                    dst[kk].copy_(vv, non_blocking=True)
            else:
                dst.copy_(v, non_blocking=True)

    def pop_stats(self):
        """Sum of the per-step losses since the last call (one host sync), as a dict."""
        if self.stats is None or self.batches == 0:
            return {}, 0
        vals = self.stats
        if self.reducer is not None:
            vals = hdist.all_reduce_sum_([vals.clone()], self.reducer.group)[0]
        vals = vals.tolist()
        res = dict(zip(self.stats_keys, vals))
        n = self.batches
        if self._tail_stats:
            self.stats.zero_()    # the tail (a captured graph) keeps accumulating into this tensor
            self.batches = 0
        else:
            self.stats = None
        return res, n


class Trainer:
    """Reference-API trainer (train.py:312-414) driving LearnerStep on one GPU rank.

    ``batcher`` is any object with ``batch()`` returning a make_batch-layout
    dict (host or device tensors); ``model`` is the env's network.
    """

    def __init__(self, args, model, batcher, device=None, graph=False, world_size=1, group=None, loss_fn=None):
        self.args = args
        self.model = model
        self.batcher = batcher
        self.device = device or torch.device('cuda', torch.cuda.current_device())
        self.default_lr = DEFAULT_LR
        # train.py:318: the EMA starts at the global batch's cell count (args['batch_size'] is per rank)
        self.data_cnt_ema = args['batch_size'] * world_size * args['forward_steps']
        self.steps = 0
        self.update_flag = False
        self.shutdown_flag = False
        self.learner = LearnerStep(model, args, self.device, lr=self.default_lr * self.data_cnt_ema,
                                   graph=graph, reduce_group=group, world_size=world_size, loss_fn=loss_fn)

    def _to_device(self, batch):
        return map_r(batch, lambda x: x.to(self.device, non_blocking=True) if x is not None else None)

    def train(self, max_steps=None):
        """One epoch: step until update_flag / shutdown (or max_steps); returns a CPU model copy."""
        self.model.train()
        n = 0
        while (n == 0 or not (self.update_flag or self.shutdown_flag)) and (max_steps is None or n < max_steps):
            batch = self._to_device(self.batcher.batch())
            B, P = batch['value'].size(0), batch['value'].size(2)
            hidden = self.model.init_hidden([B, P]) if hasattr(self.model, 'init_hidden') else None
            if hidden is not None:
                hidden = self._to_device(hidden)
            self.learner.step(batch, hidden)
            n += 1
            self.steps += 1
        sums, batch_cnt = self.learner.pop_stats()
        data_cnt = sums.pop('dcnt', 0.0)
        sums.pop('grad_norm', None)
        print('loss = %s' % ' '.join('%s:%.3f' % (k, v / max(data_cnt, 1e-9)) for k, v in sums.items()))
        self.data_cnt_ema = self.data_cnt_ema * 0.8 + data_cnt / (1e-2 + batch_cnt) * 0.2
        self.lr = self.default_lr * self.data_cnt_ema / (1 + self.steps * 1e-5)
        self.learner.set_lr(self.lr)
        model = copy.deepcopy(self.model).cpu()
        model.eval()
        return model


def clip_grad_norm_reference(params, max_norm=4.0):
    """The reference's clip (train.py:384), kept for tests that compare both forms."""
    return nn.utils.clip_grad_norm_(params, max_norm)
