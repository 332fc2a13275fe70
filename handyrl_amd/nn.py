"""HIP-backed layers for the learner's env networks, and the pass that installs them.

Env networks stay exactly as their plugins define them (Environment.net(),
handyrl/environment.py); ``accelerate(model)`` swaps, in place, the modules
whose training-mode kernels are the learner step's bottleneck on MI355X for
subclasses with identical parameters, buffers and state_dict keys:

* ``nn.BatchNorm2d`` -> ``BatchNorm2d`` (csrc/hrl_bn.hip): training-mode
  forward/backward as coalesced streaming passes with fp64 statistics.  In
  eval mode, on CPU tensors, or for shapes the kernels do not take (rows
  wider than 3072 floats, or than 1024 when not a multiple of 4) the module
  is the plain torch layer.
* ``nn.Conv2d`` (stride 1, 'same' zero padding, no dilation/groups) ->
  ``BoardConv2d`` on boards of at most ``BOARD_MAX_CELLS`` cells: on a tiny
  board a convolution IS a dense matrix, Y[N, Cout*HW] = X[N, Cin*HW] @ W_board
  with W_board[(ci,p),(co,q)] = W[co, ci, p-q+k//2] (zero off the board), so
  the layer runs as one fp32 hipBLASLt GEMM on the NCHW rows (MFMA f32, exact
  fp32 products) with the bias in the epilogue, instead of an implicit-GEMM
  convolution wrapped in NCHW<->NHWC transposes.  The backward is the two
  GEMMs of that matmul plus a gather-sum folding dW_board back onto W.
* ``nn.Linear`` -> ``Linear``: same forward; over >= 4096 rows the weight
  gradient runs as a chunked batched GEMM (see ``_xt_dy``).

The HIP path is taken whenever the input is a CUDA tensor in training mode;
if libhrl.so is missing that raises (no silent fallback).
"""

import ctypes
import operator

import os

import torch
import torch.fx
import torch.nn as nn
import torch.nn.functional as F

from . import _native

__all__ = ['BatchNorm2d', 'BoardConv2d', 'Linear', 'accelerate', 'batch_norm_train', 'fuse_bn_relu', 'unfuse']

_MAX_ROW = 3072        # float4 path (row width a multiple of 4)
_MAX_ROW_SCALAR = 1024  # scalar path


class DeferredGrads:
    """Weight gradients of a recurrent unroll, batched over time.

    A recurrent learner step runs the net T times (train.py:155-174), so every
    weight is used T (or, inside GeisterNet's DRC, 3T) times and autograd
    computes one weight-gradient convolution per use and adds them up.  Inside
    ``with deferred_weight_grads() as d:`` the HIP layers return no weight
    gradient; they record (input, output gradient) instead, and ``d.flush()``
    -- after backward -- computes each weight's gradient with ONE batched call
    over all recorded uses and adds it into ``.grad``.  Same sum, different
    fp32 association.  Only LearnerStep enables it (it calls flush).
    """

    def __init__(self):
        self.conv = {}     # (param, bias param, in slice, padding) -> [(x, dy)]
        self.late_params = set()   # ids of the weights with a late record (flushed in phase 2)
        self.affine = {}   # (weight, bias) -> [(dweight, dbias)]
        self.adjoint = {}  # (param, in slice) -> the input-gradient conv's packed weights, packed once per step

    def adjoint_pack(self, w, ci0, cin, split=False):
        """gboard_pack_adjoint(w, ci0, cin) (split: gboard_pack_adjoint_split), once per step: the weights do not
        change inside a step, and the unroll calls a cell's input gradient 3T times."""
        key = (id(w), ci0, cin, split)
        pk = self.adjoint.get(key)
        if pk is None:
            fn = gboard_pack_adjoint_split if split else gboard_pack_adjoint
            pk = self.adjoint[key] = fn(w.detach(), ci0, cin)
        return pk

    def add_conv(self, key, x, dy, late=False):
        """late: the record belongs to the unroll's innermost cells (GeisterNet's DRC), whose weight gradients a
        data-parallel step flushes last (flush(phase=2)) so the other buckets' all-reduce runs meanwhile."""
        self.conv.setdefault(key, []).append((x, dy))
        if late:
            self.late_params.add(id(key[0]))

    def add_affine(self, key, dw, db):
        self.affine.setdefault(key, []).append((dw, db))

    def late_ids(self):
        """ids of the parameters flush(phase=2) completes: the weights with a late record and the biases recorded
        with them."""
        return set(self.late_params) | {id(k[1]) for k in self.conv if id(k[0]) in self.late_params and
                                        k[1] is not None}

    @torch.no_grad()
    def flush(self, phase=None):
        """Accumulate the deferred gradients into .grad; returns the parameters that got one, each once
        (a ConvLSTM h-conv weight is recorded once per input slice).  phase 1: every weight without a late record
        (and the affine records); phase 2: the rest; None: both."""
        touched = {}
        keys = [k for k in self.conv if phase is None or ((id(k[0]) in self.late_params) == (phase == 2))]
        for key in keys:
            (w, b, sl, pad), rec = key, self.conv.pop(key)
            wv = w if sl is None else w[:, sl[0]:sl[1]]
            if GBOARD_WGRAD and _gboard_wgrad_ok(rec, wv, pad):
                # the 6x6 board: games as the MFMA K over every recorded use, no concatenation (hrl_gboard_wgrad)
                gboard_wgrad(rec, w, b, sl)
                touched[id(w)] = w
                if b is not None:
                    touched[id(b)] = b
                continue
            if b is None and _pointwise_board_ok(rec, wv, pad):
                # a 1x1 conv on the 6x6 board: one HBM pass over each recorded input (hrl_gboard_pointwise_wgrad)
                gboard_pointwise_wgrad(rec, w, sl)
                touched[id(w)] = w
                continue
            X = torch.cat([r[0] for r in rec]) if len(rec) > 1 else rec[0][0]
            DY = torch.cat([r[1] for r in rec]) if len(rec) > 1 else rec[0][1]
            if _pointwise_ok(X, wv, pad):
                # a 1x1 conv: dW[o, c] = sum over games and cells of dy[n, o, q] x[n, c, q], one GEMM
                N, C, O = X.shape[0], X.shape[1], DY.shape[1]
                dw = torch.tensordot(DY.reshape(N, O, -1), X.reshape(N, C, -1), dims=([0, 2], [0, 2]))
                _add_grad(w, dw.view(O, C, 1, 1), sl)
                touched[id(w)] = w
                if b is not None:
                    _add_grad(b, DY.sum((0, 2, 3)), None)
                    touched[id(b)] = b
                continue
            _, dw, db = torch.ops.aten.convolution_backward(
                DY, X, wv, [wv.shape[0]] if b is not None else None, [1, 1], list(pad), [1, 1], False, [0, 0], 1,
                [False, True, b is not None])
            _add_grad(w, dw, sl)
            touched[id(w)] = w
            if b is not None:
                _add_grad(b, db, None)
                touched[id(b)] = b
        if phase != 2:
            for (w, b), rec in self.affine.items():
                if w is not None:
                    _add_grad(w, rec[0][0] if len(rec) == 1 else torch.stack([r[0] for r in rec]).sum(0), None)
                    touched[id(w)] = w
                if b is not None:
                    _add_grad(b, rec[0][1] if len(rec) == 1 else torch.stack([r[1] for r in rec]).sum(0), None)
                    touched[id(b)] = b
            self.affine.clear()
        if phase != 1:
            self.conv.clear()
            self.adjoint.clear()
        return list(touched.values())


# the deferred 3x3 board convs' weight gradient on hrl_gboard_wgrad (games as the MFMA K) instead of
# aten.convolution_backward over the concatenated records
GBOARD_WGRAD = os.environ.get('HRL_GBOARD_WGRAD', '1') == '1'


def _gboard_wgrad_ok(rec, wv, pad):
    """Records hrl_gboard_wgrad covers: 3x3 'same' on the 6x6 board, fp32 CUDA, channel-contiguous games."""
    if tuple(pad) != (1, 1) or tuple(wv.shape[2:]) != (3, 3) or wv.dtype != torch.float32 or not wv.is_cuda:
        return False
    cout, cin = wv.shape[0], wv.shape[1]
    cto, cti = (cout + 31) // 32, (cin + 31) // 32
    if not ((cto == 4 and cti == 1) or (cto <= 2 and cti <= 2)):
        return False
    for x, dy in rec:
        for t, c in ((x, cin), (dy, cout)):
            if not (t.is_cuda and t.dtype == torch.float32 and t.dim() == 4 and tuple(t.shape[1:]) == (c, 6, 6)
                    and t.stride(1) == 36 and t.stride(2) == 6 and t.stride(3) == 1 and t.stride(0) % 2 == 0
                    and t.data_ptr() % 8 == 0 and t.shape[0] > 0):
                return False
    return True


def gboard_wgrad(rec, w, b, sl):
    """Add the weight (and bias) gradient of the recorded (x, dy) uses of conv weight w (input-channel slice sl)
    into w.grad / b.grad with csrc/hrl_gboard.hip's games-as-K kernel, up to 64 records per launch."""
    import ctypes
    lib = _native.load()
    ci0, cin = (0, w.shape[1]) if sl is None else (sl[0], sl[1] - sl[0])
    cout = w.shape[0]
    for p in (w, b):
        if p is not None and p.grad is None:
            p.grad = torch.zeros_like(p)
    assert w.grad.is_contiguous() and (b is None or b.grad.is_contiguous())
    stream = _native.stream_of(w.device)
    for k in range(0, len(rec), 64):
        chunk = rec[k:k + 64]
        n = len(chunk)
        xs = (ctypes.c_void_p * n)(*[r[0].data_ptr() for r in chunk])
        dys = (ctypes.c_void_p * n)(*[r[1].data_ptr() for r in chunk])
        xst = (ctypes.c_int64 * n)(*[r[0].stride(0) for r in chunk])
        dyst = (ctypes.c_int64 * n)(*[r[1].stride(0) for r in chunk])
        ns = (ctypes.c_int64 * n)(*[r[0].shape[0] for r in chunk])
        games = sum((r[0].shape[0] + 15) // 16 * 16 for r in chunk)   # one partial per 16-game tile of a record
        nbytes = lib.hrl_gboard_wgrad_workspace_bytes(cout, cin, games)
        ws = torch.empty(nbytes, dtype=torch.uint8, device=w.device)
        _native.check(lib.hrl_gboard_wgrad(
            ctypes.cast(xs, ctypes.c_void_p), ctypes.cast(xst, ctypes.c_void_p), ctypes.cast(dys, ctypes.c_void_p),
            ctypes.cast(dyst, ctypes.c_void_p), ctypes.cast(ns, ctypes.c_void_p), n, cout, cin,
            _native.ptr(w.grad), w.shape[1], ci0, None if b is None else _native.ptr(b.grad), _native.ptr(ws),
            nbytes, stream), 'hrl_gboard_wgrad')


def _pointwise_board_ok(rec, wv, pad):
    """Records hrl_gboard_pointwise_wgrad covers: a 1x1 conv (O <= 8 outputs, C <= 256 inputs) on the 6x6 board,
    fp32 CUDA, float4-aligned channel-contiguous games."""
    if (tuple(pad) != (0, 0) or tuple(wv.shape[2:]) != (1, 1) or wv.dtype != torch.float32 or not wv.is_cuda
            or wv.shape[0] > 8 or wv.shape[1] > 256):
        return False
    return all(gboard_ok(x) and gboard_ok(dy) and x.shape[1] == wv.shape[1] and dy.shape[1] == wv.shape[0]
               and x.shape[0] == dy.shape[0] for x, dy in rec)


def gboard_pointwise_wgrad(rec, w, sl):
    """Add the weight gradient of the recorded (x, dy) uses of 1x1 conv weight w (input-channel slice sl) into
    w.grad (csrc/hrl_gboard.hip, one launch pair per record)."""
    lib = _native.load()
    O = w.shape[0]
    C = w.shape[1] if sl is None else sl[1] - sl[0]
    if w.grad is None:
        w.grad = torch.zeros_like(w)
    g = w.grad if sl is None else w.grad[:, sl[0]:sl[1]]
    dst = g if g.is_contiguous() else torch.zeros(O, C, 1, 1, device=w.device)
    stream = _native.stream_of(w.device)
    for x, dy in rec:
        N = x.shape[0]
        nbytes = lib.hrl_gboard_pointwise_wgrad_workspace_bytes(C, O, N)
        ws = torch.empty(nbytes, dtype=torch.uint8, device=w.device)
        _native.check(lib.hrl_gboard_pointwise_wgrad(
            _native.ptr(x), x.stride(0), _native.ptr(dy), dy.stride(0), N, C, O, _native.ptr(dst), _native.ptr(ws),
            nbytes, stream), 'hrl_gboard_pointwise_wgrad')
    if dst is not g:
        g.add_(dst)


def _add_grad(p, g, sl):
    if p.grad is None:
        p.grad = torch.zeros_like(p)
    if sl is None:
        p.grad.add_(g)
    else:
        p.grad[:, sl[0]:sl[1]].add_(g)


_DEFER = None


class deferred_weight_grads:
    """Context manager: defer the HIP layers' weight gradients into a DeferredGrads (see there)."""

    def __enter__(self):
        global _DEFER
        self.prev = _DEFER
        _DEFER = DeferredGrads()
        return _DEFER

    def __exit__(self, *exc):
        global _DEFER
        _DEFER = self.prev
        return False


_DIRECT = None


class direct_grads:
    """Context manager (LearnerStep, feed-forward steps): the HIP Functions write a parameter's
    gradient straight into ``p.grad`` -- a view of the learner's flat gradient buffer, zeroed at the
    start of the step -- instead of returning it to autograd, whose AccumulateGrad would launch one
    add kernel per parameter.  Only the first gradient of a parameter in the step is written that
    way; any further use of the same parameter returns its gradient as usual, so sums stay right."""

    def __enter__(self):
        global _DIRECT
        self.prev = _DIRECT
        _DIRECT = set()
        return self

    def __exit__(self, *exc):
        global _DIRECT
        _DIRECT = self.prev
        return False


_FOLDS = None


class deferred_folds:
    """Context manager (LearnerStep on one GPU, with the step tail): a HIP backward Function whose parameter
    gradients are written in place (direct_grads) leaves them as its per-workgroup partial rows instead of
    launching its reduce kernel, and registers the fold here; LearnerStep folds every registered partial into the
    flat gradient buffer in the step tail's first launch (hrl_grad_fold_norm, together with the clip's norm).  The
    fused chains' BatchNorm batch counters are collected here too, for the same launch."""

    def __init__(self, enabled=True):
        self.enabled = enabled

    def __enter__(self):
        global _FOLDS
        self.prev = _FOLDS
        self.folds = []      # (partial rows (float32 tensor), stride, col0, nparts, dst gradient view, count, mode)
        self.counters = []   # int64 num_batches_tracked tensors
        self.increments = []  # and what each advances by
        self.keep = []       # workspaces read by the folds: referenced until the fold launch is enqueued
        if self.enabled:
            _FOLDS = self
        return self

    def __exit__(self, *exc):
        global _FOLDS
        if self.enabled:
            _FOLDS = self.prev
        return False

    # the step tail's launch tables (csrc/hrl_optim.hip kMaxFolds / kMaxCounters): a Function that finds no room
    # left runs its own reduce launch and a counter its own add, so a deep net degrades to launches, never fails
    MAX_FOLDS = 16
    MAX_COUNTERS = 8

    def has_room(self, folds=0, counters=0):
        return (len(self.folds) + folds <= self.MAX_FOLDS and len(self.counters) + counters <= self.MAX_COUNTERS)

    def add(self, part, stride, col0, nparts, dst, count, mode=0):
        assert len(self.folds) < self.MAX_FOLDS, 'deferred folds: table full (check has_room first)'
        self.folds.append((part, stride, col0, nparts, dst, count, mode))

    def add_counter(self, counter, inc=1):
        assert len(self.counters) < self.MAX_COUNTERS, 'deferred folds: counter table full (check has_room first)'
        self.counters.append(counter)
        self.increments.append(int(inc))


def _defer_folds(bufs, nfolds=None):
    """The deferred-folds context when the gradients in `bufs` (_grad_buffer results) may stay as partials:
    one is active, every buffer is a direct (in-place) one and its table has room for the `nfolds` folds the
    caller registers (default: one per buffer); else None (the caller folds with its own launch)."""
    if _FOLDS is None or not all(b[1] for b in bufs if b[0] is not None):
        return None
    n = sum(1 for b in bufs if b[0] is not None) if nfolds is None else nfolds
    return _FOLDS if _FOLDS.has_room(folds=n) else None


def _defer_counters(counters, inc=1):
    """Hand BatchNorm batch counters to the active deferred-folds context (the step tail advances them); False
    when there is none or its counter table is full (the caller advances them itself)."""
    if _FOLDS is None or not _FOLDS.has_room(counters=len(counters)):
        return False
    for c in counters:
        _FOLDS.add_counter(c, inc)
    return True


def _heads_backward_deferred(lib, df, bufs, N, ws, call):
    """hrl_heads_backward with the six weight-gradient pointers NULL (partials left in ws), then the folds of its
    270-float partial rows [dW1 policy (64) | dW1 value (32) | db1 (3) | dWp (162) | dWv (9)] registered."""
    call(None, None, None, None, None, None)
    dw1p, db1p, dw1v, db1v, dwp, dwv = (b[0] for b in bufs)
    part = ws.view(torch.float32)
    nparts = lib.hrl_heads_bn_parts(N)
    for dst, col0, count in ((dw1p, 0, 64), (dw1v, 64, 32), (db1p, 96, 2), (db1v, 98, 1), (dwp, 99, 162),
                             (dwv, 261, 9)):
        df.add(part, 270, col0, nparts, dst, count)
    df.keep.append(ws)


def _grad_buffer(p):
    """(buffer, direct) for p's gradient: p.grad itself when it may be written in place (see
    direct_grads), else a fresh tensor to return to autograd."""
    if p is None:
        return None, False
    g = p.grad
    if (_DIRECT is not None and p.requires_grad and g is not None and id(p) not in _DIRECT
            and g.is_contiguous() and g.dtype == p.dtype and g.shape == p.shape):
        _DIRECT.add(id(p))
        return g, True
    return torch.empty_like(p), False


def _ret(buf_direct):
    """What backward returns for a gradient from _grad_buffer: None when it was written in place."""
    buf, direct = buf_direct
    return None if direct else buf


def board_conv_ok(x, w, ci0, pad):
    """Shapes hrl_board_conv_forward covers: 'same' 3x3 zero padding, 32 input channels (a slice [ci0, ci0+32) of
    w's), Cout a multiple of 32, boards of 4..80 cells, fp32 CUDA."""
    return (x.is_cuda and x.dtype == torch.float32 and w.dtype == torch.float32 and x.dim() == 4
            and x.shape[0] > 0 and x.shape[1] == 32 and w.dim() == 4 and tuple(w.shape[2:]) == (3, 3)
            and tuple(pad) == (1, 1) and w.shape[0] % 32 == 0 and 0 <= ci0 and ci0 + 32 <= w.shape[1]
            and 4 <= x.shape[2] * x.shape[3] <= 80)


def board_conv_pack(w, ci0=0):
    """w[:, ci0:ci0+32] packed for board_conv_forward (a recurrent unroll packs each weight once per forward)."""
    lib = _native.load()
    nbytes = lib.hrl_board_conv_workspace_bytes(w.shape[0])
    wpk = torch.empty(nbytes, dtype=torch.uint8, device=w.device)
    _native.check(lib.hrl_board_conv_pack(_native.ptr(w.contiguous()), w.shape[1], ci0, w.shape[0], _native.ptr(wpk),
                                          nbytes, _native.stream_of(w.device)), 'hrl_board_conv_pack')
    return wpk


def board_conv_forward(x, w, b, ci0=0, packed=None):
    """F.conv2d(x, w[:, ci0:ci0+32], b, padding=1) on csrc/hrl_torus.hip's MFMA path (zero padding); forward
    only, no autograd (board_conv_ok must hold).  ``packed``: board_conv_pack(w, ci0) made for this forward."""
    x = x.contiguous()
    N, _, H, W = x.shape
    Cout = w.shape[0]
    wpk = board_conv_pack(w, ci0) if packed is None else packed
    y = torch.empty(N, Cout, H, W, device=x.device, dtype=x.dtype)
    _native.check(_native.load().hrl_board_conv_forward_packed(
        _native.ptr(x), N, 32, H, W, _native.ptr(wpk), Cout, _native.ptr(b.contiguous()) if b is not None else None,
        _native.ptr(y), _native.stream_of(x.device)), 'hrl_board_conv_forward_packed')
    return y


# bench.py's in-step timing of the dominant kernel: a list that collects (start, end) HIP events recorded on the
# launch stream around every chain block backward launch of an eager step (None: off; never inside a capture)
BLOCK_TIMING = None


def _block_timing_start():
    if BLOCK_TIMING is None or torch.cuda.is_current_stream_capturing():
        return None
    # an eager step is host-bound: without work queued ahead, the start event fires while the host is still
    # marshalling the launch and the interval measures that wait too.  A ~50 us spin keeps the stream busy until
    # the launch is queued behind the event, so the interval is the kernel's own duration (as rocprofv3 sees it).
    torch.cuda._sleep(100000)
    ev = torch.cuda.Event(enable_timing=True)
    ev.record()
    return ev


def _block_timing_end(ev):
    if ev is not None:
        end = torch.cuda.Event(enable_timing=True)
        end.record()
        BLOCK_TIMING.append((ev, end))


def gboard_ok(x, groups=1, x2=None):
    """Inputs hrl_gboard_forward covers: fp32 CUDA games on the 6x6 board, float4-aligned storage."""
    ts = [x] if x2 is None else [x, x2]
    return all(t.is_cuda and t.dtype == torch.float32 and t.dim() == 4 and tuple(t.shape[2:]) == (6, 6)
               and t.stride(1) == 36 and t.stride(2) == 6 and t.stride(3) == 1 and t.stride(0) % 4 == 0
               and t.data_ptr() % 16 == 0 for t in ts) and x.shape[0] > 0


def _pointwise_ok(x, wv, pad):
    """A 1x1 conv (no padding) the deferred path runs as plain GEMMs (forward, input gradient, batched weight
    gradient) instead of the vendor convolution."""
    return (wv.dim() == 4 and tuple(wv.shape[2:]) == (1, 1) and tuple(pad) == (0, 0) and x.dim() == 4
            and x.is_cuda and x.is_contiguous() and x.dtype == torch.float32 and wv.dtype == torch.float32)


def gboard_conv_ok(x, w, cin_g, pad):
    """A 'same' 3x3 conv hrl_gboard_forward covers: x (N, cin_g, 6, 6) fp32 CUDA (float4-aligned games), at most 64
    input channels, any Cout."""
    return (w.dim() == 4 and tuple(w.shape[2:]) == (3, 3) and tuple(pad) == (1, 1) and w.dtype == torch.float32
            and x.dim() == 4 and x.shape[1] == cin_g <= 64 and gboard_ok(x))


def gboard_pack(w, cin_g=None, ci0=0, out=None):
    """Input channels [ci0, ci0 + cin_g) of the 3x3 weight w (Cout, Cin_total, 3, 3) as hrl_gboard's split
    fragments (written into ``out`` when given: a graph captured over the packed buffer sees the refresh)."""
    lib = _native.load()
    Cout, cin_total = w.shape[0], w.shape[1]
    cin_g = cin_total - ci0 if cin_g is None else cin_g
    nbytes = lib.hrl_gboard_pack_bytes(Cout, cin_g)
    if nbytes < 0:
        raise ValueError('hrl_gboard_pack: unsupported weight %s' % (tuple(w.shape),))
    wpk = torch.empty(nbytes, dtype=torch.uint8, device=w.device) if out is None else out
    _native.check(lib.hrl_gboard_pack(_native.ptr(w.contiguous()), Cout, cin_g, cin_total, ci0, _native.ptr(wpk),
                                      wpk.numel(), _native.stream_of(w.device)), 'hrl_gboard_pack')
    return wpk


# the deferred convs' input gradient on hrl_gboard (the adjoint conv, K up to 4 x 32) instead of
# aten.convolution_backward; off until measured on the GPU
GBOARD_ADJOINT = os.environ.get('HRL_GBOARD_ADJOINT', '0') == '1'


def gboard_pack_adjoint(w, ci0, cin):
    """The input-gradient conv of input channels [ci0, ci0 + cin) of the 3x3 weight w (Cout, Cin_total, 3, 3),
    packed for gboard_conv (cin outputs from Cout inputs)."""
    lib = _native.load()
    nbytes = lib.hrl_gboard_pack_bytes(cin, w.shape[0])
    if nbytes < 0:
        raise ValueError('hrl_gboard_pack_adjoint: unsupported weight %s' % (tuple(w.shape),))
    wpk = torch.empty(nbytes, dtype=torch.uint8, device=w.device)
    _native.check(lib.hrl_gboard_pack_adjoint(_native.ptr(w.contiguous()), w.shape[0], w.shape[1], ci0, cin,
                                              _native.ptr(wpk), nbytes, _native.stream_of(w.device)),
                  'hrl_gboard_pack_adjoint')
    return wpk


def gboard_pack_adjoint_split(w, ci0, cin):
    """The input-gradient conv of input channels [ci0, ci0 + cin) of the 3x3 weight w (Cout, Cin_total, 3, 3) split
    over its K = Cout in 32-channel pieces: packed for gboard_conv(dy, ., S * cin, 32, groups=S), S = Cout / 32, whose
    group s is the adjoint conv of dy's channels [32s, 32s + 32) -- the S partial input gradients, summed after."""
    Cf = w.shape[0]
    S = Cf // 32
    adj = w[:, ci0:ci0 + cin].flip(2, 3).transpose(0, 1)                     # (cin, Cf, 3, 3): W'[co'][ci'][tap]
    w_grp = adj.reshape(cin, S, 32, 3, 3).transpose(0, 1).reshape(S * cin, 32, 3, 3).contiguous()
    return gboard_pack(w_grp)


# the deferred 3x3 convs' input gradient with K = 64..128 (the ConvLSTM h halves' 128 -> 32) on hrl_gboard as
# K-split partial convs (S groups of 32, one launch with S times the workgroups) + a sum, instead of
# aten.convolution_backward
GBOARD_ADJOINT_SPLIT = os.environ.get('HRL_GBOARD_ADJOINT_SPLIT', '1') == '1'


def gboard_adjoint_split(dy, w, ci0, cin, rec):
    """dx of the deferred conv (input channels [ci0, ci0 + cin) of w) for output gradient dy on hrl_gboard."""
    N, Cf = dy.shape[0], dy.shape[1]
    S = Cf // 32
    part = gboard_conv(dy, rec.adjoint_pack(w, ci0, cin, split=True), S * cin, 32, groups=S)
    return part.view(N, S, cin, 6, 6).sum(1)


def _check_gboard_packed(packed, Cout, cin_g):
    """hrl_gboard_forward reads hrl_gboard_pack_bytes(Cout, cin_g) bytes of split weights and cannot check them
    itself: a buffer packed for another shape (or for the torus board conv) is refused here."""
    need = _native.load().hrl_gboard_pack_bytes(Cout, cin_g)
    if need < 0 or packed.dtype != torch.uint8 or packed.numel() < need:
        raise ValueError('hrl_gboard: packed weights of %d bytes, (Cout %d, Cin_g %d) needs %d'
                         % (packed.numel() * packed.element_size(), Cout, cin_g, need))


def gboard_conv(x, packed, Cout, cin_g, groups=1, x2=None, bias=None, alpha=None, beta=None, relu=False, out=None):
    """F.conv2d(x, W, bias, padding=1, groups=groups) on the 6x6 board (csrc/hrl_gboard.hip, forward only, no
    autograd), W packed by gboard_pack; optional BatchNorm-apply (y*alpha + beta) and ReLU epilogue.  x may be
    a channel slice of a wider tensor; x2: channels 32.. of a two-source input (x then holds channels 0..31)."""
    N = x.shape[0]
    _check_gboard_packed(packed, Cout, cin_g)
    y = torch.empty(N, Cout, 6, 6, device=x.device, dtype=torch.float32) if out is None else out
    P = _native.ptr
    _native.check(_native.load().hrl_gboard_forward(
        P(x), x.stride(0), None if x2 is None else P(x2), 0 if x2 is None else x2.stride(0), N, cin_g, groups,
        P(packed), packed.numel() * packed.element_size(), Cout, None if bias is None else P(bias),
        None if alpha is None else P(alpha),
        None if beta is None else P(beta), int(relu), P(y), y.stride(0), _native.stream_of(x.device)),
        'hrl_gboard_forward')
    return y


def gboard_pointwise(x, w, x2=None, alpha=None, beta=None, relu=False):
    """1x1 conv (no bias) of x (and then x2's channels) on the 6x6 board with weight w (O, C, 1, 1), optional
    BatchNorm apply + ReLU (csrc/hrl_gboard.hip, forward only): F.conv2d(cat([x, x2]), w) without the cat."""
    N, C1 = x.shape[0], x.shape[1]
    C2 = 0 if x2 is None else x2.shape[1]
    O = w.shape[0]
    y = torch.empty(N, O, 6, 6, device=x.device, dtype=torch.float32)
    P = _native.ptr
    _native.check(_native.load().hrl_gboard_pointwise(
        P(x), x.stride(0), C1, None if x2 is None else P(x2), 0 if x2 is None else x2.stride(0), C2, N,
        P(w.contiguous()), O, None if alpha is None else P(alpha), None if beta is None else P(beta), int(relu),
        P(y), y.stride(0), _native.stream_of(x.device)), 'hrl_gboard_pointwise')
    return y


class _DeferredConv(torch.autograd.Function):
    """conv2d (stride 1, 'same') whose weight/bias gradient is deferred to DeferredGrads.flush().

    ``sl`` selects input channels [sl[0], sl[1]) of the weight (a ConvLSTM cell's h or x half)."""

    @staticmethod
    def forward(ctx, x, w, b, sl, pad, rec, packed=None):
        ctx.set_materialize_grads(False)
        wv = w if sl is None else w[:, sl[0]:sl[1]]
        ci0 = 0 if sl is None else sl[0]
        cin_g = wv.shape[1]
        if gboard_conv_ok(x, w, cin_g, pad):   # the 6x6 board: games as MFMA rows (csrc/hrl_gboard.hip)
            if packed is not None and packed.numel() != _native.load().hrl_gboard_pack_bytes(w.shape[0], cin_g):
                packed = None   # packed for the torus board conv or another shape: repack for this kernel
            wpk = gboard_pack(w.detach(), cin_g, ci0) if packed is None else packed
            y = gboard_conv(x, wpk, w.shape[0], cin_g, bias=None if b is None else b.detach())
        elif (b is None and _pointwise_ok(x, wv, pad) and wv.shape[0] in (1, 2, 4, 8) and x.shape[1] <= 128
              and gboard_ok(x)):
            # a 1x1 conv with a few outputs on the 6x6 board (the heads): one HIP pass over x (hrl_gboard_pointwise)
            y = gboard_pointwise(x, wv.detach())
        elif _pointwise_ok(x, wv, pad):          # a 1x1 conv: per game one (Cout x Cin) . (Cin x cells) GEMM
            N, C = x.shape[0], x.shape[1]
            y = torch.matmul(wv.detach().reshape(wv.shape[0], C), x.reshape(N, C, -1)).view(N, -1, *x.shape[2:])
            if b is not None:
                y = y + b.detach().view(1, -1, 1, 1)
        elif (sl is None or sl[1] - sl[0] == 32) and board_conv_ok(x, w, ci0, pad):
            if packed is not None and packed.numel() != _native.load().hrl_board_conv_workspace_bytes(w.shape[0]):
                packed = None   # packed for hrl_gboard (this input missed its alignment): repack for this kernel
            y = board_conv_forward(x, w.detach(), None if b is None else b.detach(), ci0, packed)
        else:
            y = F.conv2d(x, wv, b, padding=pad)
        ctx.save_for_backward(x, w)
        ctx.meta = (sl, pad, rec, b)
        return y

    @staticmethod
    def backward(ctx, dy):
        if dy is None:
            return None, None, None, None, None, None, None
        x, w = ctx.saved_tensors
        sl, pad, rec, b = ctx.meta
        dy = dy.contiguous()
        wv = w if sl is None else w[:, sl[0]:sl[1]]
        dx = _deferred_conv_dx(dy, x, w, sl, pad, rec) if ctx.needs_input_grad[0] else None
        rec.add_conv((w, b, sl, tuple(pad)), x, dy)
        return dx, None, None, None, None, None, None


def _deferred_conv_dx(dy, x, w, sl, pad, rec):
    """The input gradient of a deferred conv (input-channel slice sl of w) for output gradient dy."""
    wv = w if sl is None else w[:, sl[0]:sl[1]]
    Cf = w.shape[0]
    if (GBOARD_ADJOINT_SPLIT and tuple(pad) == (1, 1) and tuple(w.shape[2:]) == (3, 3) and gboard_ok(dy)
            and Cf % 32 == 0 and 2 <= Cf // 32 <= 8 and wv.shape[1] % 16 == 0 and wv.shape[1] == x.shape[1]
            and dy.shape[1] == Cf):
        return gboard_adjoint_split(dy, w, 0 if sl is None else sl[0], wv.shape[1], rec)
    if ((GBOARD_ADJOINT_SPLIT or GBOARD_ADJOINT) and tuple(pad) == (1, 1) and tuple(w.shape[2:]) == (3, 3)
            and gboard_ok(dy) and Cf <= 32 and wv.shape[1] == x.shape[1] and dy.shape[1] == Cf):
        # a K of one k-step (the move head's 64 -> 8: K = 8): the plain adjoint conv on hrl_gboard
        ci0 = 0 if sl is None else sl[0]
        return gboard_conv(dy, rec.adjoint_pack(w, ci0, wv.shape[1]), wv.shape[1], Cf)
    if (GBOARD_ADJOINT and tuple(pad) == (1, 1) and tuple(w.shape[2:]) == (3, 3) and gboard_ok(dy)
            and (Cf <= 64 or 96 < Cf <= 128) and wv.shape[1] == x.shape[1]):
        # the adjoint conv on hrl_gboard: K = the forward's Cout (up to 4 x 32), Cout = the slice width
        ci0 = 0 if sl is None else sl[0]
        return gboard_conv(dy, rec.adjoint_pack(w, ci0, wv.shape[1]), wv.shape[1], Cf)
    if _pointwise_ok(x, wv, pad):
        N, O = dy.shape[0], dy.shape[1]
        if O == 1:   # one output channel: dx = w[c] * dy, an outer product (the same single products as the GEMM)
            return wv.detach().reshape(1, -1, 1, 1) * dy
        return torch.matmul(wv.detach().reshape(O, -1).t(), dy.reshape(N, O, -1)).view_as(x)
    return torch.ops.aten.convolution_backward(dy, x, wv, None, [1, 1], list(pad), [1, 1], False, [0, 0], 1,
                                               [True, False, False])[0]


class _DRCStep(torch.autograd.Function):
    """The R repeats of a DRC's L ConvLSTM cells at one time step of a deferred-gradient unroll (GeisterNet's
    learner), each repeat in two launches for all L layers: the h halves as ONE grouped hrl_gboard conv over the
    layers' separate states (hrl_gboard_forward_groups) and the gates as one hrl_lstm_gates_forward_grouped (the
    per-layer kernels' float operations, so the states are those of _DeferredConv + lstm_gates bit for bit).

    Backward, per layer whose outputs carry a gradient (GeisterNet: the last one), repeats in reverse: the gate
    backward (hrl_lstm_gates_backward_ex) reads the h input gradient of the repeat after it as the S partials of
    the K-split adjoint conv (gboard_adjoint_split's grouped launch, summed in the gate kernel) and accumulates the
    x half's gradient over the repeats; each repeat records its (h, dz) for the deferred weight gradient.

    apply(meta, *zx, *h, *c) -> (*h', *c'); meta = (ws, h slice of the weights, pad, packed, DeferredGrads, R)."""

    @staticmethod
    def forward(ctx, meta, *args):
        ctx.set_materialize_grads(False)
        ws, sl, pad, packed, rec, R = meta
        L = len(ws)
        zx, hs, cs = args[:L], list(args[L:2 * L]), list(args[2 * L:])
        N, H = hs[0].shape[0], hs[0].shape[1]
        lib = _native.load()
        stream = _native.stream_of(hs[0].device)
        P = _native.ptr
        # a layer whose x half is outside autograd (DRC.x_halves: the layers that reach no output) gets no
        # backward: its gate activations are not stored
        live = [z.requires_grad for z in zx]
        zx_ptrs = _native.ptr_array(zx)
        zx_strides = _native.i64_array([z.stride(0) for z in zx])
        saved = []
        _check_gboard_packed(packed, L * 4 * H, H)
        for _ in range(R):
            zh = torch.empty(N, L * 4 * H, 6, 6, device=hs[0].device)
            _native.check(lib.hrl_gboard_forward_groups(
                _native.ptr_array(hs), _native.i64_array([h.stride(0) for h in hs]), N, H, L, P(packed),
                packed.numel() * packed.element_size(), L * 4 * H, P(zh), zh.stride(0), stream),
                'hrl_gboard_forward_groups')
            h_out = [torch.empty_like(c) for c in cs]
            c_out = [torch.empty_like(c) for c in cs]
            gates = [torch.empty(N, 4 * H, 6, 6, device=zh.device) if lv else None for lv in live]
            _native.check(lib.hrl_lstm_gates_forward_grouped(
                L, P(zh), zh.stride(0), zx_ptrs, zx_strides, _native.ptr_array(cs), N, H, 36,
                _native.ptr_array(h_out), _native.ptr_array(c_out), _native.ptr_array(gates), stream),
                'hrl_lstm_gates_forward_grouped')
            for i in range(L):
                if live[i]:
                    saved += [hs[i], cs[i], c_out[i], gates[i]]
            hs, cs = h_out, c_out
        ctx.save_for_backward(*saved)
        ctx.meta = meta
        ctx.live = live
        return (*hs, *cs)

    @staticmethod
    def backward(ctx, *grads):
        ws, sl, pad, packed, rec, R = ctx.meta
        L = len(ws)
        live = ctx.live
        nl = sum(live)
        saved = ctx.saved_tensors
        dzx, dh, dc = [None] * L, [None] * L, [None] * L
        lib = _native.load()
        k = -1
        for i in range(L):
            if not live[i]:
                if grads[i] is not None or grads[L + i] is not None:
                    raise RuntimeError('DRC step: a gradient reached layer %d, whose x half was computed without '
                                       'autograd (DRC.x_halves)' % i)
                continue
            k += 1
            gh, gc = grads[i], grads[L + i]
            if gh is None and gc is None:
                continue
            w = ws[i]
            gh = None if gh is None else gh.contiguous()
            gc = None if gc is None else gc.contiguous()
            N = saved[4 * k].shape[0]
            H = saved[4 * k].shape[1]
            G = 4 * H
            Cf = w.shape[0]
            split = (GBOARD_ADJOINT_SPLIT and Cf % 32 == 0 and 2 <= Cf // 32 <= 8 and H % 16 == 0
                     and tuple(pad) == (1, 1) and tuple(w.shape[2:]) == (3, 3))
            S = Cf // 32 if split else 1
            acc = torch.empty(N, G, 6, 6, device=w.device) if ctx.needs_input_grad[1 + i] else None
            dh_t, dh_stride, dh_parts = gh, H * 36, 1
            for r in range(R - 1, -1, -1):
                h_r, c_r, co_r, g_r = saved[4 * (r * nl + k):4 * (r * nl + k) + 4]
                dz = torch.empty_like(g_r)
                dcr = torch.empty_like(c_r)
                _native.check(lib.hrl_lstm_gates_backward_ex(
                    _native.ptr(g_r), _native.ptr(c_r), _native.ptr(co_r), _native.ptr(dh_t), dh_stride, dh_parts,
                    H * 36, _native.ptr(gc), N, H, 36, _native.ptr(dz), _native.ptr(dcr), _native.ptr(acc),
                    int(r == R - 1), _native.stream_of(dz.device)), 'hrl_lstm_gates_backward_ex')
                rec.add_conv((w, None, sl, tuple(pad)), h_r, dz, late=True)
                gc = dcr
                if r == 0 and not ctx.needs_input_grad[1 + L + i]:
                    break
                if split:   # the S partial input gradients, summed by the next gate backward (or below)
                    dh_t = gboard_conv(dz, rec.adjoint_pack(w, sl[0], H, split=True), S * H, 32, groups=S)
                    dh_stride, dh_parts = S * H * 36, S
                else:
                    dh_t = _deferred_conv_dx(dz, h_r, w, sl, pad, rec)
                    dh_stride, dh_parts = H * 36, 1
            dzx[i] = acc
            if ctx.needs_input_grad[1 + L + i]:
                dh[i] = dh_t.view(N, S, H, 6, 6).sum(1) if dh_parts > 1 else dh_t
            dc[i] = gc if ctx.needs_input_grad[1 + 2 * L + i] else None
        return (None, *dzx, *dh, *dc)


def drc_step_ok(zx, hs, cs, ws, pad):
    """_DRCStep covers: 1..4 layers of 3x3 'same' cells on the 6x6 board, H = 32 hidden channels, fp32 CUDA
    float4-aligned games (zx may be channel slices of a wider tensor)."""
    L = len(ws)
    if not (1 <= L <= 4 and tuple(pad) == (1, 1)):
        return False
    H = hs[0].shape[1]
    return (H == 32 and all(tuple(w.shape[2:]) == (3, 3) and w.shape[0] == 4 * H for w in ws)
            and all(gboard_ok(t) for t in hs) and all(gboard_ok(t) and t.is_contiguous() for t in cs)
            and all(gboard_ok(z) and z.shape[1] == 4 * H for z in zx)
            and all(t.shape[0] == hs[0].shape[0] for t in (*zx, *hs, *cs)))


def drc_step(zx, hs, cs, ws, sl, pad, packed, repeats):
    """The repeats of the DRC cells at one time step of a deferred unroll (_DRCStep); returns (hs', cs')."""
    L = len(ws)
    out = _DRCStep.apply((ws, sl, tuple(pad), packed, _DEFER, repeats), *zx, *hs, *cs)
    return list(out[:L]), list(out[L:])


def conv2d(x, w, b=None, padding=(0, 0), in_slice=None, packed=None):
    """F.conv2d (stride 1) of the env nets; inside deferred_weight_grads() the weight gradient is
    batched over the unroll (DeferredGrads) and the forward of 3x3 32-channel board convs runs on
    the MFMA board conv (``packed``: its weights packed once for the unroll -- gboard_pack on the 6x6 board
    (gboard_conv_ok), board_conv_pack otherwise)."""
    if _DEFER is not None and torch.is_grad_enabled() and w.requires_grad:
        return _DeferredConv.apply(x, w, b, in_slice, tuple(padding), _DEFER, packed)
    wv = w if in_slice is None else w[:, in_slice[0]:in_slice[1]]
    return F.conv2d(x, wv, b, padding=padding)


class _BatchNormTrain(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, running_mean, running_var, momentum, eps, relu=False, groups=1):
        N, C = x.shape[0], x.shape[1]
        HW = x[0, 0].numel()
        x = x.contiguous()
        lib = _native.load()
        ws_bytes = lib.hrl_bn_workspace_bytes_grouped(N, C, HW, groups)
        if ws_bytes < 0:
            raise ValueError('hrl_bn: unsupported shape %s (groups %d)' % (tuple(x.shape), groups))
        ws = torch.empty(ws_bytes, dtype=torch.uint8, device=x.device)
        y = torch.empty_like(x)
        mean = torch.empty(groups, C, dtype=torch.float32, device=x.device)
        invstd = torch.empty(groups, C, dtype=torch.float32, device=x.device)
        code = lib.hrl_bn_forward_train_grouped(
            _native.ptr(x), N, C, HW, groups, _native.ptr(weight), _native.ptr(bias),
            _native.ptr(running_mean), _native.ptr(running_var), float(momentum), float(eps), int(relu),
            _native.ptr(y), _native.ptr(mean), _native.ptr(invstd), _native.ptr(ws), ws_bytes,
            _native.stream_of(x.device))
        _native.check(code, 'hrl_bn_forward_train_grouped')
        ctx.save_for_backward(x, weight, bias, mean, invstd)
        ctx.has_bias = bias is not None
        ctx.relu = bool(relu)
        ctx.groups = groups
        ctx.defer = _DEFER if (weight is not None and weight.requires_grad) else None
        return y

    @staticmethod
    def backward(ctx, dy):
        x, weight, bias, mean, invstd = ctx.saved_tensors
        N, C = x.shape[0], x.shape[1]
        HW = x[0, 0].numel()
        dy = dy.contiguous()
        lib = _native.load()
        ws_bytes = lib.hrl_bn_workspace_bytes_grouped(N, C, HW, ctx.groups)
        ws = torch.empty(ws_bytes, dtype=torch.uint8, device=x.device)
        dx = torch.empty_like(x)
        # the affine gradients straight into .grad when they may be written in place (direct_grads: the
        # parameter's first use in the step), else into fresh tensors for the deferral / autograd
        bw = _grad_buffer(weight) if (weight is not None and ctx.needs_input_grad[1]) else (None, False)
        bb = _grad_buffer(bias) if (ctx.has_bias and ctx.needs_input_grad[2]) else (None, False)
        dw = bw[0] if bw[0] is not None else (torch.empty(C, dtype=torch.float32, device=x.device)
                                              if weight is not None else None)
        db = bb[0] if bb[0] is not None else (torch.empty(C, dtype=torch.float32, device=x.device)
                                              if ctx.has_bias else None)
        code = lib.hrl_bn_backward_grouped(
            _native.ptr(x), _native.ptr(dy), N, C, HW, ctx.groups, _native.ptr(weight), _native.ptr(bias),
            _native.ptr(mean), _native.ptr(invstd), int(ctx.relu), _native.ptr(dx), _native.ptr(dw), _native.ptr(db),
            _native.ptr(ws), ws_bytes, _native.stream_of(x.device))
        _native.check(code, 'hrl_bn_backward_grouped')
        dw_out = None if bw[1] else dw
        db_out = None if bb[1] else db
        if ctx.defer is not None and (dw_out is not None or db_out is not None):
            ctx.defer.add_affine((weight if dw_out is not None else None,
                                  bias if (ctx.has_bias and db_out is not None) else None), dw_out, db_out)
            return dx, None, None, None, None, None, None, None, None
        return dx, dw_out, db_out, None, None, None, None, None, None


def batch_norm_train(x, weight, bias, running_mean, running_var, momentum, eps, relu=False, groups=1):
    """F.batch_norm(..., training=True) [+ ReLU] on the HIP kernels (x: (N, C, *spatial) fp32 CUDA).
    ``groups`` > 1: rows [g*N/groups, (g+1)*N/groups) are normalised with statistics of their own, and the
    running statistics advance once per group in order -- ``groups`` sequential calls in one launch each
    way (a recurrent net's per-time-step BatchNorm over its whole unroll)."""
    return _BatchNormTrain.apply(x, weight, bias, running_mean, running_var, momentum, eps, relu, groups)


def batch_norm_eval(x, weight, bias, running_mean, running_var, eps, relu=False):
    """Inference BatchNorm [+ ReLU] from the running statistics (hrl_bn_forward_eval); not differentiable."""
    if torch.is_grad_enabled() and (x.requires_grad or (weight is not None and weight.requires_grad)):
        y = torch.nn.functional.batch_norm(x, running_mean, running_var, weight, bias, False, 0.0, eps)
        return torch.relu(y) if relu else y
    x = x.contiguous()
    N, C = x.shape[0], x.shape[1]
    y = torch.empty_like(x)
    coef = torch.empty(2 * C, dtype=torch.float32, device=x.device)
    _native.check(_native.load().hrl_bn_forward_eval(
        _native.ptr(x), N, C, x[0, 0].numel(), _native.ptr(weight), _native.ptr(bias), _native.ptr(running_mean),
        _native.ptr(running_var), float(eps), int(relu), _native.ptr(y), _native.ptr(coef),
        _native.stream_of(x.device)), 'hrl_bn_forward_eval')
    return y


BOARD_MAX_CELLS = 16
ROWS_MIN_CHUNKED = 4096


def _xt_dy(x, dy):
    """x^T @ dy for tall (M x K), (M x N) operands.

    hipBLASLt runs the single reduction-over-M GEMM at 5-55 TF on these shapes
    (M = B*T*P ~ 1e5, K or N as small as 9); split M into S chunks, one
    batched GEMM, then a sum over chunks: 2-6x faster, same fp32 accuracy.
    """
    M, K = x.shape
    N = dy.shape[1]
    S = 16 if K * N >= 32768 else 64
    if M < ROWS_MIN_CHUNKED or M % S:
        return x.t() @ dy
    return torch.bmm(x.view(S, M // S, K).transpose(1, 2), dy.view(S, M // S, N)).sum(0)


def _colsum(dy):
    """dy.sum(0) for a (M, N) CUDA fp32 matrix: csrc/hrl_board.hip (framework column sums run ~20x slower)."""
    M, N = dy.shape
    if not (dy.is_cuda and dy.dtype == torch.float32 and N <= 256 and M >= ROWS_MIN_CHUNKED):
        return dy.sum(0)
    dy = dy.contiguous()
    lib = _native.load()
    ws_bytes = lib.hrl_colsum_workspace_bytes(M, N)
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dy.device)
    out = torch.empty(N, dtype=dy.dtype, device=dy.device)
    _native.check(lib.hrl_colsum(_native.ptr(dy), M, N, _native.ptr(out), _native.ptr(ws), ws_bytes,
                                 _native.stream_of(dy.device)), 'hrl_colsum')
    return out


class _RowMatmul(torch.autograd.Function):
    """y = x @ w (+ bias) over many rows, with the chunked weight-gradient GEMM."""

    @staticmethod
    def forward(ctx, x, w, bias):
        ctx.save_for_backward(x, w)
        ctx.has_bias = bias is not None
        return torch.addmm(bias, x, w) if bias is not None else x @ w

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        dx = dy @ w.t() if ctx.needs_input_grad[0] else None
        dw = _xt_dy(x, dy) if ctx.needs_input_grad[1] else None
        db = _colsum(dy) if ctx.has_bias and ctx.needs_input_grad[2] else None
        return dx, dw, db


class Linear(nn.Linear):
    """nn.Linear whose weight gradient over many rows uses the chunked GEMM."""

    def forward(self, x):
        if not (x.is_cuda and x.dim() == 2 and x.shape[0] >= ROWS_MIN_CHUNKED and x.dtype == torch.float32):
            return super().forward(x)
        return _RowMatmul.apply(x, self.weight.t(), self.bias)


class BoardConv2d(nn.Conv2d):
    """nn.Conv2d computed as one dense GEMM over the flattened board (see module doc)."""

    def forward(self, x):
        if not (x.is_cuda and x.dim() == 4 and x.dtype == torch.float32
                and x.shape[2] * x.shape[3] <= BOARD_MAX_CELLS):
            if _DEFER is not None and x.is_cuda and self.padding_mode == 'zeros' and self.stride == (1, 1) \
                    and self.dilation == (1, 1) and self.groups == 1 and isinstance(self.padding, tuple):
                return conv2d(x, self.weight, self.bias, self.padding)
            return super().forward(x)
        N, Cin, H, W = x.shape
        if (H, W) == (3, 3) and self.kernel_size == (3, 3) and Cin == 32 and self.out_channels == 32 and N > 0:
            return _Conv3x3.apply(x.contiguous(), self.weight, self.bias)   # block-sparse MFMA kernels
        if ((H, W) == (3, 3) and self.kernel_size == (3, 3) and Cin <= 3 and self.out_channels == 32 and N > 0
                and not x.requires_grad):
            return _StemConv.apply(x.contiguous(), self.weight, self.bias)  # the observation stem
        w_board = _BoardWeight.apply(self.weight, H, W)              # (Cin*HW, Cout*HW)
        bias = _BoardBias.apply(self.bias, H * W) if self.bias is not None else None
        x2 = x.reshape(N, Cin * H * W)
        if bias is not None and Cin * H * W < 64:
            # narrow input (the stem: 3 planes x 9 cells): carry the bias as an extra all-ones
            # input column, so its gradient comes out of the weight-gradient GEMM instead of a
            # separate column reduction over all N rows
            x2 = torch.cat([x2, x2.new_ones(N, 1)], dim=1)
            w_board = torch.cat([w_board, bias.view(1, -1)], dim=0)
            bias = None
        return _RowMatmul.apply(x2, w_board, bias).view(N, self.out_channels, H, W)


class _Conv3x3(torch.autograd.Function):
    """32->32 3x3 conv on a 3x3 board: csrc/hrl_conv.hip (fp32 MFMA, off-board taps skipped)."""

    @staticmethod
    def forward(ctx, x, weight, bias):
        N = x.shape[0]
        lib = _native.load()
        ws_bytes = lib.hrl_conv3x3_workspace_bytes(N)
        ws = torch.empty(ws_bytes, dtype=torch.uint8, device=x.device)
        y = torch.empty_like(x)
        w = weight.contiguous()
        _native.check(lib.hrl_conv3x3_forward(_native.ptr(x), N, 32, 32, _native.ptr(w), _native.ptr(bias), 0,
                                              _native.ptr(y), _native.ptr(ws), ws_bytes,
                                              _native.stream_of(x.device)), 'hrl_conv3x3_forward')
        ctx.save_for_backward(x, w)
        ctx.has_bias = bias is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        dy = dy.contiguous()
        N = x.shape[0]
        lib = _native.load()
        ws_bytes = lib.hrl_conv3x3_workspace_bytes(N)
        ws = torch.empty(ws_bytes, dtype=torch.uint8, device=x.device)
        stream = _native.stream_of(x.device)
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty_like(x)
            _native.check(lib.hrl_conv3x3_forward(_native.ptr(dy), N, 32, 32, _native.ptr(w), None, 1,
                                                  _native.ptr(dx), _native.ptr(ws), ws_bytes, stream),
                          'hrl_conv3x3_forward(flip)')
        if ctx.needs_input_grad[1]:
            dw = torch.empty_like(w)
            _native.check(lib.hrl_conv3x3_wgrad(_native.ptr(x), _native.ptr(dy), N, 32, 32, _native.ptr(dw),
                                                _native.ptr(ws), ws_bytes, stream), 'hrl_conv3x3_wgrad')
        if ctx.has_bias and ctx.needs_input_grad[2]:
            db = dy.sum((0, 2, 3))
        return dx, dw, db


def torus_supported(x, weight):
    """Shapes csrc/hrl_torus.hip covers: 3x3, 17 or 32 -> 32 channels, boards of at most 80 cells."""
    return (x.is_cuda and x.dtype == torch.float32 and x.dim() == 4 and x.shape[0] > 0
            and weight.shape[0] == 32 and weight.shape[1] in (17, 32) and tuple(weight.shape[2:]) == (3, 3)
            and x.shape[1] == weight.shape[1] and x.shape[2] * x.shape[3] <= 80)


class _TorusConv(torch.autograd.Function):
    """3x3 conv on a torus board (GeeseNet TorusConv2d): csrc/hrl_torus.hip, fp32 MFMA, wrap as addressing."""

    @staticmethod
    def forward(ctx, x, weight, bias):
        x = x.contiguous()
        N, Cin, H, W = x.shape
        lib = _native.load()
        ws_bytes = lib.hrl_torus_workspace_bytes(N)
        ws = torch.empty(ws_bytes, dtype=torch.uint8, device=x.device)
        y = torch.empty(N, 32, H, W, device=x.device, dtype=x.dtype)
        w = weight.contiguous()
        _native.check(lib.hrl_torus_conv_forward(_native.ptr(x), N, Cin, 32, H, W, _native.ptr(w),
                                                 _native.ptr(bias), 0, _native.ptr(y), None, None, None,
                                                 _native.ptr(ws), ws_bytes, _native.stream_of(x.device)),
                      'hrl_torus_conv_forward')
        ctx.save_for_backward(x, w)
        ctx.has_bias = bias is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        dy = dy.contiguous()
        N, Cin, H, W = x.shape
        lib = _native.load()
        ws_bytes = lib.hrl_torus_workspace_bytes(N)
        ws = torch.empty(ws_bytes, dtype=torch.uint8, device=x.device)
        stream = _native.stream_of(x.device)
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty_like(x)
            _native.check(lib.hrl_torus_conv_forward(_native.ptr(dy), N, Cin, 32, H, W, _native.ptr(w), None, 1,
                                                     _native.ptr(dx), None, None, None, _native.ptr(ws), ws_bytes,
                                                     stream),
                          'hrl_torus_conv_forward(flip)')
        if ctx.needs_input_grad[1] or (ctx.has_bias and ctx.needs_input_grad[2]):
            dw = torch.empty_like(w)
            db = torch.empty(32, device=x.device, dtype=x.dtype) if ctx.has_bias else None
            _native.check(lib.hrl_torus_conv_wgrad(_native.ptr(x), _native.ptr(dy), N, Cin, 32, H, W,
                                                   _native.ptr(dw), _native.ptr(db), _native.ptr(ws), ws_bytes,
                                                   stream), 'hrl_torus_conv_wgrad')
            if not ctx.needs_input_grad[1]:
                dw = None
        return dx, dw, db


def torus_conv2d(x, weight, bias=None):
    return _TorusConv.apply(x, weight, bias)


class _TorusBNBlock(torch.autograd.Function):
    """One GeeseNet unit in training mode, out = relu([h +] bn(conv_torus(h))) (hungry_geese.py:48-51):

    forward : torus conv with the BatchNorm statistics in its epilogue -> finalize (running stats)
              -> one residual apply pass;
    backward: masked BatchNorm backward (gradient * [out > 0]) -> weight gradient -> input gradient
              whose store also adds the residual branch's masked gradient.
    h and out are the only activations besides the conv output y that reach HBM.
    """

    @staticmethod
    def forward(ctx, h, weight, bias, gamma, beta, running_mean, running_var, momentum, eps, residual):
        h = h.contiguous()
        N, Cin, H, W = h.shape
        HW = H * W
        dev = h.device
        lib = _native.load()
        stream = _native.stream_of(dev)
        ws_bytes = lib.hrl_torus_workspace_bytes(N)
        ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
        nparts = lib.hrl_torus_stats_blocks(N)
        part = torch.empty(nparts * 64, dtype=torch.float64, device=dev)
        y = torch.empty(N, 32, H, W, device=dev, dtype=h.dtype)
        w = weight.contiguous()
        _native.check(lib.hrl_torus_conv_forward(_native.ptr(h), N, Cin, 32, H, W, _native.ptr(w), _native.ptr(bias),
                                                 0, _native.ptr(y), _native.ptr(part), None, None, _native.ptr(ws),
                                                 ws_bytes, stream), 'hrl_torus_conv_forward(stats)')
        coef = torch.empty(4, 32, device=dev, dtype=h.dtype)   # save_mean, save_invstd, alpha, beta
        _native.check(lib.hrl_bn_finalize_stats(_native.ptr(part), nparts, 32, N * HW, _native.ptr(gamma),
                                                _native.ptr(beta), _native.ptr(running_mean),
                                                _native.ptr(running_var), momentum, eps, _native.ptr(coef[0]),
                                                _native.ptr(coef[1]), _native.ptr(coef[2]), _native.ptr(coef[3]),
                                                stream), 'hrl_bn_finalize_stats')
        out = torch.empty_like(y)
        _native.check(lib.hrl_bn_apply_residual(_native.ptr(y), _native.ptr(h) if residual else None, N, 32, HW,
                                                _native.ptr(coef[2]), _native.ptr(coef[3]), _native.ptr(out), stream),
                      'hrl_bn_apply_residual')
        ctx.save_for_backward(h, w, gamma, y, out, coef)
        ctx.residual = residual
        ctx.has_bias = bias is not None
        return out

    @staticmethod
    def backward(ctx, g):
        h, w, gamma, y, out, coef = ctx.saved_tensors
        g = g.contiguous()
        N, Cin, H, W = h.shape
        HW = H * W
        dev = h.device
        lib = _native.load()
        stream = _native.stream_of(dev)
        bn_ws_bytes = lib.hrl_bn_workspace_bytes(N, 32, HW)
        ws_bytes = max(lib.hrl_torus_workspace_bytes(N), bn_ws_bytes)
        ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
        dy = torch.empty_like(y)
        dgamma = torch.empty(32, device=dev, dtype=y.dtype)
        dbeta = torch.empty(32, device=dev, dtype=y.dtype)
        _native.check(lib.hrl_bn_backward_masked(_native.ptr(y), _native.ptr(g), _native.ptr(out), N, 32, HW,
                                                 _native.ptr(gamma), _native.ptr(coef[0]), _native.ptr(coef[1]),
                                                 _native.ptr(dy), _native.ptr(dgamma), _native.ptr(dbeta),
                                                 _native.ptr(ws), bn_ws_bytes, stream), 'hrl_bn_backward_masked')
        dw = torch.empty_like(w)
        db = torch.empty(32, device=dev, dtype=y.dtype) if ctx.has_bias else None
        _native.check(lib.hrl_torus_conv_wgrad(_native.ptr(h), _native.ptr(dy), N, Cin, 32, H, W, _native.ptr(dw),
                                               _native.ptr(db), _native.ptr(ws), ws_bytes, stream),
                      'hrl_torus_conv_wgrad')
        dh = None
        if ctx.needs_input_grad[0]:
            dh = torch.empty_like(h)
            add = g if ctx.residual else None
            _native.check(lib.hrl_torus_conv_forward(_native.ptr(dy), N, Cin, 32, H, W, _native.ptr(w), None, 1,
                                                     _native.ptr(dh), None, _native.ptr(add),
                                                     _native.ptr(out) if ctx.residual else None, _native.ptr(ws),
                                                     ws_bytes, stream), 'hrl_torus_conv_forward(flip, residual)')
        return dh, dw, db, dgamma, dbeta, None, None, None, None, None


def torus_block(h, unit, residual):
    """relu([h +] unit(h)) for a training-mode TorusConv2d ``unit`` (conv + BatchNorm2d) as one fused
    HIP Function; the BatchNorm module's batch counter and running statistics advance as in its forward."""
    bn = unit.bn
    momentum = 0.0 if bn.momentum is None else bn.momentum
    if bn.track_running_stats and bn.num_batches_tracked is not None:
        bn.num_batches_tracked.add_(1)
        if bn.momentum is None:
            momentum = 1.0 / float(bn.num_batches_tracked.item())
    return _TorusBNBlock.apply(h, unit.conv.weight, unit.conv.bias, bn.weight, bn.bias,
                               bn.running_mean if bn.track_running_stats else None,
                               bn.running_var if bn.track_running_stats else None, momentum, bn.eps, residual)


class _TorusTower(torch.autograd.Function):
    """GeeseNet's unit chain in training mode (hungry_geese.py:48-51): the stem h_1 = relu(bn_0(conv_0(x)))
    and h_{i+1} = relu(h_i + bn_i(conv_i(h_i))), with every BatchNorm pass but one folded into a conv:

    forward : stem conv (+ BN statistics) -> finalize; unit i's conv builds its input h_i from the previous
              unit's conv output in its prologue (hrl_torus_unit_forward) -> finalize; one residual apply for
              the last unit's output;
    backward: the last unit's masked BN backward; per unit: weight gradient -> input gradient whose epilogue
              adds the residual branch and sums the previous unit's masked BN backward terms
              (hrl_torus_unit_input_grad) -> finalize -> masked BN backward apply.
    Per unit only h_i and y_i reach HBM (as with the per-unit Functions); the residual-apply and masked
    reduce passes of nn.torus_block are gone.  ``units`` carries each BatchNorm's running statistics,
    momentum and eps; ``params`` is (conv weight, conv bias, bn weight, bn bias) per unit.

    residual_in: the chain starts at a residual unit whose input x is also its residual (the upper part of a
    tower split in two, torus_tower's `split`): h_1 = relu(x + bn_0(conv_0(x))), and the input gradient adds
    the residual branch (g_1 [h_1 > 0]) to the first conv's adjoint.
    """

    @staticmethod
    def forward(ctx, x, units, residual_in, *params):
        x = x.contiguous()
        N, Cin, H, W = x.shape
        HW = H * W
        dev = x.device
        lib = _native.load()
        stream = _native.stream_of(dev)
        n = len(units)
        ws_bytes = max(lib.hrl_torus_workspace_bytes(N), lib.hrl_bn_workspace_bytes(N, 32, HW))
        ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
        nparts = lib.hrl_torus_stats_blocks(N)
        part = torch.empty(nparts * 64, dtype=torch.float64, device=dev)
        coef = torch.empty(n, 4, 32, device=dev, dtype=x.dtype)   # per unit: save_mean, save_invstd, alpha, beta
        ws_ = (_native.ptr(ws), ws_bytes, stream)
        P = _native.ptr
        weights = [params[4 * i].contiguous() for i in range(n)]
        ys, hs = [], [x]
        for i in range(n):
            w, b, gamma, beta = weights[i], params[4 * i + 1], params[4 * i + 2], params[4 * i + 3]
            y = torch.empty(N, 32, H, W, device=dev, dtype=x.dtype)
            if i == 0:
                _native.check(lib.hrl_torus_conv_forward(P(x), N, Cin, 32, H, W, P(w), P(b), 0, P(y), P(part), None,
                                                         None, *ws_), 'hrl_torus_conv_forward(stats)')
            else:
                h = torch.empty(N, 32, H, W, device=dev, dtype=x.dtype)
                res = hs[-1] if (i >= 2 or residual_in) else None
                _native.check(lib.hrl_torus_unit_forward(P(ys[-1]), P(res), P(coef[i - 1, 2]),
                                                         P(coef[i - 1, 3]), P(h), N, H, W, P(w), P(b), P(y), P(part),
                                                         *ws_), 'hrl_torus_unit_forward')
                hs.append(h)
            rm, rv, momentum, eps = units[i]
            _native.check(lib.hrl_bn_finalize_stats(P(part), nparts, 32, N * HW, P(gamma), P(beta), P(rm), P(rv),
                                                    momentum, eps, P(coef[i, 0]), P(coef[i, 1]), P(coef[i, 2]),
                                                    P(coef[i, 3]), stream), 'hrl_bn_finalize_stats')
            ys.append(y)
        out = torch.empty_like(ys[-1])
        _native.check(lib.hrl_bn_apply_residual(P(ys[-1]), P(hs[-1]) if (n >= 2 or residual_in) else None, N, 32, HW,
                                                P(coef[n - 1, 2]), P(coef[n - 1, 3]), P(out), stream),
                      'hrl_bn_apply_residual')
        gammas = [params[4 * i + 2] for i in range(n)]
        ctx.save_for_backward(out, coef, *weights, *gammas, *ys, *hs)
        ctx.n = n
        ctx.residual_in = bool(residual_in)
        ctx.has_bias = [params[4 * i + 1] is not None for i in range(n)]
        return out

    @staticmethod
    def backward(ctx, g):
        n = ctx.n
        saved = ctx.saved_tensors
        out, coef = saved[0], saved[1]
        weights, gammas = saved[2:2 + n], saved[2 + n:2 + 2 * n]
        ys, hs = saved[2 + 2 * n:2 + 3 * n], saved[2 + 3 * n:]
        g = g.contiguous()
        x = hs[0]
        N, Cin, H, W = x.shape
        HW = H * W
        dev = x.device
        lib = _native.load()
        stream = _native.stream_of(dev)
        P = _native.ptr
        bn_ws_bytes = lib.hrl_bn_workspace_bytes(N, 32, HW)
        ws_bytes = max(lib.hrl_torus_workspace_bytes(N), bn_ws_bytes)
        ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
        nparts = lib.hrl_torus_stats_blocks(N)
        part = torch.empty(nparts * 64, dtype=torch.float64, device=dev)
        kg = torch.empty(2, 32, device=dev, dtype=g.dtype)   # k, mean(dy) of the unit being applied
        grads = [None] * (4 * n)
        for i in range(n):
            grads[4 * i + 2] = torch.empty(32, device=dev, dtype=g.dtype)
            grads[4 * i + 3] = torch.empty(32, device=dev, dtype=g.dtype)
        # TOWER_BN_FOLD: every unit's masked BN backward apply is formed in its weight gradient's staging
        # (hrl_torus_conv_wgrad_bn, which writes dy for the input gradient) instead of a pass of its own
        fold = TOWER_BN_FOLD
        dy = torch.empty_like(ys[-1])
        if fold:
            _native.check(lib.hrl_bn_backward_masked_coefs(P(ys[-1]), P(g), P(out), N, 32, HW, P(gammas[-1]),
                                                           P(coef[n - 1, 0]), P(coef[n - 1, 1]), P(kg[0]), P(kg[1]),
                                                           P(grads[4 * n - 2]), P(grads[4 * n - 1]), P(ws),
                                                           bn_ws_bytes, stream), 'hrl_bn_backward_masked_coefs')
        else:
            _native.check(lib.hrl_bn_backward_masked(P(ys[-1]), P(g), P(out), N, 32, HW, P(gammas[-1]),
                                                     P(coef[n - 1, 0]), P(coef[n - 1, 1]), P(dy), P(grads[4 * n - 2]),
                                                     P(grads[4 * n - 1]), P(ws), bn_ws_bytes, stream),
                          'hrl_bn_backward_masked')
        g_cur = g
        dx = None
        for i in range(n - 1, -1, -1):
            dw = torch.empty_like(weights[i])
            db = torch.empty(32, device=dev, dtype=g.dtype) if ctx.has_bias[i] else None
            cin = Cin if i == 0 else 32
            if fold:
                residual = 1 if (i >= 1 or ctx.residual_in) else 0   # unit i's block output relu([h_i +] bn(y_i))
                _native.check(lib.hrl_torus_conv_wgrad_bn(P(hs[i]), N, cin, H, W, P(ys[i]), P(g_cur), P(coef[i, 2]),
                                                          P(coef[i, 3]), residual, P(gammas[i]), P(coef[i, 0]),
                                                          P(coef[i, 1]), P(kg[0]), P(kg[1]), P(dy), P(dw), P(db),
                                                          P(ws), ws_bytes, stream), 'hrl_torus_conv_wgrad_bn')
            else:
                _native.check(lib.hrl_torus_conv_wgrad(P(hs[i]), P(dy), N, cin, 32, H, W, P(dw), P(db), P(ws),
                                                       ws_bytes, stream), 'hrl_torus_conv_wgrad')
            grads[4 * i], grads[4 * i + 1] = dw, db
            if i == 0:
                if ctx.needs_input_grad[0]:
                    dx = torch.empty_like(x)
                    # residual_in: + the residual branch g_1 [h_1 > 0] (h_1: the next unit's input, or the output)
                    add, mask = (g_cur, hs[1] if n > 1 else out) if ctx.residual_in else (None, None)
                    _native.check(lib.hrl_torus_conv_forward(P(dy), N, Cin, 32, H, W, P(weights[0]), None, 1, P(dx),
                                                             None, P(add), P(mask), P(ws), ws_bytes, stream),
                                  'hrl_torus_conv_forward(flip)')
                break
            out_i = hs[i + 1] if i + 1 < n else out
            g_prev = torch.empty_like(g_cur)
            _native.check(lib.hrl_torus_unit_input_grad(P(dy), N, H, W, P(weights[i]), P(g_cur), P(out_i), P(g_prev),
                                                        P(hs[i]), P(ys[i - 1]), P(coef[i - 1, 0]), P(part), P(ws),
                                                        ws_bytes, stream), 'hrl_torus_unit_input_grad')
            _native.check(lib.hrl_bn_finalize_backward(P(part), nparts, 32, N * HW, P(gammas[i - 1]),
                                                       P(coef[i - 1, 1]), P(grads[4 * i - 2]), P(grads[4 * i - 1]),
                                                       P(kg[0]), P(kg[1]), stream), 'hrl_bn_finalize_backward')
            if not fold:
                dy = torch.empty_like(dy)
                _native.check(lib.hrl_bn_backward_apply_masked(P(ys[i - 1]), P(g_prev), P(hs[i]), N, 32, HW,
                                                               P(gammas[i - 1]), P(coef[i - 1, 0]), P(coef[i - 1, 1]),
                                                               P(kg[0]), P(kg[1]), P(dy), stream),
                              'hrl_bn_backward_apply_masked')
            g_cur = g_prev
        return (dx, None, None, *grads)


# _TorusTower's backward forms each unit's masked BatchNorm backward apply inside its weight gradient (True) or
# runs it as a pass of its own (False; bit-identical, tests/test_geese.py::test_tower_bn_fold_is_bit_identical)
TOWER_BN_FOLD = True

# A data-parallel learner's segmented capture (trainer.LearnerStep._grab_cut_tensor): called with the tensor
# between the two parts of a split tower, it returns the view that is the backward's cut
_CUT_FN = None


def torus_tower(x, units):
    """The chain relu(bn(conv(x))) -> relu(h + bn(conv(h))) ... over training-mode TorusConv2d ``units``
    (GeeseNet's conv0 and blocks, hungry_geese.py:48-51) as one HIP Function (_TorusTower); each
    BatchNorm module's batch counter and running statistics advance as in its forward.

    ``units[0].tower_split = k`` (set by a data-parallel LearnerStep) runs it as two Functions, units [0, k) and
    [k, n) (the second with residual_in), so the backward can be cut between them and the upper part's gradient
    all-reduce overlaps the lower part's backward; the value between them passes through _CUT_FN when set."""
    k = getattr(units[0], 'tower_split', None)
    if k is not None and 0 < k < len(units):
        h = _tower_part(x, units[:k], False)
        if _CUT_FN is not None:
            h = _CUT_FN(h)
        return _tower_part(h, units[k:], True)
    return _tower_part(x, units, False)


def _tower_part(x, units, residual_in):
    meta, params = [], []
    for unit in units:
        bn = unit.bn
        momentum = 0.0 if bn.momentum is None else bn.momentum
        if bn.track_running_stats and bn.num_batches_tracked is not None:
            bn.num_batches_tracked.add_(1)
            if bn.momentum is None:
                momentum = 1.0 / float(bn.num_batches_tracked.item())
        meta.append((bn.running_mean if bn.track_running_stats else None,
                     bn.running_var if bn.track_running_stats else None, momentum, bn.eps))
        params += [unit.conv.weight, unit.conv.bias, bn.weight, bn.bias]
    return _TorusTower.apply(x, meta, residual_in, *params)


class _GeesePool(torch.autograd.Function):
    """GeeseNet's head pooling (hungry_geese.py:52-53): h_head = sum over cells of h * x[:, :1],
    h_avg = mean over cells of h, as csrc/hrl_torus.hip head_pool / head_unpool (one pass each way).
    x is the net's input (data): no gradient flows to it."""

    @staticmethod
    def forward(ctx, h, x):
        h = h.contiguous()
        x = x.contiguous()
        N, C, H, W = h.shape
        lib = _native.load()
        head = torch.empty(N, C, device=h.device, dtype=h.dtype)
        avg = torch.empty(N, C, device=h.device, dtype=h.dtype)
        _native.check(lib.hrl_torus_head_pool(_native.ptr(h), _native.ptr(x), N, H, W, x.shape[1] * H * W,
                                              _native.ptr(head), _native.ptr(avg), _native.stream_of(h.device)),
                      'hrl_torus_head_pool')
        ctx.save_for_backward(x)
        ctx.hshape = h.shape
        return head, avg

    @staticmethod
    def backward(ctx, dhead, davg):
        x, = ctx.saved_tensors
        N, C, H, W = ctx.hshape
        lib = _native.load()
        dhead = torch.zeros(N, C, device=x.device, dtype=x.dtype) if dhead is None else dhead.contiguous()
        davg = torch.zeros(N, C, device=x.device, dtype=x.dtype) if davg is None else davg.contiguous()
        g = torch.empty(N, C, H, W, device=x.device, dtype=x.dtype)
        _native.check(lib.hrl_torus_head_unpool(_native.ptr(dhead), _native.ptr(davg), _native.ptr(x), N, H, W,
                                                x.shape[1] * H * W, _native.ptr(g), _native.stream_of(x.device)),
                      'hrl_torus_head_unpool')
        return g, None


def geese_pool(h, x):
    """(h_head, h_avg) of GeeseNet's heads on the GPU (HIP, one pass each way); h (N, 32, H, W)."""
    if h.shape[1] != 32 or h.dtype != torch.float32 or x.dtype != torch.float32:
        raise RuntimeError('geese_pool: expects float32 h with 32 channels, got %s %s'
                           % (tuple(h.shape), h.dtype))
    return _GeesePool.apply(h, x)


def _board_head_spec(m):
    """(conv, fc) of a TicTacToe-style Head (tictactoe.py:35-49): 1x1 conv with bias and no BatchNorm ->
    LeakyReLU(0.1) -> flatten -> bias-free Linear; None for anything else.  Matches the reference's Head
    (``activation = nn.LeakyReLU(0.1)``) and envs.tictactoe.BoardHead (``LEAKY_SLOPE``)."""
    unit, fc = getattr(m, 'conv', None), getattr(m, 'fc', None)
    conv = getattr(unit, 'conv', None)
    if not isinstance(fc, nn.Linear) or fc.bias is not None or not isinstance(conv, nn.Conv2d):
        return None
    if getattr(unit, 'bn', 0) is not None or conv.bias is None or conv.kernel_size != (1, 1) or \
            conv.stride != (1, 1) or conv.groups != 1 or conv.padding_mode != 'zeros':
        return None
    act = getattr(m, 'activation', None)
    slope = act.negative_slope if isinstance(act, nn.LeakyReLU) else getattr(m, 'LEAKY_SLOPE', None)
    return (conv, fc) if slope == 0.1 else None


def _head_pair(model):
    """The (policy, value) heads csrc/hrl_heads.hip fuses: 32->2 conv + Linear(18, 9) and 32->1 conv +
    Linear(9, 1) on a 3x3 board (SimpleConv2dModel, tictactoe.py:59-60), or None."""
    pol = val = None
    for m in model.modules():
        spec = _board_head_spec(m)
        if spec is None:
            continue
        conv, fc = spec
        shape = (conv.in_channels, conv.out_channels, fc.in_features, fc.out_features)
        if shape == (32, 2, 18, 9):
            pol = m if pol is None else False
        elif shape == (32, 1, 9, 1):
            val = m if val is None else False
    return (pol, val) if pol and val else None


class _BoardHeadsFn(torch.autograd.Function):
    """Both heads of SimpleConv2dModel as csrc/hrl_heads.hip (one streaming pass over h each way)."""

    @staticmethod
    def forward(ctx, h, w1p, b1p, w1v, b1v, wp, wv):
        h = h.contiguous()
        N = h.shape[0]
        dev = h.device
        lib = _native.load()
        a_p = torch.empty(N, 18, device=dev, dtype=h.dtype)
        a_v = torch.empty(N, 9, device=dev, dtype=h.dtype)
        p = torch.empty(N, 9, device=dev, dtype=h.dtype)
        v = torch.empty(N, 1, device=dev, dtype=h.dtype)
        P = _native.ptr
        w1p, w1v, wp, wv = w1p.contiguous(), w1v.contiguous(), wp.contiguous(), wv.contiguous()
        _native.check(lib.hrl_heads_forward(P(h), N, P(w1p), P(b1p.contiguous()), P(w1v), P(b1v.contiguous()),
                                            P(wp), P(wv), None, None, P(a_p), P(a_v), P(p), P(v), 0,
                                            _native.stream_of(dev)), 'hrl_heads_forward')
        ctx.save_for_backward(h, w1p, w1v, wp, wv, a_p, a_v)
        ctx.biases = (b1p, b1v)
        return p, v

    @staticmethod
    def backward(ctx, dp, dv):
        h, w1p, w1v, wp, wv, a_p, a_v = ctx.saved_tensors
        N = h.shape[0]
        dev = h.device
        lib = _native.load()
        dp, dv = dp.contiguous(), dv.contiguous()
        dh = torch.empty_like(h)
        b1p, b1v = ctx.biases
        bufs = [_grad_buffer(t) for t in (w1p, b1p, w1v, b1v, wp, wv)]
        ws_bytes = lib.hrl_heads_workspace_bytes(N)
        ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
        P = _native.ptr

        def call(*dws):
            _native.check(lib.hrl_heads_backward(P(h), N, P(w1p), P(w1v), P(wp), P(wv), None, None, None, None,
                                                 P(a_p), P(a_v), P(dp), P(dv), None, P(dh), *(P(t) for t in dws),
                                                 P(ws), ws_bytes, _native.stream_of(dev)), 'hrl_heads_backward')
        df = _defer_folds(bufs, 6) if lib.hrl_heads_set_bwd_form(0) == 2 else None   # deferral needs form 2
        if df is not None:
            _heads_backward_deferred(lib, df, bufs, N, ws, call)
        else:
            call(*(b[0] for b in bufs))
        return (dh, *(_ret(b) for b in bufs))


class _FusedHeads(nn.Module):
    """The policy and value heads reading the same body output, as one _BoardHeadsFn (fuse_bn_relu's
    rewrite).  The heads are referenced, not registered; other inputs run the heads one by one."""

    def __init__(self, head_p, head_v):
        super().__init__()
        object.__setattr__(self, 'head_p', head_p)
        object.__setattr__(self, 'head_v', head_v)

    def forward(self, x):
        if not (x.is_cuda and x.dtype == torch.float32 and x.dim() == 4 and tuple(x.shape[1:]) == (32, 3, 3)
                and x.shape[0] > 0):
            return self.head_p(x), self.head_v(x)
        (cp, fp), (cv, fv) = _board_head_spec(self.head_p), _board_head_spec(self.head_v)
        params = (cp.weight, cp.bias, cv.weight, cv.bias, fp.weight, fv.weight)
        if torch.is_grad_enabled() and (x.requires_grad or any(t.requires_grad for t in params)):
            return _BoardHeadsFn.apply(x, *params)
        # inference (self-play, evaluation): outputs only, no saved activations
        x = x.contiguous()
        N = x.shape[0]
        p = torch.empty(N, 9, device=x.device, dtype=x.dtype)
        v = torch.empty(N, 1, device=x.device, dtype=x.dtype)
        P = _native.ptr
        _native.check(_native.load().hrl_heads_forward(P(x), N, P(cp.weight.contiguous()), P(cp.bias.contiguous()),
                                                       P(cv.weight.contiguous()), P(cv.bias.contiguous()),
                                                       P(fp.weight.contiguous()), P(fv.weight.contiguous()), None,
                                                       None, None, None, P(p), P(v), 0, _native.stream_of(x.device)),
                      'hrl_heads_forward')
        return p, v


def _fuse_heads(gm, heads):
    """Replace the two head calls on one activation with one _FusedHeads call; returns 0 or 1."""
    head_p, head_v = heads
    calls = {}
    for node in gm.graph.nodes:
        if node.op == 'call_module':
            m = gm.get_submodule(node.target)
            if m is head_p or m is head_v:
                calls.setdefault('p' if m is head_p else 'v', []).append(node)
    if len(calls.get('p', [])) != 1 or len(calls.get('v', [])) != 1:
        return 0
    np_, nv_ = calls['p'][0], calls['v'][0]
    if np_.args != nv_.args or len(np_.args) != 1 or np_.kwargs or nv_.kwargs:
        return 0
    gm.add_submodule('_hrl_heads', _FusedHeads(head_p, head_v))
    first = np_ if list(gm.graph.nodes).index(np_) < list(gm.graph.nodes).index(nv_) else nv_
    with gm.graph.inserting_before(first):
        call = gm.graph.call_module('_hrl_heads', np_.args)
        outs = [gm.graph.call_function(operator.getitem, (call, i)) for i in range(2)]
    np_.replace_all_uses_with(outs[0])
    nv_.replace_all_uses_with(outs[1])
    gm.graph.erase_node(np_)
    gm.graph.erase_node(nv_)
    return 1


class _StemConv(torch.autograd.Function):
    """3x3 conv of <= 3 observation planes into 32 channels on a 3x3 board (tictactoe.py:57):
    csrc/hrl_stem.hip (fp32 MFMA on the dense board matrix, B fragments held in registers)."""

    @staticmethod
    def forward(ctx, x, weight, bias):
        N, Cin = x.shape[0], x.shape[1]
        lib = _native.load()
        y = torch.empty(N, 32, 3, 3, device=x.device, dtype=x.dtype)
        w = weight.contiguous()
        b = bias.contiguous() if bias is not None else None
        _native.check(lib.hrl_stem_forward(_native.ptr(x), N, Cin, _native.ptr(w), _native.ptr(b), _native.ptr(y),
                                           _native.stream_of(x.device)), 'hrl_stem_forward')
        ctx.save_for_backward(x, w)
        ctx.params = (weight, bias)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        weight, bias = ctx.params
        N, Cin = x.shape[0], x.shape[1]
        lib = _native.load()
        ws_bytes = lib.hrl_stem_workspace_bytes(N)
        ws = torch.empty(ws_bytes, dtype=torch.uint8, device=x.device)
        bw = _grad_buffer(weight)
        bb = _grad_buffer(bias) if bias is not None else (None, False)
        df = _defer_folds([bw, bb]) if lib.hrl_stem_set_wgrad_form(0) == 2 else None   # deferral needs form 2
        dwp, dbp = (None, None) if df is not None else (bw[0], bb[0])
        _native.check(lib.hrl_stem_wgrad(_native.ptr(x), _native.ptr(dy.contiguous()), N, Cin, _native.ptr(dwp),
                                         _native.ptr(dbp), _native.ptr(ws), ws_bytes,
                                         _native.stream_of(x.device)), 'hrl_stem_wgrad')
        if df is not None:   # partial rows [dW (32, Cin, 3, 3) | db (32)] left in ws
            row = ctypes.c_int64(0)
            nparts = lib.hrl_stem_wgrad_partials(N, ctypes.byref(row))
            part = ws.view(torch.float32)
            nw = 32 * Cin * 9
            df.add(part, row.value, 0, nparts, bw[0], nw)
            if bb[0] is not None:
                df.add(part, row.value, nw, nparts, bb[0], 32)
            df.keep.append(ws)
        return None, _ret(bw), _ret(bb)


class _BoardWeight(torch.autograd.Function):
    """W -> W_board (csrc/hrl_board.hip); backward folds dW_board onto W (deterministic)."""

    @staticmethod
    def forward(ctx, weight, H, W):
        Cout, Cin, kh, kw = weight.shape
        w = weight.contiguous()
        out = torch.empty(Cin * H * W, Cout * H * W, dtype=w.dtype, device=w.device)
        _native.check(_native.load().hrl_board_weight(_native.ptr(w), Cout, Cin, kh, kw, H, W, _native.ptr(out),
                                                       _native.stream_of(w.device)), 'hrl_board_weight')
        ctx.geom = (Cout, Cin, kh, kw, H, W)
        ctx.weight = weight
        return out

    @staticmethod
    def backward(ctx, grad):
        Cout, Cin, kh, kw, H, W = ctx.geom
        g = grad.contiguous()
        buf = _grad_buffer(ctx.weight)
        _native.check(_native.load().hrl_board_fold(_native.ptr(g), Cout, Cin, kh, kw, H, W, _native.ptr(buf[0]),
                                                     _native.stream_of(g.device)), 'hrl_board_fold')
        return _ret(buf), None, None


class _BoardBias(torch.autograd.Function):
    """b -> b_board[co*HW + q] = b[co]; backward sums over the board cells."""

    @staticmethod
    def forward(ctx, bias, HW):
        out = torch.empty(bias.shape[0] * HW, dtype=bias.dtype, device=bias.device)
        _native.check(_native.load().hrl_board_bias(_native.ptr(bias.contiguous()), bias.shape[0], HW,
                                                     _native.ptr(out), _native.stream_of(bias.device)), 'hrl_board_bias')
        ctx.shape = (bias.shape[0], HW)
        ctx.bias = bias
        return out

    @staticmethod
    def backward(ctx, grad):
        Cout, HW = ctx.shape
        g = grad.contiguous()
        buf = _grad_buffer(ctx.bias)
        _native.check(_native.load().hrl_board_bias_fold(_native.ptr(g), Cout, HW, _native.ptr(buf[0]),
                                                          _native.stream_of(g.device)), 'hrl_board_bias_fold')
        return _ret(buf), None


class _LSTMGates(torch.autograd.Function):
    """ConvLSTM cell gates (csrc/hrl_lstm.hip): z = zx + zh -> (h', c'), saved gate activations."""

    @staticmethod
    def forward(ctx, zx, zh, c, save=True, bias=None, bias_rows=1, out=None):
        ctx.set_materialize_grads(False)   # a cell whose outputs reach no loss stays out of backward
        N, G, Hh, Ww = zh.shape
        H, HW = G // 4, Hh * Ww
        zh = zh.contiguous()
        c = c.contiguous()
        if zx is not None and (zx.shape != zh.shape or zx.stride()[1:] != zh.stride()[1:]):
            zx = zx.contiguous()
        if out is not None:   # inference: given (h', c') buffers, possibly c itself (same-index read then write)
            h_out, c_out = out
            assert not save and h_out.shape == c.shape and c_out.shape == c.shape
            assert h_out.is_contiguous() and c_out.is_contiguous()
        else:
            h_out = torch.empty_like(c)
            c_out = torch.empty_like(c)
        # inference (self-play) saves nothing for a backward: the kernel skips the 4 gate streams
        gates = torch.empty_like(zh) if save else None
        lib = _native.load()
        if bias is not None:
            assert zx is not None and not save and bias.is_contiguous() and bias.numel() == bias_rows * G
        _native.check(lib.hrl_lstm_gates_forward(_native.ptr(zx), 0 if zx is None else zx.stride(0), _native.ptr(zh),
                                                 _native.ptr(c), N, H, HW, _native.ptr(bias), bias_rows,
                                                 _native.ptr(h_out), _native.ptr(c_out), _native.ptr(gates),
                                                 _native.stream_of(zh.device)),
                      'hrl_lstm_gates_forward')
        ctx.save_for_backward(gates, c, c_out)
        ctx.has_zx = zx is not None
        return h_out, c_out

    @staticmethod
    def backward(ctx, dh, dc_out):
        if dh is None and dc_out is None:
            return None, None, None, None, None, None, None
        gates, c, c_out = ctx.saved_tensors
        N, G, Hh, Ww = gates.shape
        dz = torch.empty_like(gates)
        dc = torch.empty_like(c)
        dh = None if dh is None else dh.contiguous()
        dc_out = None if dc_out is None else dc_out.contiguous()
        _native.check(_native.load().hrl_lstm_gates_backward(
            _native.ptr(gates), _native.ptr(c), _native.ptr(c_out), _native.ptr(dh), _native.ptr(dc_out),
            N, G // 4, Hh * Ww, _native.ptr(dz), _native.ptr(dc), _native.stream_of(gates.device)),
            'hrl_lstm_gates_backward')
        return (dz if ctx.has_zx else None), dz, dc, None, None, None, None


def lstm_gates(zx, zh, c, bias=None, bias_rows=1, out=None):
    """(h', c') of a ConvLSTM cell from its gate pre-activations zx + zh (i, f, o, g order).

    ``zx`` (may be None) can be a channel slice of a wider tensor; the HIP
    kernels run forward and backward in one launch each.  ``bias`` (inference
    only): the x half's convolution bias, (bias_rows, 4H) for rows n % bias_rows,
    added as (zx + bias) + zh.
    """
    if not zh.is_cuda:
        raise RuntimeError('lstm_gates runs on the HIP device only (no CPU fallback)')
    save = torch.is_grad_enabled() and any(t is not None and t.requires_grad for t in (zx, zh, c))
    if (bias is not None or out is not None) and save:
        raise ValueError('lstm_gates: the folded bias and output buffers are inference-only forms')
    return _LSTMGates.apply(zx, zh, c, save, bias, bias_rows, out)


def _live(xs):
    return [k for k, x in enumerate(xs) if x is not None]


def _rows_view(t, lead):
    """t as (rows, features) with unit-stride features (rows may be any stride apart: a channel slice of a wider
    gradient), flattening the first `lead` dims into rows; a contiguous copy only when that is not possible."""
    rows = t.flatten(lead) if t.dim() > lead else t.unsqueeze(-1)
    if rows.stride(-1) != 1:
        rows = rows.contiguous()
    rows = rows.reshape(-1, rows.shape[-1]) if lead > 1 else rows
    if rows.stride(-1) != 1 or (rows.shape[0] > 1 and rows.stride(0) < rows.shape[-1]):
        rows = rows.contiguous()
    return rows


class _HiddenGather(torch.autograd.Function):
    """Per-step recurrent input (csrc/hrl_hidden.hip, train.py:157-164), one launch for every state tensor.

    apply(m, summed, B, P, *H): H[l] is (B, P, *shape_l); returns sum_p H[l] * m (summed, (B, *shape_l))
    or H[l] * m as (B*P, *shape_l), then H itself again (views) for the step's _HiddenUpdate: the state then has
    one autograd consumer, and the backward adds the update's keep-path gradient into its own launch
    (hrl_hidden_gather_backward_add) instead of autograd adding the two.  Tensors whose gradients are None get
    None back.
    """

    @staticmethod
    def forward(ctx, m, summed, B, P, *H):
        ctx.set_materialize_grads(False)   # a state tensor without a gradient stays None (pruned)
        H = [h.contiguous() for h in H]
        rows = B if summed else B * P
        outs = [torch.empty(rows, *h.shape[2:], dtype=h.dtype, device=h.device) for h in H]
        F = [h[0, 0].numel() for h in H]
        _native.check(_native.load().hrl_hidden_gather(
            _native.ptr_array(H), _native.ptr(m), B, P, len(H), _native.i64_array(F), int(summed),
            _native.ptr_array(outs), _native.stream_of(m.device)), 'hrl_hidden_gather')
        ctx.save_for_backward(m)
        ctx.meta = (summed, B, P, [tuple(h.shape) for h in H])
        return (*outs, *[h.view_as(h) for h in H])

    @staticmethod
    def backward(ctx, *grads):
        (m,) = ctx.saved_tensors
        summed, B, P, shapes = ctx.meta
        n = len(shapes)
        gout, galias = grads[:n], grads[n:]
        dH = [None] * n
        live = [k for k in range(n) if gout[k] is not None]
        for k in range(n):   # only the update's gradient: it is the state's
            if gout[k] is None and galias[k] is not None:
                dH[k] = galias[k]
        if live:
            g = [gout[k].contiguous() for k in live]
            F = [int(torch.Size(shapes[k][2:]).numel()) for k in live]
            add = [None if galias[k] is None else _rows_view(galias[k], 2) for k in live]
            d = [torch.empty(shapes[k], dtype=m.dtype, device=m.device) for k in live]
            _native.check(_native.load().hrl_hidden_gather_backward_add(
                _native.ptr_array(g), _native.ptr(m), B, P, len(live), _native.i64_array(F), int(summed),
                _native.ptr_array(add) if any(a is not None for a in add) else None,
                _native.i64_array([a.stride(-2) if a is not None else f for a, f in zip(add, F)]),
                _native.ptr_array(d), _native.stream_of(m.device)), 'hrl_hidden_gather_backward_add')
            for k, t in zip(live, d):
                dH[k] = t
        return (None, None, None, None, *dH)


def masked_rows_copy_(dst, src, mask):
    """dst[l][e] = src[l][e] where mask[e], for every tensor pair, in ONE launch (csrc/hrl_selfplay.hip):
    self-play's recurrent state advance (generation.py:38-41, only the mover's state moves).  dst[l], src[l]:
    (E, *shape) fp32 with contiguous rows (any row stride, e.g. the mover's slice h[:, p] of an (E, P, ...)
    state or a channel slice of a stacked one); mask: (E,) bool.  Exactly torch.where(mask, src, dst)."""
    E = mask.shape[0]
    assert mask.dtype == torch.bool and mask.is_contiguous() and len(dst) == len(src)
    F = []
    for d, x in zip(dst, src):
        assert d.is_cuda and d.dtype == torch.float32 and x.dtype == torch.float32
        assert d.shape == x.shape and d.shape[0] == E and d[0].is_contiguous() and x[0].is_contiguous()
        F.append(d[0].numel())
    _native.check(_native.load().hrl_masked_rows_copy(
        len(dst), _native.ptr_array(dst), _native.i64_array([d.stride(0) for d in dst]), _native.ptr_array(src),
        _native.i64_array([x.stride(0) for x in src]), _native.i64_array(F), _native.ptr(mask), E,
        _native.stream_of(mask.device)), 'hrl_masked_rows_copy')


class _HiddenUpdate(torch.autograd.Function):
    """New state H[l] * (1 - m) + nh[l] * m (csrc/hrl_hidden.hip, train.py:167-174), one launch for all.

    apply(m, B, P, Pn, n, out_k, *H, *nh): H[l] (B, P, *shape_l), nh[l] (B*Pn, *shape_l).  out_k >= 0: nh[out_k]
    is also the step's output (a recurrent net's h_last): it is returned again (a view) after the new states, so
    its consumers' gradient comes back here and is added into dnh[out_k] in the adjoint's launch
    (hrl_hidden_update_backward_add) instead of by autograd.  Tensors whose output gradient is None get None back
    (their producers are pruned, as with the torch ops).
    """

    @staticmethod
    def forward(ctx, m, B, P, Pn, n, out_k, *tensors):
        ctx.set_materialize_grads(False)   # a state tensor without a gradient stays None (pruned)
        H = [h.contiguous() for h in tensors[:n]]
        nh = [x.contiguous() for x in tensors[n:]]
        outs = [torch.empty_like(h) for h in H]
        F = [h[0, 0].numel() for h in H]
        _native.check(_native.load().hrl_hidden_update(
            _native.ptr_array(H), _native.ptr_array(nh), Pn, _native.ptr(m), B, P, n, _native.i64_array(F),
            _native.ptr_array(outs), _native.stream_of(m.device)), 'hrl_hidden_update')
        ctx.save_for_backward(m)
        ctx.meta = (B, P, Pn, n, out_k, [tuple(h.shape) for h in H], [tuple(x.shape) for x in nh])
        if out_k >= 0:
            return (*outs, tensors[n + out_k].view_as(tensors[n + out_k]))
        return tuple(outs)

    @staticmethod
    def backward(ctx, *douts):
        (m,) = ctx.saved_tensors
        B, P, Pn, n, out_k, h_shapes, nh_shapes = ctx.meta
        dout = douts[:n]
        gk = douts[n] if out_k >= 0 else None
        live = _live(dout)
        dH, dnh = [None] * n, [None] * n
        if gk is not None and dout[out_k] is None:
            dnh[out_k] = gk
        if live:
            g = [dout[k].contiguous() for k in live]
            # the step output's gradient: typically a channel slice of the heads' input gradient, read in place
            add = [_rows_view(gk, 1) if (k == out_k and gk is not None) else None for k in live]
            a = [torch.empty(h_shapes[k], dtype=m.dtype, device=m.device) for k in live]
            b = [torch.empty(nh_shapes[k], dtype=m.dtype, device=m.device) for k in live]
            F = [int(torch.Size(h_shapes[k][2:]).numel()) for k in live]
            _native.check(_native.load().hrl_hidden_update_backward_add(
                _native.ptr_array(g), _native.ptr(m), B, P, Pn, len(live), _native.i64_array(F),
                _native.ptr_array(add) if any(x is not None for x in add) else None,
                _native.i64_array([x.stride(-2) if x is not None else f for x, f in zip(add, F)]),
                _native.ptr_array(a), _native.ptr_array(b), _native.stream_of(m.device)),
                'hrl_hidden_update_backward_add')
            for k, x, y in zip(live, a, b):
                dH[k], dnh[k] = x, y
        return (None, None, None, None, None, None, *dH, *dnh)


class _HiddenUpdateGather(torch.autograd.Function):
    """Step t's _HiddenUpdate fused with step t+1's _HiddenGather (round 5): one launch each way
    (hrl_hidden_update_gather[_backward]) where the unroll ran two, bit for bit the same values.

    apply(m, m_next, summed, B, P, Pn, n, out_k, *H, *nh) -> (*gathered (step t+1's input), *state (views of the
    new state, for step t+1's update), [nh[out_k] again if out_k >= 0: the step's output])."""

    @staticmethod
    def forward(ctx, m, m_next, summed, B, P, Pn, n, out_k, *tensors):
        ctx.set_materialize_grads(False)
        H = [h.contiguous() for h in tensors[:n]]
        nh = [x.contiguous() for x in tensors[n:]]
        outs = [torch.empty_like(h) for h in H]
        rows = B if summed else B * P
        gath = [torch.empty(rows, *h.shape[2:], dtype=h.dtype, device=h.device) for h in H]
        F = [h[0, 0].numel() for h in H]
        _native.check(_native.load().hrl_hidden_update_gather(
            _native.ptr_array(H), _native.ptr_array(nh), Pn, _native.ptr(m), _native.ptr(m_next), B, P, n,
            _native.i64_array(F), int(summed), _native.ptr_array(outs), _native.ptr_array(gath),
            _native.stream_of(m.device)), 'hrl_hidden_update_gather')
        ctx.save_for_backward(m, m_next)
        ctx.meta = (summed, B, P, Pn, n, out_k, [tuple(h.shape) for h in H], [tuple(x.shape) for x in nh])
        res = (*gath, *[o.view_as(o) for o in outs])
        if out_k >= 0:
            res = res + (tensors[n + out_k].view_as(tensors[n + out_k]),)
        return res

    @staticmethod
    def backward(ctx, *grads):
        m, m_next = ctx.saved_tensors
        summed, B, P, Pn, n, out_k, h_shapes, nh_shapes = ctx.meta
        ggath, gstate = grads[:n], grads[n:2 * n]
        gk = grads[2 * n] if out_k >= 0 else None
        dH, dnh = [None] * n, [None] * n
        live = [k for k in range(n) if ggath[k] is not None or gstate[k] is not None]
        if gk is not None and out_k not in live:
            dnh[out_k] = gk
        if live:
            g = [None if ggath[k] is None else ggath[k].contiguous() for k in live]
            st = [None if gstate[k] is None else _rows_view(gstate[k], 2) for k in live]
            add = [_rows_view(gk, 1) if (k == out_k and gk is not None) else None for k in live]
            F = [int(torch.Size(h_shapes[k][2:]).numel()) for k in live]
            a = [torch.empty(h_shapes[k], dtype=m.dtype, device=m.device) for k in live]
            b = [torch.empty(nh_shapes[k], dtype=m.dtype, device=m.device) for k in live]
            _native.check(_native.load().hrl_hidden_update_gather_backward(
                _native.ptr_array(g), _native.ptr(m), _native.ptr(m_next), B, P, Pn, len(live), _native.i64_array(F),
                int(summed), _native.ptr_array(st) if any(x is not None for x in st) else None,
                _native.i64_array([x.stride(-2) if x is not None else f for x, f in zip(st, F)]),
                _native.ptr_array(add) if any(x is not None for x in add) else None,
                _native.i64_array([x.stride(-2) if x is not None else f for x, f in zip(add, F)]),
                _native.ptr_array(a), _native.ptr_array(b), _native.stream_of(m.device)),
                'hrl_hidden_update_gather_backward')
            for k, x, y in zip(live, a, b):
                dH[k], dnh[k] = x, y
        return (None, None, None, None, None, None, None, None, *dH, *dnh)


def _board_conv_ok(m):
    k = m.kernel_size
    return (m.stride == (1, 1) and m.dilation == (1, 1) and m.groups == 1 and m.padding_mode == 'zeros'
            and isinstance(m.padding, tuple) and m.padding == (k[0] // 2, k[1] // 2) and k[0] % 2 == 1
            and k[1] % 2 == 1)


class BatchNorm2d(nn.BatchNorm2d):
    """nn.BatchNorm2d whose training-mode CUDA path runs csrc/hrl_bn.hip.

    ``fused_relu`` (set by ``fuse_bn_relu``) makes the module apply the ReLU
    that followed it in the net's forward: inside the kernels on the HIP path,
    as ``F.relu`` otherwise.
    """

    fused_relu = False

    def forward(self, x):
        row = x.shape[1] * x.shape[2] * x.shape[3] if x.dim() == 4 else 0
        shape_ok = (x.is_cuda and x.dtype == torch.float32 and x.dim() == 4
                    and x.shape[0] > 0 and (row <= _MAX_ROW_SCALAR or (row % 4 == 0 and row <= _MAX_ROW)))
        if shape_ok and not self.training and self.track_running_stats and self.running_mean is not None:
            return batch_norm_eval(x, self.weight, self.bias, self.running_mean, self.running_var, self.eps,
                                   self.fused_relu)
        use_hip = shape_ok and self.training
        if not use_hip:
            y = super().forward(x)
            return torch.relu(y) if self.fused_relu else y
        self._check_input_dim(x)
        momentum = 0.0 if self.momentum is None else self.momentum
        if self.track_running_stats and self.num_batches_tracked is not None:
            self.num_batches_tracked.add_(1)
            if self.momentum is None:  # cumulative moving average
                momentum = 1.0 / float(self.num_batches_tracked.item())
        rm = self.running_mean if self.track_running_stats else None
        rv = self.running_var if self.track_running_stats else None
        return batch_norm_train(x, self.weight, self.bias, rm, rv, momentum, self.eps, self.fused_relu)


def accelerate(model):
    """Swap HIP-backed layers into ``model`` in place (same parameters and state_dict); returns it.

    BoardConv2d checks the board size of every input and runs the plain
    convolution on boards larger than BOARD_MAX_CELLS cells.
    """
    for name, child in list(model.named_children()):
        if type(child) is nn.Conv2d and _board_conv_ok(child):
            new = BoardConv2d(child.in_channels, child.out_channels, child.kernel_size, stride=1,
                              padding=child.padding, bias=child.bias is not None,
                              device=child.weight.device, dtype=child.weight.dtype)
            new.weight = child.weight
            if child.bias is not None:
                new.bias = child.bias
            new.train(child.training)
            setattr(model, name, new)
        elif type(child) is nn.Linear:
            new = Linear(child.in_features, child.out_features, bias=child.bias is not None,
                         device=child.weight.device, dtype=child.weight.dtype)
            new.weight = child.weight
            if child.bias is not None:
                new.bias = child.bias
            new.train(child.training)
            setattr(model, name, new)
        elif type(child) is nn.BatchNorm2d:
            new = BatchNorm2d(child.num_features, eps=child.eps, momentum=child.momentum,
                              affine=child.affine, track_running_stats=child.track_running_stats)
            new.weight, new.bias = child.weight, child.bias
            if child.track_running_stats:
                new.running_mean, new.running_var = child.running_mean, child.running_var
                new.num_batches_tracked = child.num_batches_tracked
            new.train(child.training)
            setattr(model, name, new)
        else:
            accelerate(child)
    if hasattr(model, 'use_hip'):   # modules with their own HIP fast path (e.g. envs.geister.DRC)
        model.use_hip = True
    return model


class _MultiBoardConv(nn.Module):
    """Sibling BoardConv2d layers reading the same activation, as ONE GEMM.

    The env nets' heads (tictactoe.py:35-49, e.g. head_p / head_v) each start
    with a 1x1 conv of the same body output; concatenating their board
    matrices reads the activation once and, in backward, produces the summed
    input gradient in one GEMM instead of two GEMMs and an add.  The convs are
    referenced, not registered, so parameters and state_dict are unchanged.
    """

    def __init__(self, convs):
        super().__init__()
        object.__setattr__(self, 'convs', list(convs))

    def forward(self, x):
        convs = self.convs
        if not (x.is_cuda and x.dim() == 4 and x.dtype == torch.float32
                and x.shape[2] * x.shape[3] <= BOARD_MAX_CELLS):
            return tuple(c(x) for c in convs)
        N, Cin, H, W = x.shape
        HW = H * W
        wb = torch.cat([_BoardWeight.apply(c.weight, H, W) for c in convs], dim=1)
        parts = [_BoardBias.apply(c.bias, HW) if c.bias is not None else c.weight.new_zeros(c.out_channels * HW)
                 for c in convs]
        y = _RowMatmul.apply(x.reshape(N, Cin * HW), wb, torch.cat(parts))
        outs, off = [], 0
        for c in convs:
            n = c.out_channels * HW
            outs.append(y[:, off:off + n].reshape(N, c.out_channels, H, W))
            off += n
        return tuple(outs)


_UNIT = {}

# True: the chain's BatchNorm finalizes run in the prologue of the kernel that consumes them
# (hrl_conv3x3_forward_bnfold, hrl_conv3x3_block_backward_bnfold: five launches fewer per TicTacToe step,
# bit-identical).  Off by default: every workgroup re-reading the 128 KB of partial rows cost more than the five
# launches it saves (+14..25 us per step, profiles/r06_fold_ab.txt); tests keep both paths equal.
FOLD_BN = False


def _unit_coefs(dev):
    """(alpha, beta) = (1, 0) per channel: the stem ReLU in front of a chain as an identity BN + ReLU (cached)."""
    u = _UNIT.get(dev)
    if u is None:
        u = _UNIT[dev] = torch.stack([torch.ones(32, device=dev), torch.zeros(32, device=dev)])
    return u


def _chain_forward(h0, meta, relu_in, params, apply_out=True):
    """Forward of a conv -> BN -> ReLU chain (see _BoardChain): returns (out | None, ys, coefs, unit)."""
    lib = _native.load()
    M = h0.shape[0]
    dev = h0.device
    stream = _native.stream_of(dev)
    P = _native.ptr
    ws_bytes = lib.hrl_conv3x3_workspace_bytes(M)
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
    nblk = lib.hrl_conv3x3_stats_blocks(M)
    # conv i's statistics rows alternate between two buffers: conv i+1 reads them in its prologue (FOLD_BN) while
    # its own epilogue writes the other
    parts = torch.empty(2, nblk * 32 * 2, dtype=torch.float64, device=dev)
    fold = FOLD_BN
    unit = _unit_coefs(dev) if relu_in else None
    x = h0
    a_prev, b_prev = (unit[0], unit[1]) if relu_in else (None, None)
    ys, coefs = [], []
    # every conv's forward and input-gradient weight layouts in one launch (the backward reuses them)
    weights = [params[3 * i].contiguous() for i in range(len(meta))]
    packed = torch.empty(len(weights), 2, 9216, dtype=torch.float32, device=dev)
    for k in range(0, len(weights), 8):       # hrl_conv3x3_pack_n takes up to 8 weights per launch
        _native.check(lib.hrl_conv3x3_pack_n(_native.ptr_array(weights[k:k + 8]), len(weights[k:k + 8]),
                                             P(packed[k]), stream), 'hrl_conv3x3_pack_n')
    n = len(meta)
    for i, (rm, rv, momentum, eps) in enumerate(meta):
        w, gamma, beta = params[3 * i:3 * i + 3]
        y = torch.empty_like(h0)
        part = parts[i % 2]
        if fold and i > 0:
            # BN_{i-1}'s finalize runs in conv i's prologue and fills coefs[i-1] (hrl_conv3x3_forward_bnfold)
            prm, prv, pmom, peps = meta[i - 1]
            pc = coefs[i - 1]
            _native.check(lib.hrl_conv3x3_forward_bnfold(
                P(x), M, P(parts[(i - 1) % 2]), nblk, P(params[3 * i - 2]), P(params[3 * i - 1]), P(prm), P(prv),
                float(pmom), float(peps), P(pc[0]), P(pc[1]), P(pc[2]), P(pc[3]), P(packed[i, 0]), P(y), P(part),
                P(ws), ws_bytes, stream), 'hrl_conv3x3_forward_bnfold')
        else:
            _native.check(lib.hrl_conv3x3_forward_ex(P(x), M, P(a_prev), P(b_prev), P(packed[i, 0]), None, 2, P(y),
                                                     1, None, None, None, None, P(part), P(ws), ws_bytes, stream),
                          'hrl_conv3x3_forward_ex')
        coef = torch.empty(4, 32, dtype=torch.float32, device=dev)   # mean, invstd, alpha, beta
        if not fold or i == n - 1:
            _native.check(lib.hrl_bn_finalize_stats(P(part), nblk, 32, M * 9, P(gamma), P(beta), P(rm), P(rv),
                                                    float(momentum), float(eps), P(coef[0]), P(coef[1]),
                                                    P(coef[2]), P(coef[3]), stream), 'hrl_bn_finalize_stats')
        ys.append(y)
        coefs.append(coef)
        x, a_prev, b_prev = y, coef[2], coef[3]
    out = None
    if apply_out:
        out = torch.empty_like(h0)
        _native.check(lib.hrl_bn_apply(P(x), M, 32, 9, P(a_prev), P(b_prev), 1, P(out), stream), 'hrl_bn_apply')
    return out, ys, coefs, unit, packed


def _chain_backward(h0, ys, coefs, unit, params, relu_in, g, need_input_grad, packed, part_in=None, nblk_in=0):
    """Backward of the chain from g = dL/d(chain output); with part_in the last BN's backward sums were already
    formed by the consumer (fused heads).  Returns (dL/dh0 | None, parameter gradients)."""
    lib = _native.load()
    n = len(ys)
    M = h0.shape[0]
    dev = h0.device
    stream = _native.stream_of(dev)
    P = _native.ptr
    ws_bytes = lib.hrl_conv3x3_workspace_bytes(M)
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
    bn_ws_bytes = lib.hrl_bn_workspace_bytes(M, 32, 9)
    bn_ws = torch.empty(bn_ws_bytes, dtype=torch.uint8, device=dev)
    # the block backward's epilogue-2 sum rows (its workgroups) or the input-gradient conv's
    nblk = max(lib.hrl_conv3x3_block_sum_blocks(M), lib.hrl_conv3x3_stats_blocks(M))
    # block i writes BN_{i-1}'s sums into parts[i % 2] while (FOLD_BN) its prologue reads BN_i's from the other
    parts = torch.empty(2, nblk * 32 * 2, dtype=torch.float64, device=dev)
    fold = FOLD_BN
    g = g.contiguous()
    grads = [None] * (3 * n)
    sums, sums_n = (part_in, nblk_in) if part_in is not None else (None, 0)   # BN_i's backward sums, if formed
    for i in reversed(range(n)):
        w, gamma, beta = params[3 * i:3 * i + 3]
        mean, invstd = coefs[i][0], coefs[i][1]
        bw, bgam, bbet = _grad_buffer(w), _grad_buffer(gamma), _grad_buffer(beta)
        dgam, dbet = bgam[0], bbet[0]
        if i == 0:
            x, a, b = h0, (unit[0] if unit is not None else None), (unit[1] if unit is not None else None)
        else:
            x, a, b = ys[i - 1], coefs[i - 1][2], coefs[i - 1][3]
        dw = bw[0]
        part = parts[i % 2]
        if sums is not None:
            # BN_i's backward sums are formed (by the consumer or block i+1's input-gradient epilogue): the block's
            # BN backward apply, weight gradient and input gradient run as ONE launch (conv3x3_block_bwd_kernel),
            # with BN_i's finalize in its prologue (FOLD_BN, hrl_conv3x3_block_backward_bnfold)
            kg = torch.empty(2, 32, dtype=torch.float32, device=dev)
            if not fold:
                _native.check(lib.hrl_bn_finalize_backward(P(sums), sums_n, 32, M * 9, P(gamma), P(invstd),
                                                           P(dgam), P(dbet), P(kg[0]), P(kg[1]), stream),
                              'hrl_bn_finalize_backward')
            gin, epi, ep = None, 0, (None, None, None)
            if i > 0:
                gin, epi, ep = torch.empty_like(h0), 2, (coefs[i - 1][0], coefs[i - 1][2], coefs[i - 1][3])
            elif need_input_grad:
                gin, epi = torch.empty_like(h0), (3 if relu_in else 0)
            df = _defer_folds([bw])
            wsb = ws if df is None else torch.empty(ws_bytes, dtype=torch.uint8, device=dev)   # partials live on
            ev = _block_timing_start()
            if fold:
                _native.check(lib.hrl_conv3x3_block_backward_bnfold(
                    P(g), P(ys[i]), M, P(gamma), P(beta), P(mean), P(invstd), P(sums), sums_n, P(dgam), P(dbet),
                    P(kg[0]), P(kg[1]), P(x), P(a), P(b), P(packed[i, 1]), None if df is not None else P(dw), P(gin),
                    epi, P(ep[0]), P(ep[1]), P(ep[2]), P(part) if i > 0 else None, P(wsb), ws_bytes, stream),
                    'hrl_conv3x3_block_backward_bnfold')
            else:
                _native.check(lib.hrl_conv3x3_block_backward(
                    P(g), P(ys[i]), M, P(gamma), P(beta), P(mean), P(invstd), P(kg[0]), P(kg[1]), P(x), P(a), P(b),
                    P(packed[i, 1]), None if df is not None else P(dw), P(gin), epi, P(ep[0]), P(ep[1]), P(ep[2]),
                    P(part) if i > 0 else None, P(wsb), ws_bytes, stream), 'hrl_conv3x3_block_backward')
            _block_timing_end(ev)
            if df is not None:   # [block][tap][ci][co] partial rows -> dW (co, ci, kh, kw): fold mode 1
                off = ctypes.c_int64(0)
                nparts = lib.hrl_conv3x3_wgrad_partials(M, ctypes.byref(off))
                df.add(wsb[off.value:].view(torch.float32), 9216, 0, nparts, dw, 9216, mode=1)
                df.keep.append(wsb)
            grads[3 * i:3 * i + 3] = [_ret(bw), _ret(bgam), _ret(bbet)]
            g = gin
            if i > 0:   # read by the next block's finalize before its launch rewrites part
                sums, sums_n = part, lib.hrl_conv3x3_block_sum_blocks(M)
            continue
        dy = torch.empty_like(h0)
        _native.check(lib.hrl_bn_backward(P(ys[i]), P(g), M, 32, 9, P(gamma), P(beta), P(mean), P(invstd),
                                          1, P(dy), P(dgam), P(dbet), P(bn_ws), bn_ws_bytes, stream),
                      'hrl_bn_backward')
        _native.check(lib.hrl_conv3x3_wgrad_ex(P(x), P(a), P(b), P(dy), M, P(dw), P(ws), ws_bytes, stream),
                      'hrl_conv3x3_wgrad_ex')
        grads[3 * i:3 * i + 3] = [_ret(bw), _ret(bgam), _ret(bbet)]
        if i > 0:   # dL/dh_i, and BN_{i-1}'s backward sums in the same launch
            g = torch.empty_like(h0)
            _native.check(lib.hrl_conv3x3_forward_ex(P(dy), M, None, None, P(packed[i, 1]), None, 3, P(g), 2,
                                                     P(ys[i - 1]),
                                                     P(coefs[i - 1][0]), P(coefs[i - 1][2]),
                                                     P(coefs[i - 1][3]), P(part), P(ws), ws_bytes, stream),
                          'hrl_conv3x3_forward_ex(flip, bn sums)')
            sums, sums_n = part, lib.hrl_conv3x3_stats_blocks(M)
        elif need_input_grad:
            g = torch.empty_like(h0)
            _native.check(lib.hrl_conv3x3_forward_ex(P(dy), M, None, None, P(packed[i, 1]), None, 3, P(g),
                                                     3 if relu_in else 0, P(h0) if relu_in else None,
                                                     None, None, None, None, P(ws), ws_bytes, stream),
                          'hrl_conv3x3_forward_ex(flip)')
        else:
            g = None
    return g, grads


class _BoardChain(torch.autograd.Function):
    """[relu ->] [3x3 conv 32->32 (no bias) -> BatchNorm (training) -> ReLU] x n on 3x3 boards.

    The TicTacToe body (tictactoe.py:57-65; ``relu_in``: the stem's ReLU in
    front of it, tictactoe.py:62).  Fused around the MFMA conv
    (csrc/hrl_conv.hip, conv3x3_kernel<PRO, EPI>):
      forward   conv_i's epilogue emits the BatchNorm statistics of its output
                y_i; conv_{i+1} (and in backward the weight-gradient kernel)
                applies BN_i + ReLU to y_i as it reads it;
      backward  the input-gradient launch of conv_{i+1} also produces BN_i's
                backward sums from y_i in its epilogue, so only BN_{n-1}
                needs the separate reduce pass; with ``relu_in`` the first
                input-gradient launch applies the stem ReLU's mask.
    Only the raw conv outputs y_i and the chain's output reach HBM.
    """

    @staticmethod
    def forward(ctx, h0, meta, relu_in, *params):
        h0 = h0.contiguous()
        out, ys, coefs, unit, packed = _chain_forward(h0, meta, relu_in, params)
        ctx.save_for_backward(h0, *ys, *coefs, packed, *params)
        ctx.n = len(meta)
        ctx.relu_in = relu_in
        return out

    @staticmethod
    def backward(ctx, g):
        n = ctx.n
        t = ctx.saved_tensors
        h0, ys, coefs, packed, params = t[0], list(t[1:1 + n]), list(t[1 + n:1 + 2 * n]), t[1 + 2 * n], t[2 + 2 * n:]
        unit = _unit_coefs(h0.device) if ctx.relu_in else None
        g_in, grads = _chain_backward(h0, ys, coefs, unit, params, ctx.relu_in, g, ctx.needs_input_grad[0], packed)
        return (g_in, None, None, *grads)


class _ChainHeadsFn(torch.autograd.Function):
    """The TicTacToe body chain and both heads as one Function: the chain's last BN + ReLU is applied by the
    heads kernels as they read its raw input (csrc/hrl_heads.hip BnIn), so the body output never reaches HBM;
    the heads backward also forms that BN's backward sums, so the chain backward needs no reduce pass."""

    @staticmethod
    def forward(ctx, h0, meta, relu_in, tanh_v, w1p, b1p, w1v, b1v, wp, wv, *params):
        h0 = h0.contiguous()
        _, ys, coefs, unit, packed = _chain_forward(h0, meta, relu_in, params, apply_out=False)
        y, coef = ys[-1], coefs[-1]
        N = h0.shape[0]
        dev = h0.device
        lib = _native.load()
        a_p = torch.empty(N, 18, device=dev, dtype=h0.dtype)
        a_v = torch.empty(N, 9, device=dev, dtype=h0.dtype)
        p = torch.empty(N, 9, device=dev, dtype=h0.dtype)
        v = torch.empty(N, 1, device=dev, dtype=h0.dtype)
        P = _native.ptr
        w1p, w1v, wp, wv = w1p.contiguous(), w1v.contiguous(), wp.contiguous(), wv.contiguous()
        _native.check(lib.hrl_heads_forward(P(y), N, P(w1p), P(b1p.contiguous()), P(w1v), P(b1v.contiguous()),
                                            P(wp), P(wv), P(coef[2]), P(coef[3]), P(a_p), P(a_v), P(p), P(v),
                                            int(tanh_v), _native.stream_of(dev)), 'hrl_heads_forward(bn)')
        ctx.save_for_backward(h0, *ys, *coefs, a_p, a_v, w1p, w1v, wp, wv, packed, v, *params)
        ctx.tanh_v = tanh_v
        ctx.biases = (b1p, b1v)
        ctx.n = len(meta)
        ctx.relu_in = relu_in
        return p, v

    @staticmethod
    def backward(ctx, dp, dv):
        n = ctx.n
        t = ctx.saved_tensors
        h0, ys, coefs = t[0], list(t[1:1 + n]), list(t[1 + n:1 + 2 * n])
        a_p, a_v, w1p, w1v, wp, wv, packed, v = t[1 + 2 * n:9 + 2 * n]
        params = t[9 + 2 * n:]
        b1p, b1v = ctx.biases
        N = h0.shape[0]
        dev = h0.device
        lib = _native.load()
        P = _native.ptr
        y, coef = ys[-1], coefs[-1]
        dp, dv = dp.contiguous(), dv.contiguous()
        dh = torch.empty_like(h0)
        hbufs = [_grad_buffer(x) for x in (w1p, b1p, w1v, b1v, wp, wv)]
        ws_bytes = lib.hrl_heads_workspace_bytes(N)
        ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
        nparts = lib.hrl_heads_bn_parts(N)
        bn_part = torch.empty(nparts * 64, dtype=torch.float64, device=dev)
        def call(*dws):
            _native.check(lib.hrl_heads_backward(P(y), N, P(w1p), P(w1v), P(wp), P(wv), P(coef[2]), P(coef[3]),
                                                 P(coef[0]), P(bn_part), P(a_p), P(a_v), P(dp), P(dv),
                                                 P(v) if ctx.tanh_v else None, P(dh), *(P(t) for t in dws),
                                                 P(ws), ws_bytes, _native.stream_of(dev)), 'hrl_heads_backward(bn)')
        df = _defer_folds(hbufs, 6) if lib.hrl_heads_set_bwd_form(0) == 2 else None
        if df is not None:
            _heads_backward_deferred(lib, df, hbufs, N, ws, call)
        else:
            call(*(b[0] for b in hbufs))
        unit = _unit_coefs(dev) if ctx.relu_in else None
        g_in, grads = _chain_backward(h0, ys, coefs, unit, params, ctx.relu_in, dh, ctx.needs_input_grad[0], packed,
                                      part_in=bn_part, nblk_in=nparts)
        return (g_in, None, None, None, *(_ret(b) for b in hbufs), *grads)


class _ConvBNChain(nn.Module):
    """[relu ->] [BoardConv2d -> BatchNorm2d(fused_relu)] x n as one _BoardChain (set up by fuse_bn_relu).

    The layers are referenced, not registered (parameters and state_dict
    unchanged).  Anything but a training-mode 32-channel 3x3-board batch on the
    GPU runs the layers one by one.
    """

    def __init__(self, convs, bns, relu_in=False):
        super().__init__()
        object.__setattr__(self, 'convs', list(convs))
        object.__setattr__(self, 'bns', list(bns))
        self.relu_in = relu_in

    @staticmethod
    def layers_ok(convs, bns):
        return all(type(c) is BoardConv2d and c.bias is None and tuple(c.weight.shape) == (32, 32, 3, 3)
                   and _board_conv_ok(c) for c in convs) and \
            all(isinstance(b, BatchNorm2d) and b.affine and b.track_running_stats and b.momentum is not None
                and b.num_features == 32 for b in bns)

    def forward(self, x):
        convs, bns = self.convs, self.bns
        if not self.fused_ok(x):
            if self.relu_in:
                x = torch.relu(x)
            for c, b in zip(convs, bns):
                x = b(c(x))
            return x
        meta, params = self.meta_params()
        return _BoardChain.apply(x, meta, self.relu_in, *params)

    def fused_ok(self, x):
        return (x.is_cuda and x.dtype == torch.float32 and x.dim() == 4 and tuple(x.shape[1:]) == (32, 3, 3)
                and x.shape[0] > 0 and all(b.training and b.fused_relu for b in self.bns)
                and torch.is_grad_enabled())

    def meta_params(self):
        """Advance the BatchNorms' batch counters (as their forward would) and collect the chain's arguments."""
        counters = [b.num_batches_tracked for b in self.bns]
        if not _defer_counters(counters):          # else advanced by the step tail's first launch
            torch._foreach_add_(counters, 1)       # one launch for all counters
        meta, params = [], []
        for c, b in zip(self.convs, self.bns):
            meta.append((b.running_mean, b.running_var, b.momentum, b.eps))
            params += [c.weight, b.weight, b.bias]
        return meta, params


class _ChainHeads(nn.Module):
    """A _ConvBNChain whose only consumer is the _FusedHeads pair, as one _ChainHeadsFn (fuse_bn_relu's
    rewrite); anything the fused path does not take runs the two modules one after the other."""

    def __init__(self, chain, heads):
        super().__init__()
        object.__setattr__(self, 'chain', chain)
        object.__setattr__(self, 'heads', heads)
        self.tanh_v = False   # the model's torch.tanh on the value output, folded in by _fuse_chain_heads

    def forward(self, x):
        if not self.chain.fused_ok(x):
            p, v = self.heads(self.chain(x))
            return p, (torch.tanh(v) if self.tanh_v else v)
        (cp, fp), (cv, fv) = _board_head_spec(self.heads.head_p), _board_head_spec(self.heads.head_v)
        meta, params = self.chain.meta_params()
        return _ChainHeadsFn.apply(x, meta, self.chain.relu_in, self.tanh_v, cp.weight, cp.bias, cv.weight, cv.bias,
                                   fp.weight, fv.weight, *params)


def _fuse_chain_heads(gm):
    """Merge a chain call whose only user is the fused heads call into one _ChainHeads call; 0 or 1."""
    for node in list(gm.graph.nodes):
        if node.op != 'call_module' or not isinstance(gm.get_submodule(node.target), _FusedHeads):
            continue
        src = node.args[0] if len(node.args) == 1 else None
        if not (isinstance(src, torch.fx.Node) and src.op == 'call_module'
                and isinstance(gm.get_submodule(src.target), _ConvBNChain) and len(src.users) == 1):
            return 0
        fused = _ChainHeads(gm.get_submodule(src.target), gm.get_submodule(node.target))
        gm.add_submodule('_hrl_chain_heads', fused)
        with gm.graph.inserting_before(src):
            call = gm.graph.call_module('_hrl_chain_heads', src.args)
        node.replace_all_uses_with(call)
        gm.graph.erase_node(node)
        gm.graph.erase_node(src)
        # value = torch.tanh(heads[1]) as the value output's only use (tictactoe.py:62): the kernels apply it
        for item in list(call.users):
            if item.op == 'call_function' and item.target is operator.getitem and item.args[1] == 1 \
                    and len(item.users) == 1:
                user = next(iter(item.users))
                if _is_tanh(user, item):
                    user.replace_all_uses_with(item)
                    gm.graph.erase_node(user)
                    fused.tanh_v = True
        return 1
    return 0


class _LeafTracer(torch.fx.Tracer):
    """Trace the env net, keeping the HIP-backed modules (and ``leaves``) as opaque calls."""

    def __init__(self, leaves=()):
        super().__init__()
        self.extra = set(id(m) for m in leaves)

    def is_leaf_module(self, m, qualname):
        return isinstance(m, (BatchNorm2d, BoardConv2d, Linear, _MultiBoardConv, _ConvBNChain)) or \
            id(m) in self.extra or super().is_leaf_module(m, qualname)


def _is_tanh(node, arg):
    if node.op == 'call_function' and node.target in (torch.tanh, torch.nn.functional.tanh):
        return node.args == (arg,) and not node.kwargs
    if node.op == 'call_method' and node.target == 'tanh':
        return node.args == (arg,) and not node.kwargs
    return False


def _is_relu(gm, node):
    if node.op == 'call_function' and node.target in (torch.relu, torch.nn.functional.relu):
        return len(node.args) == 1
    if node.op == 'call_method' and node.target == 'relu':
        return len(node.args) == 1
    if node.op == 'call_module':
        return isinstance(gm.get_submodule(node.target), nn.ReLU)
    return False


def fuse_bn_relu(model, example=None):
    """Rewrite ``model.forward`` with torch.fx: every BatchNorm2d -> ReLU pair is
    folded into the BatchNorm, and sibling BoardConv2d layers reading the same
    activation become one _MultiBoardConv GEMM.

    The model keeps its class, parameters and state_dict; only its forward is
    replaced by the rewritten graph.  Recurrent nets (``init_hidden``) and nets
    that do not trace are left as they are.  With ``example`` (an observation
    batch), the rewritten forward is checked against the original (eval mode)
    and dropped on any mismatch.  Returns the number of rewrites.
    """
    if hasattr(model, 'init_hidden') or 'forward' in model.__dict__:
        return 0
    try:
        heads = _head_pair(model)
        graph = _LeafTracer(leaves=heads or ()).trace(model)
    except Exception:
        return 0
    gm = torch.fx.GraphModule(model, graph)
    pairs = []
    for node in gm.graph.nodes:
        if node.op == 'call_module' and isinstance(gm.get_submodule(node.target), BatchNorm2d):
            users = list(node.users)
            if len(users) == 1 and _is_relu(gm, users[0]) and users[0].args[0] is node:
                pairs.append((node, users[0]))
    for bn_node, relu_node in pairs:
        relu_node.replace_all_uses_with(bn_node)
        gm.graph.erase_node(relu_node)
    bns = [gm.get_submodule(n.target) for n, _ in pairs]
    chains = _fuse_chains(gm, set(n for n, _ in pairs))
    merged = 0
    for node in list(gm.graph.nodes):
        sibs = [u for u in node.users if u.op == 'call_module' and type(gm.get_submodule(u.target)) is BoardConv2d
                and u.args == (node,) and not u.kwargs]
        if len(sibs) < 2:
            continue
        name = '_hrl_multiconv%d' % merged
        gm.add_submodule(name, _MultiBoardConv([gm.get_submodule(u.target) for u in sibs]))
        with gm.graph.inserting_after(node):
            multi = gm.graph.call_module(name, (node,))
        anchor = multi
        for i, u in enumerate(sibs):
            with gm.graph.inserting_after(anchor):
                item = gm.graph.call_function(operator.getitem, (multi, i))
            u.replace_all_uses_with(item)
            gm.graph.erase_node(u)
            anchor = item
        merged += 1
    fused_heads = _fuse_heads(gm, heads) if heads else 0
    if fused_heads:
        fused_heads += _fuse_chain_heads(gm)
    if not pairs and not merged and not fused_heads:
        return 0
    gm.graph.lint()
    gm.recompile()
    if example is not None:
        was = model.training
        model.eval()
        with torch.no_grad():
            ref = model(example, None)
            for bn in bns:
                bn.fused_relu = True
            new = gm(example, None)
        model.train(was)
        same = _same_outputs(ref, new, rtol=1e-4, atol=1e-5)
        if same and chains and example.is_cuda:
            same = _same_training_outputs(model, gm, bns, example)
        if not same:
            for bn in bns:
                bn.fused_relu = False
            return 0
    for bn in bns:
        bn.fused_relu = True
    model.forward = gm.forward
    object.__setattr__(model, '_hrl_graph', gm)   # the rewritten graph, unregistered: state_dict unchanged
    return len(pairs) + merged + chains + fused_heads


def _same_outputs(ref, new, rtol=1e-5, atol=1e-6):
    return set(ref) == set(new) and all(
        torch.allclose(ref[k], new[k], rtol=rtol, atol=atol) for k in ref if ref[k] is not None)


def _same_training_outputs(model, gm, bns, example):
    """Training-mode check of the fused chains (batch statistics): original vs rewritten
    forward on the example, BatchNorm buffers restored afterwards."""
    buffers = [(b.running_mean.clone(), b.running_var.clone(), b.num_batches_tracked.clone()) for b in bns]

    def restore():
        for b, (m, v, n) in zip(bns, buffers):
            b.running_mean.copy_(m)
            b.running_var.copy_(v)
            b.num_batches_tracked.copy_(n)
    was = model.training
    model.train()
    try:
        for bn in bns:
            bn.fused_relu = False
        ref = model(example, None)
        restore()
        for bn in bns:
            bn.fused_relu = True
        new = gm(example, None)
        restore()
    finally:
        model.train(was)
    ref = {k: v.detach() for k, v in ref.items() if v is not None}
    new = {k: v.detach() for k, v in new.items() if v is not None}
    return _same_outputs(ref, new, rtol=1e-4, atol=1e-5)


def _fuse_chains(gm, fused_bn_nodes):
    """Replace maximal [BoardConv2d -> BatchNorm2d(+ReLU)] chains with one _ConvBNChain call.

    A link continues while the conv's only user is the BN and the BN's only
    user is the next conv; the last BN's output may have any users.  Returns
    the number of chains."""
    def conv_bn(node):
        if node.op != 'call_module' or type(gm.get_submodule(node.target)) is not BoardConv2d or node.kwargs:
            return None
        users = list(node.users)
        if len(users) != 1 or users[0] not in fused_bn_nodes or users[0].args != (node,):
            return None
        return users[0]

    chains, seen = [], set()
    for node in list(gm.graph.nodes):
        if node in seen:
            continue
        bn = conv_bn(node)
        if bn is None:
            continue
        links = [(node, bn)]
        while True:
            users = list(links[-1][1].users)
            if len(users) != 1:
                break
            nxt = conv_bn(users[0])
            if nxt is None:
                break
            links.append((users[0], nxt))
        convs = [gm.get_submodule(c.target) for c, _ in links]
        bns = [gm.get_submodule(b.target) for _, b in links]
        if not _ConvBNChain.layers_ok(convs, bns):
            continue
        for c, b in links:
            seen.update((c, b))
        chains.append((links, convs, bns))
    for k, (links, convs, bns) in enumerate(chains):
        name = '_hrl_chain%d' % k
        first, last = links[0][0], links[-1][1]
        src = first.args[0]
        relu_in = (isinstance(src, torch.fx.Node) and _is_relu(gm, src) and len(src.users) == 1
                   and src.op != 'call_module')
        gm.add_submodule(name, _ConvBNChain(convs, bns, relu_in=relu_in))
        with gm.graph.inserting_before(first):
            call = gm.graph.call_module(name, (src.args[0],) if relu_in else first.args)
        last.replace_all_uses_with(call)
        for c, b in reversed(links):
            gm.graph.erase_node(b)
            gm.graph.erase_node(c)
        if relu_in:
            gm.graph.erase_node(src)
    return len(chains)


def unfuse(model):
    """Undo fuse_bn_relu (e.g. before pickling the model for CPU workers)."""
    if 'forward' in model.__dict__:
        del model.forward
    model.__dict__.pop('_hrl_graph', None)
    for m in model.modules():
        if isinstance(m, BatchNorm2d):
            m.fused_relu = False
    return model
