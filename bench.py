#!/usr/bin/env python
"""Learner throughput on MI355X — BASELINE.json metric.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N \
        --master-addr 127.0.0.1 --master-port P bench.py --gpus N --steps K --warmup W

A "step" is one learner update (handyrl/train.py:372-392 body) on a
device-resident synthetic replay batch in the make_batch layout: TicTacToe
SimpleConv2dModel forward, IS ratios, the fused HIP V-trace/UPGO target scan,
losses, backward, SUM all-reduce of the gradients over RCCL (N > 1), grad
clip 4.0 and Adam.  Every rank trains its own B=4096 x T=32 batch (weak
scaling); value = N*B*T*K / max-over-ranks time of the K timed steps.

Rank 0 prints ONE JSON line with, besides the metric:
  roofline      the step's dominant kernel, one chain block's backward (conv3x3_block_bwd2_kernel + its
                weight-gradient fold, 3 launches, ~40% of the step): algorithmic bytes per launch / mean
                duration from HIP events on the launch stream around the step's own launches (eager steps
                after the timed region); its split-MFMA fraction beside it;
  scan_roofline the B1 operator, the V-trace scan kernel: algorithmic bytes per launch / mean launch time
                from HIP events, at the step's own size and at a cold, larger-than-Infinity-Cache size;
  loss_roofline the step's fused loss forward (csrc/hrl_loss.hip, the scans inside it), algorithmic bytes
                / HIP-event time;
  block_roofline the same block backward launched alone on random data (back-to-back launches);
  cpu_baseline  the CPU learner oracle (oracle/learner.py, restating
                train.py:218-258 + 382-385) timed on this host, 1 thread as the
                reference ships (model.py:8), on a bounded sample (N=1 only).
"""

import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

from handyrl_amd import distributed as hdist          # noqa: E402
from handyrl_amd.envs.tictactoe import SimpleConv2dModel  # noqa: E402
from handyrl_amd.synthetic import tictactoe_batch, default_args  # noqa: E402
from handyrl_amd.trainer import LearnerStep            # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
# PMC passes on the final round-6 tree (tools/gpu_r6i.sh: rocprofv3 FETCH_SIZE / WRITE_SIZE, gfx950-corrected)
SCAN_PMC = 'r06_scan_pmc.json'     # the scan kernel (tools/scan_pmc.py, tools/scan_pmc_json.py)
BLOCK_PMC = 'r06_block_pmc.json'   # the chain block backward, form 1 (tools/conv_pmc.py bwd 1, tools/pmc_bytes.py)
FWD_PMC = 'r06_fwd_pmc.json'       # the ring forward conv, fwd form 2 (tools/conv_pmc.py fwd 2, tools/pmc_bytes.py)


def scan_bytes_per_launch(B, T, P=2, Pp=1, rewards=False):
    """Algorithmic bytes of one V-trace value-head launch.

    read values 4P + rho 4Pp + c 4Pp (+ rewards 4P), write targets 4P + advantages 4P
    per env-step, plus the 4P-byte bootstrap per trajectory.
    """
    per_step = 12 * P + 8 * Pp + (4 * P if rewards else 0)
    return B * T * per_step + B * 4 * P


def time_scan(device, B, T, iters, cold=False):
    """Mean duration of the fused value-head scan launch (VTRACE target + UPGO advantages)."""
    from handyrl_amd.losses import compute_targets_fused
    g = torch.Generator(device=device).manual_seed(7)
    n_sets = 1
    if cold:
        # rotate through enough input sets that every launch misses the 256 MiB Infinity Cache
        per_set = scan_bytes_per_launch(B, T)
        n_sets = max(2, int(3 * 256 * 2 ** 20 // per_set) + 1)
    sets = []
    for _ in range(n_sets):
        v = torch.tanh(torch.randn(B, T, 2, 1, device=device, generator=g))
        ret = torch.randint(-1, 2, (B, 1, 2, 1), device=device, generator=g).float()
        rho = torch.rand(B, T, 1, 1, device=device, generator=g)
        cs = torch.rand(B, T, 1, 1, device=device, generator=g)   # a separate tensor, as in the learner
        sets.append((v, ret, rho, cs))

    def launch(i):
        st = sets[i % n_sets]
        compute_targets_fused('VTRACE', 'UPGO', st[0], st[1], None, 0.7, 1, st[2], st[3])
    for i in range(2):
        launch(i)
    # capture the launches back to back in one HIP graph so the timing is the
    # GPU's, not the Python launch path's (the learner step is graph-captured too)
    graph = torch.cuda.CUDAGraph()
    side = torch.cuda.Stream(device)
    side.wait_stream(torch.cuda.current_stream(device))
    with torch.cuda.stream(side):
        launch(0)
    torch.cuda.current_stream(device).wait_stream(side)
    with torch.cuda.graph(graph):
        for i in range(iters):
            launch(i)
    stream = torch.cuda.current_stream(device)
    graph.replay()
    start = torch.cuda.Event(enable_timing=True)
    end = torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize(device)
    start.record(stream)
    graph.replay()
    end.record(stream)
    end.synchronize()
    ms = start.elapsed_time(end) / iters
    nbytes = scan_bytes_per_launch(B, T)
    return {'B': B, 'T': T, 'us_per_launch': ms * 1e3, 'bytes_per_launch': nbytes,
            'GBps': nbytes / (ms * 1e-3) / 1e9, 'cold': cold}


MFMA_F32_PEAK_TFLOPS = 157.3   # MI355X dense fp32 MFMA (MI355X_MICROARCH.md)
MFMA_BF16_PEAK_TFLOPS = 16 * MFMA_F32_PEAK_TFLOPS   # dense bf16 MFMA: 16x the fp32 rate (MI355X_MICROARCH.md)
SPLIT_PRODUCTS = 6   # exact three-way bf16 split of both operands: hh, hm, mh, hl, lh, mm


FWD_KERNEL = {1: 'conv3x3_block_bwd2_kernel<true,1> (the tile-shared form)',
              2: 'conv3x3_fwd_dma_kernel<true> (the LDS-DMA ring form)'}


def time_conv(device, M, iters=20):
    """The chain's forward conv as the step runs it (hrl_conv3x3_forward_ex: epilogue 1 = the output's BN
    statistics, packed weights, the previous block's BN + ReLU as prologue; csrc/hrl_conv.hip) at M = B*T rows,
    HIP events on the launch stream over `iters` back-to-back launches.

    Algorithmic bytes per launch: x read + y written (151 MB each at M = 131,072); FLOPs: 49 on-board 32x32 tap
    blocks x 2 per sample (the 32 off-board blocks of the dense 9x9 board matrix are not work).
    """
    from handyrl_amd import _native
    lib = _native.load()
    form = lib.hrl_conv3x3_set_fwd_form(1)
    lib.hrl_conv3x3_set_fwd_form(form)
    g = torch.Generator(device=device).manual_seed(3)
    x = torch.randn(M, 288, device=device, generator=g)
    w = torch.randn(32, 32, 3, 3, device=device, generator=g) * 0.1
    alpha = torch.rand(32, device=device, generator=g) + 0.5
    beta = torch.randn(32, device=device, generator=g) * 0.3
    y = torch.empty_like(x)
    P = _native.ptr
    stream = _native.stream_of(device)
    packed = torch.empty(1, 2, 9216, device=device)
    _native.check(lib.hrl_conv3x3_pack_n(_native.ptr_array([w]), 1, P(packed), stream), 'pack')
    ws_bytes = lib.hrl_conv3x3_workspace_bytes(M)
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=device)
    part = torch.empty(lib.hrl_conv3x3_stats_blocks(M) * 64, dtype=torch.float64, device=device)
    tstream = torch.cuda.current_stream(device)

    def launch():
        _native.check(lib.hrl_conv3x3_forward_ex(P(x), M, P(alpha), P(beta), P(packed[0, 0]), None, 2, P(y), 1,
                                                 None, None, None, None, P(part), P(ws), ws_bytes, stream),
                      'hrl_conv3x3_forward_ex')
    for _ in range(3):
        launch()
    start = torch.cuda.Event(enable_timing=True)
    end = torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize(device)
    start.record(tstream)
    for _ in range(iters):
        launch()
    end.record(tstream)
    end.synchronize()
    us = start.elapsed_time(end) * 1e3 / iters
    nbytes = 2 * M * 288 * 4
    gbs = nbytes / (us * 1e-6) / 1e9
    flops = 2.0 * M * 49 * 32 * 32
    tf = flops / (us * 1e-6) / 1e12
    # each fp32 product runs as six bf16 MFMA partial products (the exact split), so the MFMA ceiling for
    # fp32-accurate work is the bf16 dense peak / 6
    peak = MFMA_BF16_PEAK_TFLOPS / SPLIT_PRODUCTS
    return {'kernel': FWD_KERNEL.get(form, 'form %d' % form), 'fwd_form': form, 'bound': 'hbm',
            'achieved': round(gbs, 1), 'peak': HBM_PEAK_GBS, 'unit': 'GB/s', 'frac': round(gbs / HBM_PEAK_GBS, 4),
            'bytes_per_launch': nbytes, 'us_per_launch': round(us, 2), 'M': M,
            'mfma_achieved_TFLOPs': round(tf, 1), 'mfma_frac_split': round(tf / peak, 4),
            'launches_per_step': 3,
            'traffic': _pmc_bytes(FWD_PMC) if form == 2 else None,
            'traffic_source': ('profiles/%s (rocprofv3 FETCH_SIZE/WRITE_SIZE passes, gfx950-corrected)' % FWD_PMC
                               if form == 2 else None),
            'note': 'the step\'s chain forward (BN statistics epilogue, BN + ReLU prologue) on random data; bytes = x '
                    'read + y written; split ceiling = bf16 dense peak / 6 partial products'}


def loss_bytes_per_launch(B, T, P=2, Pp=1, A=9):
    """Algorithmic bytes of the fused loss forward (csrc/hrl_loss.hip, value head only).

    Per env-step (b, t): reads target and behaviour logits 8*Pp*A, action 8*Pp, episode mask 4, progress 4,
    turn / observation masks and the value head 12*P; writes the backward's entropy 4*Pp, value target 4*P and
    turn advantage 4; per trajectory the outcome 4*P.
    """
    per_step = 8 * Pp * A + 8 * Pp + 8 + 12 * P + 4 * Pp + 4 * P + 4
    return B * T * per_step + B * 4 * P


def time_loss(device, B, T, iters=50):
    """The step's loss forward as it runs in the step (loss_fused_kernel + its fixed-order fold), timed with
    HIP events on the launch stream over `iters` launches captured in one HIP graph."""
    from handyrl_amd.train import _FusedLoss
    from handyrl_amd import _native
    batch = tictactoe_batch(B, T, device, seed=5)
    g = torch.Generator(device=device).manual_seed(4)
    tpol = (torch.randn(B, T, 1, 9, device=device, generator=g) - batch['action_mask']).contiguous()
    value = torch.tanh(torch.randn(B, T, 2, 1, device=device, generator=g))
    args = default_args(T, B)
    alg = _native.ALG
    cfg = {'value_target': alg[args['value_target']], 'policy_target': alg[args['policy_target']], 'symmetrize': 1,
           'lambda': float(args['lambda']), 'gamma': float(args['gamma']),
           'ent_coef': float(args['entropy_regularization']), 'ent_decay': float(args['entropy_regularization_decay'])}

    def launch():
        with torch.no_grad():
            _FusedLoss.apply(tpol, value, None, batch['policy'], batch['action'], batch['episode_mask'],
                             batch['turn_mask'], batch['observation_mask'], batch['progress'], batch['outcome'],
                             None, None, cfg)
    for _ in range(3):
        launch()
    graph = torch.cuda.CUDAGraph()
    side = torch.cuda.Stream(device)
    side.wait_stream(torch.cuda.current_stream(device))
    with torch.cuda.stream(side):
        launch()
    torch.cuda.current_stream(device).wait_stream(side)
    with torch.cuda.graph(graph):
        for _ in range(iters):
            launch()
    stream = torch.cuda.current_stream(device)
    graph.replay()
    start, end = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize(device)
    start.record(stream)
    graph.replay()
    end.record(stream)
    end.synchronize()
    us = start.elapsed_time(end) * 1e3 / iters
    nbytes = loss_bytes_per_launch(B, T)
    gbs = nbytes / (us * 1e-6) / 1e9
    return {'kernel': 'loss_fused_kernel<VTRACE,UPGO,value,no return,A=9> + loss_reduce_kernel (the step\'s fused '
                      'loss forward, its scans included)',
            'bound': 'hbm', 'achieved': round(gbs, 1), 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
            'frac': round(gbs / HBM_PEAK_GBS, 4), 'traffic': None, 'bytes_per_launch': nbytes,
            'us_per_launch': round(us, 3), 'B': B, 'T': T,
            'note': 'algorithmic bytes (DESIGN.md §4.4) / HIP-event time of the two launches; latency-bound at '
                    'the step size (the wave\'s prep -> scan chain -> terms critical path)'}


def time_block_backward(device, M, iters=20):
    """The step's dominant kernel: one chain block's backward (conv3x3_block_bwd2_kernel, BN backward apply +
    weight gradient + input gradient, csrc/hrl_conv.hip) at M = B*T rows, HIP events over back-to-back launches
    (its weight-gradient fold launch included)."""
    from handyrl_amd import _native
    lib = _native.load()
    P = _native.ptr
    stream = _native.stream_of(device)
    g0 = torch.Generator(device=device).manual_seed(1)
    rnd = lambda *sh: torch.randn(*sh, device=device, generator=g0)   # noqa: E731
    g, y, x = rnd(M, 288), rnd(M, 288), rnd(M, 288)
    w = rnd(32, 32, 3, 3) * 0.1
    c = [rnd(32).abs() + 0.5 for _ in range(11)]
    packed = torch.empty(1, 2, 9216, device=device)
    _native.check(lib.hrl_conv3x3_pack_n(_native.ptr_array([w]), 1, P(packed), stream), 'pack')
    ws_bytes = lib.hrl_conv3x3_workspace_bytes(M)
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=device)
    part = torch.empty(lib.hrl_conv3x3_stats_blocks(M) * 64, dtype=torch.float64, device=device)
    dw, gin = torch.empty(32, 32, 3, 3, device=device), torch.empty_like(g)

    def launch():
        _native.check(lib.hrl_conv3x3_block_backward(
            P(g), P(y), M, *[P(t) for t in c[:6]], P(x), P(c[6]), P(c[7]), P(packed[0, 1]), P(dw), P(gin), 2,
            P(c[8]), P(c[9]), P(c[10]), P(part), P(ws), ws_bytes, stream), 'block')
    for _ in range(3):
        launch()
    s0, e0 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize(device)
    s0.record(torch.cuda.current_stream(device))
    for _ in range(iters):
        launch()
    e0.record(torch.cuda.current_stream(device))
    e0.synchronize()
    us = s0.elapsed_time(e0) * 1e3 / iters
    nbytes = 4 * M * 288 * 4                       # reads g, y, x; writes gin
    flops = 2 * (2.0 * M * 49 * 32 * 32)           # weight gradient + input gradient
    gbs, tf = nbytes / (us * 1e-6) / 1e9, flops / (us * 1e-6) / 1e12
    mfma_peak = MFMA_BF16_PEAK_TFLOPS / SPLIT_PRODUCTS
    return {'kernel': 'conv3x3_block_bwd2_kernel<PRO, EPI=2> + wgrad fold (one chain block backward)',
            'bound': 'hbm+mfma', 'achieved_GBps': round(gbs, 1), 'frac_hbm': round(gbs / HBM_PEAK_GBS, 4),
            'achieved_TFLOPs': round(tf, 1), 'frac_mfma_split': round(tf / mfma_peak, 4),
            'bytes_per_launch': nbytes, 'flops_per_launch': flops, 'us_per_launch': round(us, 2), 'M': M,
            'launches_per_step': 3,
            'note': 'bytes = g, y, x read + gin written (dY and x\' stay on chip); flops = weight + input gradient '
                    'on the 49 on-board tap blocks; split ceiling = bf16 dense peak / 6'}


def time_block_in_step(learner, batch, device, steps=4):
    """The dominant kernel as the step runs it: HIP events on the launch stream around every chain block backward
    launch (conv3x3_block_bwd2_kernel; its partials are folded by the step tail) of a few EAGER learner steps (the same
    kernels the graph replays, on the step's own data), after the timed region."""
    from handyrl_amd import nn as hnn
    hnn.BLOCK_TIMING = []
    reducer = learner.reducer
    # each rank's update would use its own un-reduced gradients: the training state is put back afterwards, so
    # the replicas stay identical (and equal to the state after the timed steps)
    snap = learner.snapshot()
    if reducer is not None:
        reducer.enabled = False     # no gradient all-reduce in these steps: nothing to pair across ranks, and
    try:                            # no collective between the timed launches on the stream
        for _ in range(steps):
            learner._body(batch, None)
        torch.cuda.synchronize(device)
        ts = [s.elapsed_time(e) * 1e3 for s, e in hnn.BLOCK_TIMING[3:]]   # the first eager step warms up
    finally:
        hnn.BLOCK_TIMING = None
        learner.restore(snap)
        if reducer is not None:
            reducer.enabled = True
            reducer.reset()
    return sum(ts) / max(len(ts), 1), len(ts)


def block_traffic():
    """HBM bytes per chain block backward launch from the committed rocprofv3 PMC passes (profiles/), or None."""
    return _pmc_bytes(BLOCK_PMC)


def _pmc_bytes(name):
    path = os.path.join(ROOT, 'profiles', name)
    if not os.path.exists(path):
        return None
    with open(path) as f:
        return json.load(f).get('bytes_per_launch')


def pmc_traffic(B, T):
    """HBM bytes per launch of the scan from the committed rocprofv3 PMC passes (profiles/), or None."""
    path = os.path.join(ROOT, 'profiles', SCAN_PMC)
    if not os.path.exists(path):
        return None
    with open(path) as f:
        for c in json.load(f)['configs']:
            if c['B'] == B and c['T'] == T:
                return c['traffic_bytes']
    return None


def cpu_model():
    """The host CPU's model name (lscpu's 'Model name', read from /proc/cpuinfo), or None."""
    try:
        with open('/proc/cpuinfo') as f:
            for line in f:
                if line.startswith('model name'):
                    return line.split(':', 1)[1].strip()
    except OSError:
        pass
    return None


def cpu_learner_rate(B, T, steps, threads):
    """env-steps/s and seconds of the CPU learner oracle on `threads` torch threads."""
    from oracle.learner import CpuLearner
    saved = torch.get_num_threads()
    torch.set_num_threads(threads)
    try:
        torch.manual_seed(0)
        net = SimpleConv2dModel()
        args = default_args(T, B)
        batch = tictactoe_batch(B, T, torch.device('cpu'), seed=11)
        learner = CpuLearner(net, args)
        learner.step(batch)  # warm-up
        t0 = time.perf_counter()
        for _ in range(steps):
            learner.step(batch)
        dt = time.perf_counter() - t0
    finally:
        torch.set_num_threads(saved)
    return B * T * steps / dt, dt


def cpu_baseline(B=4096, T=32, steps=3, threads_secondary=8):
    """The CPU learner oracle on this host, 1 thread (train.py as shipped: model.py:8), at the metric's
    B=4096 T=32 (about 4 s per step on the GPU box's host cores), and the 8-thread variant as the
    secondary.  Calibrated against the reference itself in the build container by
    tools/calibrate_cpu.py (profiles/r02_cpu_calibration.json: the port runs at 0.91-1.07x the
    reference's time)."""
    v1, dt1 = cpu_learner_rate(B, T, steps, 1)
    v8, dt8 = cpu_learner_rate(B, T, steps, threads_secondary)
    return {'value': v1, 'unit': 'env-steps/s', 'cores': 1, 'kind': 'port',
            'sample': 'oracle.learner.CpuLearner (restates train.py:218-258,382-385), TicTacToe net, '
                      'synthetic B=%d T=%d, %d timed steps after 1 warm-up, torch 1 thread, %.1f s'
                      % (B, T, steps, dt1),
            'secondary_threads': {'value': v8, 'unit': 'env-steps/s', 'cores': threads_secondary,
                                  'seconds': round(dt8, 2),
                                  'note': 'the same sample on %d torch threads (the reference ships 1 thread, '
                                          'model.py:8)' % threads_secondary},
            'host': {'cpu_model': cpu_model(), 'os_cpu_count': os.cpu_count()}}


def secondary_t9(device, steps=40, warmup=20, B=4096, T=9):
    """BASELINE.json configs[1]: TicTacToe B=4096 T=9, the north star's >=50x point."""
    args = default_args(T, B)
    torch.manual_seed(0)
    net = SimpleConv2dModel().to(device)
    batch = tictactoe_batch(B, T, device, seed=77)
    learner = LearnerStep(net, args, device, graph=True)
    for _ in range(max(warmup, 1)):
        learner.step(batch)
    torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    for _ in range(steps):
        learner.step(batch)
    torch.cuda.synchronize(device)
    dt = time.perf_counter() - t0
    value = B * T * steps / dt
    ref_cpu = 18.7e3   # reference train.py, 1 thread, B=4096 T=9 (survey container CPU)
    return {'config': 'TicTacToe B=4096 T=9 (BASELINE.json configs[1])', 'value': round(value, 1),
            'unit': 'env-steps/s', 'ms_per_step': round(dt / steps * 1e3, 4),
            'vs_reference_cpu_1thread': round(value / ref_cpu, 1),
            'reference_cpu_source': 'BASELINE.md, 18.7k env-steps/s measured in the survey container'}


def secondary_rollout(device, E=16384, reps=5):
    """Device self-play throughput: E concurrent TicTacToe games, one batched forward per ply."""
    from handyrl_amd.rollout import TicTacToeBatch, DeviceGenerator, DeviceReplay
    from handyrl_amd.nn import accelerate
    torch.manual_seed(0)
    net = accelerate(SimpleConv2dModel().to(device))
    gen = DeviceGenerator(TicTacToeBatch(E, device), net)
    rep = DeviceReplay(4 * E, 9, (3, 3, 3), 9, 2, device)
    g = torch.Generator(device=device).manual_seed(0)
    rep.add(gen.generate(generator=g))   # warm-up
    torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    plies = 0
    for _ in range(reps):
        ep = gen.generate(generator=g)
        rep.add(ep)
        plies += ep['length'].sum()
    torch.cuda.synchronize(device)
    dt = time.perf_counter() - t0
    plies = int(plies)
    return {'config': 'TicTacToe device self-play, %d concurrent games, SimpleConv2dModel inference' % E,
            'value': round(plies / dt, 1), 'unit': 'env-steps/s', 'games_per_s': round(E * reps / dt, 1),
            'reference_cpu_worker': 1840.0,
            'reference_cpu_source': 'SURVEY §6: generation.py per worker process, measured in the survey container'}


def secondary_geister_learner(device, B=256, T=16, steps=20, warmup=10):
    """recurrent learner step (GeisterNet unrolled over T, config.yaml batch 256)."""
    from handyrl_amd.envs.geister import GeisterNet
    from handyrl_amd.synthetic import geister_batch
    args = default_args(T, B)
    torch.manual_seed(0)
    net = GeisterNet().to(device)
    batch = geister_batch(B, T, device, seed=5)
    hidden = tuple([h.to(device) for h in hs] for hs in net.init_hidden([B, 2]))
    learner = LearnerStep(net, args, device, graph=True)
    for _ in range(max(warmup, 1)):
        learner.step(batch, hidden)
    torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    for _ in range(steps):
        learner.step(batch, hidden)
    torch.cuda.synchronize(device)
    dt = time.perf_counter() - t0
    value = B * T * steps / dt
    ref_cpu = 929.0
    return {'config': 'Geister recurrent learner B=%d T=%d (GeisterNet, UPGO/VTRACE)' % (B, T),
            'value': round(value, 1), 'unit': 'env-steps/s', 'ms_per_step': round(dt / steps * 1e3, 3),
            'vs_reference_cpu_1thread': round(value / ref_cpu, 1),
            'reference_cpu_source': 'tools/ref_geister_cpu.py: reference compute_loss+backward+Adam, '
                                    'B=64 T=16, 1 thread, 929 env-steps/s (build container)'}


def secondary_geese_learner(device, B=2048, T=64, steps=5, warmup=3):
    """BASELINE.json configs[3]: Hungry Geese GeeseNet learner, B=2048 T=64, solo training (P = Pp = 1),
    UPGO policy / VTRACE value targets; 13 torus 3x3 convs (csrc/hrl_torus.hip) over B*T boards."""
    from handyrl_amd.envs.hungry_geese import GeeseNet
    from handyrl_amd.synthetic import geese_batch, geese_args
    from oracle.learner import CpuLearner
    args = geese_args(T, B)
    torch.manual_seed(0)
    net = GeeseNet().to(device)
    batch = geese_batch(B, T, device, seed=5)
    learner = LearnerStep(net, args, device, graph=True)
    for _ in range(max(warmup, 1)):
        learner.step(batch)
    torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    for _ in range(steps):
        learner.step(batch)
    torch.cuda.synchronize(device)
    dt = time.perf_counter() - t0
    value = B * T * steps / dt
    del learner, batch, net
    torch.cuda.empty_cache()
    # the CPU oracle learner on the same layout, 1 thread, bounded sample (B=16)
    threads = torch.get_num_threads()
    torch.set_num_threads(1)
    try:
        torch.manual_seed(0)
        cb, cpu_batch = 16, geese_batch(16, T, torch.device('cpu'), seed=5)
        cpu = CpuLearner(GeeseNet(), geese_args(T, cb))
        cpu.step(cpu_batch)
        c0 = time.perf_counter()
        cpu.step(cpu_batch)
        cpu_rate = cb * T / (time.perf_counter() - c0)
    finally:
        torch.set_num_threads(threads)
    flops = 2.0 * B * T * 77 * 32 * 9 * (32 * 12 * 3 + 17 * 2)   # fwd + dgrad + wgrad (no stem dgrad)
    return {'config': 'Hungry Geese GeeseNet learner B=%d T=%d (BASELINE.json configs[3]; solo training, '
                      'UPGO/VTRACE)' % (B, T),
            'value': round(value, 1), 'unit': 'env-steps/s', 'ms_per_step': round(dt / steps * 1e3, 3),
            'conv_tflops_per_step': round(flops / 1e12, 3),
            # the whole step's time charged to the conv FLOPs: a floor on the torus kernels' MFMA rate
            'conv_tflops_per_s_whole_step': round(flops / (dt / steps) / 1e12, 1),
            'cpu_oracle': {'value': round(cpu_rate, 1), 'unit': 'env-steps/s', 'cores': 1, 'kind': 'port',
                           'sample': 'oracle.learner.CpuLearner, GeeseNet, B=16 T=64, 1 step after 1 warm-up'},
            'vs_cpu_oracle': round(value / cpu_rate, 1)}


def secondary_host_rollout(device, E=256):
    """The host-env generator (hostgen.HostBatchGenerator: any plugin env through the Environment API, one batched
    GPU forward per ply; generation.py:20-88) on ParallelTicTacToe (simultaneous turns) and Geister with
    observation=True (every player observes, recurrent state per game and player), E = 256 game slots."""
    from handyrl_amd.environment import make_env
    from handyrl_amd.hostgen import HostBatchGenerator
    from handyrl_amd.nn import accelerate
    out = {}
    for name, games, observation in (('ParallelTicTacToe', 2048, False), ('Geister', 256, True)):
        env_args = {'env': name}
        torch.manual_seed(0)
        net = accelerate(make_env(env_args).net()().to(device))   # HIP inference BatchNorm etc., as self-play
        gen = HostBatchGenerator(lambda: make_env(env_args), net, {'observation': observation, 'gamma': 0.8}, E=E)
        gen.generate(E)                      # warm-up
        torch.cuda.synchronize(device)
        t0 = time.perf_counter()
        eps = gen.generate(games)
        dt = time.perf_counter() - t0
        steps = sum(e['steps'] for e in eps)
        out[name] = {'value': round(steps / dt, 1), 'unit': 'env-steps/s', 'episodes': len(eps), 'plies': steps,
                     'seconds': round(dt, 2), 'observation': observation,
                     'time_split_s': {k: round(v, 3) for k, v in gen.timing.items()}}
    out['E'] = E
    out['reference_cpu_worker'] = {'TicTacToe': 1840.0, 'Geister': 349.0}
    out['note'] = ('one host process; time_split: requests = env observations (the plugin\'s own code), launch = '
                   'stacking + H2D + forward launch, wait = host blocked on a forward, advance = masks, sampling, '
                   'env.step/reward and moment records')
    return out


def secondary_player_rollout(device):
    """The per-player device generator (rollout.DeviceGenerator's per-player ply, generation.py:35-62): every
    player's view through one forward per ply, per-player records and state, into a PlayerReplay -- the modes the
    host generator served before round 6: TicTacToe with observation=True, ParallelTicTacToe (simultaneous
    moves, parallel_tictactoe.py:20-24) and Geister with observation=True (recurrent state per player and game)."""
    from handyrl_amd.envs.geister import GeisterNet, GeisterBatch
    from handyrl_amd.rollout import TicTacToeBatch, ParallelTicTacToeBatch, DeviceGenerator, PlayerReplay
    from handyrl_amd.nn import accelerate
    out = {}
    for name, cls, make_net, E, reps, obs in (('TicTacToe_observation', TicTacToeBatch, SimpleConv2dModel, 16384, 5,
                                               True),
                                              ('ParallelTicTacToe', ParallelTicTacToeBatch, SimpleConv2dModel, 16384,
                                               5, False),
                                              ('Geister_observation', GeisterBatch, GeisterNet, 2048, 1, True)):
        torch.manual_seed(0)
        net = accelerate(make_net().to(device))
        gen = DeviceGenerator(cls(E, device), net, observation=obs)
        rep = PlayerReplay(2 * E, cls.MAX_PLIES, cls.OBS_SHAPE, cls.A, cls.P, device, obs_dtype=torch.uint8,
                           mover=not obs)
        g = torch.Generator(device=device).manual_seed(0)
        rep.add(gen.generate(generator=g))   # warm-up (and the ply graph's capture)
        torch.cuda.synchronize(device)
        t0 = time.perf_counter()
        plies = 0
        for _ in range(reps):
            ep = gen.generate(generator=g)
            rep.add(ep)
            plies += ep['length'].sum()
        torch.cuda.synchronize(device)
        dt = time.perf_counter() - t0
        plies = int(plies)
        out[name] = {'value': round(plies / dt, 1), 'unit': 'env-steps/s', 'games': E * reps,
                     'games_per_s': round(E * reps / dt, 1), 'mean_plies': round(plies / (E * reps), 1),
                     'observation': obs}
        del gen, rep, net
        torch.cuda.empty_cache()
    out['note'] = ('one forward per ply over all P x E (player, game) views; env-steps = plies; the host generator '
                   'served these modes before (host_rollout)')
    return out


def secondary_geister_rollout(device, E=2048, reps=2):
    """BASELINE.json configs[2]: Geister device self-play, E concurrent games, recurrent GeisterNet inference."""
    from handyrl_amd.envs.geister import GeisterNet, GeisterBatch
    from handyrl_amd.rollout import DeviceGenerator, DeviceReplay
    from handyrl_amd.nn import accelerate
    torch.manual_seed(0)
    net = accelerate(GeisterNet().to(device))
    gen = DeviceGenerator(GeisterBatch(E, device), net)
    rep = DeviceReplay(4 * E, GeisterBatch.MAX_PLIES, GeisterBatch.OBS_SHAPE, GeisterBatch.A, 2, device,
                       obs_dtype=torch.uint8)
    g = torch.Generator(device=device).manual_seed(0)
    rep.add(gen.generate(generator=g))   # warm-up
    torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    plies = 0
    for _ in range(reps):
        ep = gen.generate(generator=g)
        rep.add(ep)
        plies += ep['length'].sum()
    torch.cuda.synchronize(device)
    dt = time.perf_counter() - t0
    plies = int(plies)
    return {'config': 'Geister device self-play, %d concurrent games, GeisterNet (DRC ConvLSTM) inference '
                      '(BASELINE.json configs[2])' % E,
            'value': round(plies / dt, 1), 'unit': 'env-steps/s', 'games_per_s': round(E * reps / dt, 1),
            'mean_plies': round(plies / (E * reps), 1),
            'reference_cpu_worker': 349.0,
            'reference_cpu_source': 'tools/ref_geister_gen_cpu.py: reference Generator + GeisterNet, 1 thread, '
                                    'build container'}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    # the warm-up covers the eager steps, the capture and the first graph replays, which run ~10% slow while
    # the clocks settle after the capture's idle GPU (profiles/r05_replay_gaps.txt: replays 0-9)
    ap.add_argument('--steps', type=int, default=50)
    ap.add_argument('--warmup', type=int, default=30)
    ap.add_argument('--batch', type=int, default=4096, help='trajectories per GPU (B)')
    ap.add_argument('--seq', type=int, default=32, help='forward_steps (T)')
    ap.add_argument('--graph', type=int, default=1, help='capture the step in HIP graphs (N>1: backward and update graphs around the all-reduce)')
    ap.add_argument('--cpu-baseline', type=int, default=1)
    ap.add_argument('--scan-iters', type=int, default=200)
    ap.add_argument('--secondary', type=int, default=1, help='also time the B=4096 T=9 config (N=1)')
    opts = ap.parse_args()

    rank, world, local = hdist.world_from_env()
    if world != opts.gpus:
        if world == 1 and opts.gpus > 1:
            raise SystemExit('--gpus %d needs torch.distributed.run with %d processes' % (opts.gpus, opts.gpus))
    # ranks beyond the visible GPUs share them (HRL_DIST_BACKEND=gloo rehearsal on a one-GPU box)
    device = torch.device('cuda', local % max(torch.cuda.device_count(), 1))
    torch.cuda.set_device(device)
    hdist.init_process_group('cuda')

    B, T = opts.batch, opts.seq
    args = default_args(T, B)
    torch.manual_seed(0)                       # identical initial weights on every rank
    net = SimpleConv2dModel().to(device)
    net.train()
    batch = tictactoe_batch(B, T, device, seed=1000 + rank)  # each rank its own shard
    use_graph = bool(opts.graph)
    learner = LearnerStep(net, args, device, graph=use_graph, world_size=world)

    for _ in range(opts.warmup):
        learner.step(batch)
    if use_graph and opts.warmup == 0:
        learner.step(batch)  # capture outside the timed region

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(device)

    barrier()
    t0 = time.perf_counter()
    for _ in range(opts.steps):
        learner.step(batch)
    barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=device, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()
    stats, nb = learner.pop_stats()
    # the roofline line is the step's dominant kernel, timed inside eager learner steps after the timed region,
    # with the gradient all-reduce off (every rank runs them, so the ranks stay in step; rank 0 reports)
    us_blk, n_blk = time_block_in_step(learner, batch, device)
    if world > 1:
        dist.barrier()

    if rank == 0:
        steps_total = world * B * T * opts.steps
        value = steps_total / elapsed
        hot = time_scan(device, B, T, opts.scan_iters)
        cold = time_scan(device, 1 << 18, T, 60, cold=True)
        scan_roof = {
            'kernel': 'targets_kernel<VTRACE,UPGO> value head (hrl_compute_targets_fused)',
            'in_step': False,
            'in_step_note': 'the B1 operator boundary (compute_target, losses.py:61) on the step-size batch; the '
                            'learner step runs the same scan code (hrl_scan.h recur_chunk) inside '
                            'loss_fused_kernel (loss_roofline), so this kernel is not in the step sequence',
            'bound': 'hbm',
            'achieved': round(hot['GBps'], 1),
            'peak': HBM_PEAK_GBS,
            'unit': 'GB/s',
            'frac': round(hot['GBps'] / HBM_PEAK_GBS, 4),
            'traffic': pmc_traffic(B, T),
            'traffic_source': 'profiles/%s (rocprofv3 FETCH_SIZE/WRITE_SIZE passes, gfx950-corrected)' % SCAN_PMC,
            'bytes_per_launch': hot['bytes_per_launch'],
            'us_per_launch': round(hot['us_per_launch'], 3),
            'cold_large_B': {'B': cold['B'], 'T': T, 'achieved': round(cold['GBps'], 1),
                             'frac': round(cold['GBps'] / HBM_PEAK_GBS, 4),
                             'us_per_launch': round(cold['us_per_launch'], 2),
                             'traffic': pmc_traffic(cold['B'], T)},
        }
        net_roof = time_conv(device, B * T)
        loss_roof = time_loss(device, B, T)
        block_roof = time_block_backward(device, B * T)
        # the roofline line is the step's dominant kernel: the chain block backward (3 launches, ~40% of the step)
        blk_bytes = block_roof['bytes_per_launch']
        blk_gbs = blk_bytes / (us_blk * 1e-6) / 1e9
        blk_tf = block_roof['flops_per_launch'] / (us_blk * 1e-6) / 1e12
        roof = {
            'kernel': 'conv3x3_block_bwd2_kernel: one chain block backward of the step (BN backward apply + weight '
                      'gradient + input gradient, csrc/hrl_conv.hip; its weight-gradient partials are folded by the '
                      'step tail)',
            'bound': 'hbm',
            'achieved': round(blk_gbs, 1),
            'peak': HBM_PEAK_GBS,
            'unit': 'GB/s',
            'frac': round(blk_gbs / HBM_PEAK_GBS, 4),
            'traffic': block_traffic(),
            'traffic_source': 'profiles/%s (rocprofv3 FETCH_SIZE/WRITE_SIZE passes over '
                              'tools/conv_pmc.py bwd 1, gfx950-corrected)' % BLOCK_PMC,
            'bytes_per_launch': blk_bytes,
            'us_per_launch': round(us_blk, 2),
            'launches_timed': n_blk,
            'timing': 'HIP events on the launch stream around each of the step\'s block backward launches in eager '
                      'steps after the timed region (the graph replays the same launches), each start event queued '
                      'behind a ~50 us GPU spin so the host\'s launch latency is not inside the interval',
            'mfma_achieved_TFLOPs': round(blk_tf, 1),
            'mfma_frac_split': round(blk_tf / (MFMA_BF16_PEAK_TFLOPS / SPLIT_PRODUCTS), 4),
        }
        cpu = cpu_baseline() if (opts.cpu_baseline and world == 1) else None
        t9 = secondary_t9(device) if (opts.secondary and world == 1) else None
        ro = secondary_rollout(device) if (opts.secondary and world == 1) else None
        gro = secondary_geister_rollout(device) if (opts.secondary and world == 1) else None
        gle = secondary_geister_learner(device) if (opts.secondary and world == 1) else None
        gee = secondary_geese_learner(device) if (opts.secondary and world == 1) else None
        hro = secondary_host_rollout(device) if (opts.secondary and world == 1) else None
        pro = secondary_player_rollout(device) if (opts.secondary and world == 1) else None
        line = {
            'metric': 'learner env-steps/sec at B=4096 T=32 (TicTacToe net, UPGO/VTRACE)',
            'value': round(value, 1),
            'unit': 'env-steps/s',
            'n_gpus': world,
            'steps': opts.steps,
            'warmup': opts.warmup,
            'ms_per_step': round(elapsed / opts.steps * 1e3, 4),
            'timing_note': ('the first ~30 graph replays after the capture run 5-25% slow while the GPU clock '
                            'settles, MFMA-bound kernels most (profiles/r06_replay_clock_ramp.txt); fewer warm-up '
                            'steps put part of that ramp in the timed region'),
            'higher_is_better': True,
            'scaling': 'weak',
            'vs_baseline': None,
            'dtype': 'f32',
            'data': 'synthetic (make_batch layout, SURVEY §8d D2), random-init weights',
            'config': {'workload': 'TicTacToe SimpleConv2dModel learner step: forward + IS ratios + fused '
                                   'HIP V-trace/UPGO scans + losses + backward + grad all-reduce + clip + Adam',
                       'global_batch': world * B, 'per_gpu_batch': B, 'seq_len': T, 'players': 2,
                       'parallelism': 'dp%d' % world, 'hip_graph': use_graph},
            'roofline': roof,
            'scan_roofline': scan_roof,
            'net_roofline': net_roof,
            'loss_roofline': loss_roof,
            'block_roofline': block_roof,
            'cpu_baseline': cpu,
            'loss_per_dcnt': {k: v / max(stats.get('dcnt', 1.0), 1e-9) for k, v in stats.items()
                              if k in ('p', 'v', 'ent', 'total')},
        }
        if cpu is not None:
            line['speedup_vs_cpu_baseline'] = round(value / cpu['value'], 1)
        if t9 is not None:
            line['secondary'] = t9
        if ro is not None:
            line['rollout'] = ro
        if gro is not None:
            line['geister_rollout'] = gro
        if gle is not None:
            line['geister_learner'] = gle
        if gee is not None:
            line['geese_learner'] = gee
        if hro is not None:
            line['host_rollout'] = hro
        if pro is not None:
            line['player_rollout'] = pro
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
