#!/bin/bash
# Learner step vs per-GPU batch (T=32 and T=9): one bench line per size into gpurun_out/sweep_B*.log
set -e
cd "${GRAFT_REPO_ROOT:-.}"
for T in 32 9; do
  for B in 1024 2048 4096 8192 16384; do
    timeout -k 10 200 python -u bench.py --batch $B --seq $T --cpu-baseline 0 --secondary 0 --scan-iters 50 > gpurun_out/sweep_B${B}_T${T}.log 2>&1
  done
done
