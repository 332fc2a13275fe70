#!/bin/bash
# round 6: the output-mask kernels with 32-bit indices -- parity (learner GPU tests), then the step and its kernels
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
out=gpurun_out/r6q
mkdir -p $out
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_learner_gpu.py > $out/test.log 2>&1 || { tail -30 $out/test.log; exit 1; }
tail -2 $out/test.log
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $out/trace -o run -- python3 bench.py --steps 60 --warmup 30 --cpu-baseline 0 --secondary 0 > $out/prof.log 2>&1 || { tail -20 $out/prof.log; exit 1; }
tr=$(ls $out/trace/*kernel_trace.csv | head -1)
python3 tools/replay_gaps.py $tr --marker adam_clip_kernel --skip 33 --count 40 > $out/replay.txt || exit 1
rm -f $tr
tail -28 $out/replay.txt
