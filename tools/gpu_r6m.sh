#!/bin/bash
# round 6: the BatchNorm finalizes folded into their consumers (ABI 26) -- parity, then the step and its kernels
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
out=gpurun_out/r6m
mkdir -p $out
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_bn_gpu.py tests/test_learner_gpu.py tests/test_optim_gpu.py > $out/test.log 2>&1 || { tail -30 $out/test.log; exit 1; }
tail -3 $out/test.log
timeout -k 10 300 python -u tools/fwd_form_bench.py --forms 2,3,2,3 > $out/step.log 2>&1 || { tail -20 $out/step.log; exit 1; }
cat $out/step.log
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $out/trace -o run -- python3 bench.py --steps 40 --warmup 5 --cpu-baseline 0 --secondary 0 > $out/prof.log 2>&1 || { tail -20 $out/prof.log; exit 1; }
tr=$(ls $out/trace/*kernel_trace.csv | head -1)
python3 tools/replay_gaps.py $tr --marker adam_clip_kernel --skip 8 --count 30 > $out/replay.txt || exit 1
rm -f $tr
tail -32 $out/replay.txt
