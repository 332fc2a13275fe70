#!/bin/bash
# GPU tests of the round's kernels, a kernel trace of the bench (per-replay gaps and the step's kernel list), then a
# plain bench line:  bash tools/gpu_round.sh <tag> [pytest targets...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
tag=$1; shift
out=gpurun_out/$tag
mkdir -p $out
targets="${@:-tests/test_abi.py tests/test_optim_gpu.py tests/test_learner_gpu.py tests/test_bn_gpu.py}"
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu $targets \
  > $out/tests.log 2>&1 || { tail -60 $out/tests.log; exit 1; }
tail -2 $out/tests.log
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $out/trace -o run -- python3 bench.py --cpu-baseline 0 --secondary 0 > $out/bench_trace.log 2>&1 || { tail -20 $out/bench_trace.log; exit 1; }
tr=$(ls $out/trace/*kernel_trace.csv)
python3 tools/replay_gaps.py $tr --marker adam_clip_kernel --skip 30 --count 40 > $out/replay_gaps.txt
rm -f $tr
sed -n '21,60p' $out/replay_gaps.txt
timeout -k 10 300 python3 bench.py > $out/bench.log 2>&1 || { tail -20 $out/bench.log; exit 1; }
tail -1 $out/bench.log | cut -c1-300
