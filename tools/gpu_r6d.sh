#!/bin/bash
# round 6: block form 2 without spills -- parity tests, standalone forms 2 / 1 per epilogue, stagger sweep, step bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
out=gpurun_out/r6d
mkdir -p $out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  "tests/test_bn_gpu.py::test_block_backward_matches_unfused_launches" \
  "tests/test_bn_gpu.py::test_block_backward_weight_gradient_exact_on_integer_data" > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -2 $out/tests.log
for e in 2 3; do
  timeout -k 10 120 python3 tools/block_bench.py --iters 50 --epi $e --forms 2,1 >> $out/bb.jsonl 2>> $out/bb.err || { tail -20 $out/bb.err; exit 1; }
done
for st in 2 4; do
  HRL_BB4_STAGGER=$st timeout -k 10 120 python3 tools/block_bench.py --iters 50 --epi 2 --forms 2 | sed "s/^/{\"stagger\": $st} /" >> $out/bb.jsonl 2>> $out/bb.err || { tail -20 $out/bb.err; exit 1; }
done
cat $out/bb.jsonl
timeout -k 10 300 python3 bench.py --cpu-baseline 0 --secondary 0 > $out/bench.log 2>&1 || { tail -20 $out/bench.log; exit 1; }
tail -1 $out/bench.log | cut -c1-300
