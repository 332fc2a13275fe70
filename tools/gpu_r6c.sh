#!/bin/bash
# round 6: block form 2 with the per-CU stagger of the later workgroup (HRL_BB4_STAGGER = s_sleep(32) count)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
out=gpurun_out/r6c
mkdir -p $out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  "tests/test_bn_gpu.py::test_block_backward_matches_unfused_launches" > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -2 $out/tests.log
for st in 0 1 2 3 4 6 8; do
  HRL_BB4_STAGGER=$st timeout -k 10 120 python3 tools/block_bench.py --iters 50 --epi 2 --forms 2 | sed "s/^/{\"stagger\": $st} /" >> $out/bb.jsonl 2>> $out/bb.err || { tail -20 $out/bb.err; exit 1; }
done
cat $out/bb.jsonl
