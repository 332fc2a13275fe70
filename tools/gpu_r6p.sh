#!/bin/bash
# round 6: heads backward with two 8-row groups in flight -- parity tests, then old vs new build standalone
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
out=gpurun_out/r6p
mkdir -p $out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_bn_gpu.py -k "heads" > $out/test.log 2>&1 || { tail -30 $out/test.log; exit 1; }
tail -2 $out/test.log
for r in 1 2 3; do
  HRL_LIB_PATH=tools/variants/libhrl_heads_old.so timeout -k 10 120 python -u tools/heads_bwd_bench.py --iters 100 >> $out/bench.log 2>&1 || { tail -20 $out/bench.log; exit 1; }
  timeout -k 10 120 python -u tools/heads_bwd_bench.py --iters 100 >> $out/bench.log 2>&1 || { tail -20 $out/bench.log; exit 1; }
done
grep '^{' $out/bench.log
timeout -k 10 300 python -u tools/fold_bench.py --rounds 1 > $out/step.log 2>&1 || { tail -20 $out/step.log; exit 1; }
grep '^{' $out/step.log
