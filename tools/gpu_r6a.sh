#!/bin/bash
# round 6: the two-workgroup block backward (block form 2) -- its parity tests, the step-tail fold fixes,
# the standalone block bench (forms 2 / 1 / 0), then the learner step bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
out=gpurun_out/r6a
mkdir -p $out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  "tests/test_bn_gpu.py::test_block_backward_matches_unfused_launches" \
  "tests/test_bn_gpu.py::test_block_backward_weight_gradient_exact_on_integer_data" \
  tests/test_optim_gpu.py > $out/tests.log 2>&1 || { tail -60 $out/tests.log; exit 1; }
tail -3 $out/tests.log
timeout -k 10 120 python3 tools/block_bench.py --iters 50 > $out/block_bench.json 2>&1 || { tail -20 $out/block_bench.json; exit 1; }
cat $out/block_bench.json
timeout -k 10 300 python3 bench.py --cpu-baseline 0 --secondary 0 > $out/bench.log 2>&1 || { tail -20 $out/bench.log; exit 1; }
tail -1 $out/bench.log | cut -c1-600
