#!/bin/bash
# round 6: the ping-pong ring forward (fwd form 3) -- parity against the other forms, standalone and in-step timing
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
out=gpurun_out/r6k
mkdir -p $out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_bn_gpu.py -k "tile_shared_forward or chain or block" > $out/test.log 2>&1 || { tail -30 $out/test.log; exit 1; }
tail -3 $out/test.log
timeout -k 10 120 python -u tools/fwd_bench.py --forms 2,3,2,3 > $out/fwd.log 2>&1 || { tail -20 $out/fwd.log; exit 1; }
cat $out/fwd.log
timeout -k 10 300 python -u tools/fwd_form_bench.py --forms 2,3,2,3 > $out/step.log 2>&1 || { tail -20 $out/step.log; exit 1; }
cat $out/step.log
