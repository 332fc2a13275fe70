#!/bin/bash
# round 6: finalize folding A/B (tools/fold_bench.py) and its bit-identity tests
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
out=gpurun_out/r6n
mkdir -p $out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_bn_gpu.py -k "fold or chain" > $out/test.log 2>&1 || { tail -30 $out/test.log; exit 1; }
tail -2 $out/test.log
timeout -k 10 300 python -u tools/fold_bench.py --rounds 3 > $out/fold.log 2>&1 || { tail -20 $out/fold.log; exit 1; }
timeout -k 10 300 python -u tools/fold_bench.py --rounds 2 --fwd-form 3 >> $out/fold.log 2>&1 || { tail -20 $out/fold.log; exit 1; }
grep '^{' $out/fold.log
