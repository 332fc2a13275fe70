#!/bin/bash
# round 6 final tree: the whole GPU suite, smoke(), bench.py under the driver's arguments and with its defaults
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
out=gpurun_out/r6z
mkdir -p $out
timeout -k 10 840 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > $out/gpu_tests.log 2>&1
rc=$?
grep -E "FAILED|ERROR" $out/gpu_tests.log | head -20
tail -2 $out/gpu_tests.log
# 1 = some tests failed (the GPU is fine: go on); anything else (timeout, crash) ends the call here
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 240 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $out/smoke.log 2>&1 || { tail -20 $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $out/bench_driver_args.log 2>&1 || { tail -20 $out/bench_driver_args.log; exit 1; }
grep '^{' $out/bench_driver_args.log | cut -c1-400
