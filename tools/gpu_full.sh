#!/bin/bash
# the whole GPU test suite (one process), smoke, and the bench line: bash tools/gpu_full.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
out=gpurun_out/$1
mkdir -p $out
timeout -k 10 1500 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests > $out/gputests.log 2>&1; rc=$?
tail -5 $out/gputests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { tail -20 $out/smoke.log; exit 1; }
tail -2 $out/smoke.log
timeout -k 10 400 python3 bench.py > $out/bench.log 2>&1 || { tail -20 $out/bench.log; exit 1; }
tail -1 $out/bench.log | cut -c1-300
