#!/bin/bash
# round 6: bench.py after its JSON gained the timing note (driver arguments)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
out=gpurun_out/r6t
mkdir -p $out
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $out/bench.log 2>&1 || { tail -20 $out/bench.log; exit 1; }
grep '^{' $out/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['timing_note'][:60], sorted(d)[:40])"
