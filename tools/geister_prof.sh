#!/bin/bash
# Geister learner (B=256, T=16, HIP graph) timing and rocprofv3 kernel statistics.
#   bash tools/geister_prof.sh TAG
set -e
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
out=gpurun_out/$1
mkdir -p $out
timeout -k 10 300 python -u tools/geister_bench.py --B 256 --T 16 --graph 1 > $out/bench.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o run -- python3 tools/geister_bench.py --B 256 --T 16 --graph 1 --steps 3 --warmup 2 > $out/prof.log 2>&1
cp $out/trace/*kernel_stats.csv $out/ 2>/dev/null || true
rm -f $out/trace/*kernel_trace.csv
