#!/bin/bash
# round 6 final tree: rocprofv3 --kernel-trace --stats of bench.py under the driver's arguments
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
out=gpurun_out/r6s
mkdir -p $out
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > $out/bench.log 2>&1 || { tail -20 $out/bench.log; exit 1; }
st=$(ls $out/prof/*kernel_stats.csv | head -1)
cp $st $out/kernel_stats.csv
rm -f $out/prof/*kernel_trace.csv
grep '^{' $out/bench.log | cut -c1-300
head -12 $out/kernel_stats.csv | cut -d, -f1-4
