#!/bin/bash
# GPU-box kernel trace of the device self-play (GPU kernel time vs wall): bash tools/profile_rollout.sh TAG [env] [games]
set -e
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
tag=${1:-ro}; env=${2:-geister}; games=${3:-2048}
out=gpurun_out/$tag
mkdir -p $out
trap 'rm -f $out/trace/*kernel_trace.csv' EXIT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o run -- python3 tools/rollout_bench.py --env $env --games $games --reps 1 > $out/bench.log 2>&1
tr=$(ls $out/trace/*kernel_trace.csv | head -1)
python3 tools/prof_summary.py $tr 1 > $out/summary.md
