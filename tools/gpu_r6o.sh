#!/bin/bash
# round 6: which kernels run slow in the first graph replays after the capture (bench.py under the driver's warmup)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
out=gpurun_out/r6o
mkdir -p $out
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $out/trace -o run -- python3 bench.py --steps 60 --warmup 5 --cpu-baseline 0 --secondary 0 > $out/prof.log 2>&1 || { tail -20 $out/prof.log; exit 1; }
tr=$(ls $out/trace/*kernel_trace.csv | head -1)
python3 tools/replay_kernels.py $tr --skip 3 --early 0:5 --late 45:55 > $out/early_late.txt || exit 1
python3 tools/replay_gaps.py $tr --marker adam_clip_kernel --skip 3 --count 62 > $out/replay.txt || exit 1
rm -f $tr
cat $out/early_late.txt
head -70 $out/replay.txt | cut -c1-70
