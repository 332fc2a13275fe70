#!/bin/bash
# round 6: the Geister recurrent learner (B=256, T=16, graph) -- timing and a kernel trace of its replays
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
out=gpurun_out/r6j
mkdir -p $out
timeout -k 10 300 python -u tools/geister_bench.py --B 256 --T 16 --graph 1 > $out/bench.log 2>&1 || { tail -20 $out/bench.log; exit 1; }
tail -2 $out/bench.log
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $out/trace -o run -- python3 tools/geister_bench.py --B 256 --T 16 --graph 1 --steps 6 --warmup 3 > $out/prof.log 2>&1 || { tail -20 $out/prof.log; exit 1; }
tr=$(ls $out/trace/*kernel_trace.csv | head -1)
python3 tools/replay_gaps.py $tr --marker adam_clip_kernel --skip 3 --count 4 > $out/replay.txt || exit 1
rm -f $tr
head -8 $out/replay.txt
