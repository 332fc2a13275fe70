#!/bin/bash
# round 6, final tree: PMC traffic (FETCH_SIZE / WRITE_SIZE passes, gfx950-corrected) of the block backward (form 1),
# the ring forward (fwd form 2) and the scan; the bench under a kernel trace (per-replay kernels and gaps) and under
# --stats; the bench with the driver's own arguments
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
out=gpurun_out/r6i
mkdir -p $out
pmc() {   # pmc TAG COUNTER CMD...
  local tag=$1 ctr=$2; shift 2
  timeout -s KILL 90 rocprofv3 --pmc $ctr --output-format csv -d $out/$tag -o run -- "$@" > $out/$tag.log 2>&1 || { echo "pmc $tag failed"; tail -5 $out/$tag.log; return 1; }
  ls $out/$tag/*counter_collection.csv | head -1
}
fb=$(pmc blk_fetch FETCH_SIZE python3 tools/conv_pmc.py bwd 1 --iters 10) && wb=$(pmc blk_write WRITE_SIZE python3 tools/conv_pmc.py bwd 1 --iters 10) || exit 1
python3 tools/pmc_bytes.py conv3x3_block_bwd2_kernel 603979776 $fb $wb --label "block form 1, tools/conv_pmc.py bwd 1, M=131072" > $out/r06_block_pmc.json || exit 1
ff=$(pmc fwd_fetch FETCH_SIZE python3 tools/conv_pmc.py fwd 2 --iters 10) && wf=$(pmc fwd_write WRITE_SIZE python3 tools/conv_pmc.py fwd 2 --iters 10) || exit 1
python3 tools/pmc_bytes.py conv3x3_fwd_dma_kernel 301989888 $ff $wf --label "fwd form 2, tools/conv_pmc.py fwd 2, M=131072" > $out/r06_fwd_pmc.json || exit 1
fs=$(pmc scan_fetch FETCH_SIZE python3 tools/scan_pmc.py) && ws=$(pmc scan_write WRITE_SIZE python3 tools/scan_pmc.py) || exit 1
python3 tools/scan_pmc_json.py $fs $ws > $out/r06_scan_pmc.json || exit 1
rm -f $out/*/*counter_collection.csv
cat $out/r06_block_pmc.json $out/r06_fwd_pmc.json
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $out/trace -o run -- python3 bench.py --cpu-baseline 0 --secondary 0 > $out/bench_under_trace.log 2>&1 || { tail -20 $out/bench_under_trace.log; exit 1; }
tr=$(ls $out/trace/*kernel_trace.csv | head -1)
python3 tools/replay_gaps.py $tr --marker adam_clip_kernel --skip 4 --count 40 > $out/replay_gaps.txt
rm -f $tr
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/stats -o run -- python3 bench.py --cpu-baseline 0 --secondary 0 > $out/bench_under_stats.log 2>&1 || { tail -20 $out/bench_under_stats.log; exit 1; }
cp $(ls $out/stats/*kernel_stats.csv | head -1) $out/bench_kernel_stats.csv
rm -f $out/stats/*kernel_trace.csv
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $out/bench_driver_args.log 2>&1 || { tail -20 $out/bench_driver_args.log; exit 1; }
tail -1 $out/bench_driver_args.log | cut -c1-300
head -45 $out/replay_gaps.txt | tail -30
