#!/bin/bash
# GPU-box profiling of the bench: kernel trace + stats, and the scan's HBM traffic (separate PMC passes).
set -e
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
tag=${1:-prof}
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o run -- python3 bench.py --cpu-baseline 0 --secondary 0 > $out/bench.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out/pmc_fetch -o run -- python3 tools/scan_pmc.py > $out/pmc_fetch.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $out/pmc_write -o run -- python3 tools/scan_pmc.py > $out/pmc_write.log 2>&1
# summaries on the box (the raw traces exceed gpurun's 64 MiB copy-back)
tr=$(ls $out/trace/*kernel_trace.csv | head -1)
python3 tools/prof_summary.py $tr per:FusedAdam > $out/step_kernels.md
python3 tools/kernel_by_grid.py $tr targets_kernel > $out/scan_by_grid.md
python3 tools/step_sequence.py $tr --marker FusedAdam > $out/step_sequence.txt || true
python3 tools/pmc_summary.py $(ls $out/pmc_fetch/*counter_collection.csv | head -1) targets_kernel > $out/pmc_fetch.txt
python3 tools/pmc_summary.py $(ls $out/pmc_write/*counter_collection.csv | head -1) targets_kernel > $out/pmc_write.txt
rm -f $out/trace/*kernel_trace.csv $out/pmc_*/*.csv.bak
du -sh $out
