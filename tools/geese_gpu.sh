set -e
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
out=gpurun_out/$1
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_geese.py tests/test_geese_golden.py -m gpu -x -v --timeout 120 --timeout-method thread > $out/gputests.log 2>&1
timeout -k 10 300 python -u tools/geese_bench.py --B 2048 --T 64 --graph 1 > $out/geese_bench.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o run -- python3 tools/geese_bench.py --B 2048 --T 64 --graph 1 --steps 3 --warmup 2 > $out/geese_prof.log 2>&1
cp $out/trace/*kernel_stats.csv $out/ 2>/dev/null || true
rm -f $out/trace/*kernel_trace.csv
