#!/bin/bash
# GPU-box iteration check: selected GPU tests, profiled bench (step sequence), optional extra commands.
#   bash tools/gpu_quick.sh TAG "tests/test_a.py tests/test_b.py" ["extra command" ...]
set -e
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
tag=${1:-quick}
tests=${2:-tests}
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 600 python -u -m pytest $tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/gputests.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o run -- python3 bench.py --cpu-baseline 0 --secondary 0 > $out/bench.log 2>&1
tr=$(ls $out/trace/*kernel_trace.csv | head -1)
python3 tools/step_sequence.py $tr --marker FusedAdam > $out/step_sequence.txt
python3 tools/prof_summary.py $tr per:FusedAdam > $out/step_kernels.md
rm -f $out/trace/*kernel_trace.csv
shift 2 || true
i=0
for c in "$@"; do
  i=$((i+1))
  timeout -k 10 300 bash -c "$c" > $out/extra$i.log 2>&1
done
