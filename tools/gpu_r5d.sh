#!/bin/bash
# round 5: lane-per-channel stem forward, heads forward / backward occupancy and prefetch, 16-wave folds: GPU tests,
# a kernel trace of the bench (per-replay gaps and the step's kernel list), stem forward A/B, the heads forms'
# first-step gradient difference, a plain bench line
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
out=gpurun_out/r5d
mkdir -p $out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_abi.py \
  tests/test_optim_gpu.py tests/test_learner_gpu.py tests/test_bn_gpu.py \
  "tests/test_geister.py::test_recurrent_learner_step_at_bench_size_vs_oracle" \
  > $out/tests.log 2>&1 || { tail -60 $out/tests.log; exit 1; }
tail -3 $out/tests.log
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $out/trace -o run -- python3 bench.py --cpu-baseline 0 --secondary 0 > $out/bench_trace.log 2>&1 || { tail -20 $out/bench_trace.log; exit 1; }
tr=$(ls $out/trace/*kernel_trace.csv)
python3 tools/replay_gaps.py $tr --marker adam_clip_kernel --skip 4 --count 20 > $out/replay_gaps.txt
rm -f $tr
sed -n '21,60p' $out/replay_gaps.txt
timeout -k 10 300 python3 tools/form_ab.py --setter hrl_stem_set_fwd_form --forms 1,2,1,2 >> $out/form_ab.jsonl 2>> $out/form_ab.err || { tail -5 $out/form_ab.err; exit 1; }
cat $out/form_ab.jsonl
timeout -k 10 300 python3 tools/diag_forms.py --setter hrl_heads_set_bwd_form --forms 1,2 --steps 12 > $out/diag_forms.txt 2>&1 || { tail -5 $out/diag_forms.txt; exit 1; }
cat $out/diag_forms.txt
timeout -k 10 300 python3 bench.py > $out/bench.log 2>&1 || { tail -20 $out/bench.log; exit 1; }
tail -1 $out/bench.log | cut -c1-400
