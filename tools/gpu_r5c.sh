#!/bin/bash
# round 5: step-tail fold coalescing + in-tail running statistics: GPU tests, the bench under a kernel trace
# (per-replay gaps), heads / stem form A/B with fold deferral following the form, a plain bench line, then the
# PMC passes of tools/gpu_r5b.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
out=gpurun_out/r5c
mkdir -p $out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_abi.py \
  tests/test_optim_gpu.py tests/test_learner_gpu.py "tests/test_bn_gpu.py::test_heads_backward_forms_agree" \
  "tests/test_bn_gpu.py::test_stem_conv_matches_torch_cpu" \
  "tests/test_geister.py::test_recurrent_learner_step_at_bench_size_vs_oracle" \
  > $out/tests.log 2>&1 || { tail -60 $out/tests.log; exit 1; }
tail -3 $out/tests.log
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $out/trace -o run -- python3 bench.py --cpu-baseline 0 --secondary 0 > $out/bench_trace.log 2>&1 || { tail -20 $out/bench_trace.log; exit 1; }
tr=$(ls $out/trace/*kernel_trace.csv)
python3 tools/replay_gaps.py $tr --marker adam_clip_kernel --skip 4 --count 20 > $out/replay_gaps.txt
rm -f $tr
head -24 $out/replay_gaps.txt
for ab in "hrl_heads_set_bwd_form 1,2,1,2" "hrl_stem_set_wgrad_form 1,2,1,2"; do
  set -- $ab
  timeout -k 10 300 python3 tools/form_ab.py --setter $1 --forms $2 >> $out/form_ab.jsonl 2>> $out/form_ab.err || { tail -5 $out/form_ab.err; exit 1; }
done
cat $out/form_ab.jsonl
timeout -k 10 300 python3 bench.py > $out/bench.log 2>&1 || { tail -20 $out/bench.log; exit 1; }
tail -1 $out/bench.log | cut -c1-600
bash tools/gpu_r5b.sh
