#!/bin/bash
# round 5: the new kernels' GPU tests (ABI 19, heads / stem backward forms, step tail, bench-size Geister parity),
# the learner parity tests, a kernel trace of the bench for the per-replay gap analysis, then PMC passes
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
out=gpurun_out/r5a
mkdir -p $out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_abi.py \
  tests/test_optim_gpu.py "tests/test_bn_gpu.py::test_heads_backward_forms_agree" \
  "tests/test_bn_gpu.py::test_fused_heads_match_torch_cpu" "tests/test_bn_gpu.py::test_stem_conv_matches_torch_cpu" \
  "tests/test_bn_gpu.py::test_block_backward_matches_unfused_launches" \
  "tests/test_bn_gpu.py::test_tile_shared_forward_matches_per_wave_conv" \
  tests/test_learner_gpu.py tests/test_gboard_gpu.py \
  "tests/test_geister.py::test_recurrent_learner_step_at_bench_size_vs_oracle" \
  > $out/tests.log 2>&1 || { tail -60 $out/tests.log; exit 1; }
tail -3 $out/tests.log
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $out/trace -o run -- python3 bench.py --cpu-baseline 0 --secondary 0 > $out/bench.log 2>&1 || { tail -20 $out/bench.log; exit 1; }
tr=$(ls $out/trace/*kernel_trace.csv | head -1)
python3 tools/replay_gaps.py $tr --marker adam_clip_kernel --skip 4 --count 20 > $out/replay_gaps.txt
rm -f $tr
head -30 $out/replay_gaps.txt
tail -1 $out/bench.log | cut -c1-400
for ab in "hrl_conv3x3_set_fwd_form 2,3,2,3" "hrl_heads_set_bwd_form 1,2,1,2" "hrl_stem_set_wgrad_form 1,2,1,2"; do
  set -- $ab
  timeout -k 10 300 python3 tools/form_ab.py --setter $1 --forms $2 >> $out/form_ab.jsonl 2>> $out/form_ab.err || { tail -5 $out/form_ab.err; exit 1; }
done
cat $out/form_ab.jsonl
