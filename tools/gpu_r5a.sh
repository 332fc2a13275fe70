#!/bin/bash
# round 5: ABI-19 tests, the new heads / stem backward forms, bench-size Geister parity; then a kernel trace of
# the bench for the per-replay gap analysis
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
out=gpurun_out/r5a
mkdir -p $out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_abi.py \
  tests/test_gboard_gpu.py "tests/test_geister.py::test_recurrent_learner_step_at_bench_size_vs_oracle" \
  "tests/test_bn_gpu.py::test_heads_backward_forms_agree" "tests/test_bn_gpu.py::test_fused_heads_match_torch_cpu" \
  "tests/test_bn_gpu.py::test_stem_conv_matches_torch_cpu" "tests/test_learner_gpu.py::test_full_size_learner_step_vs_oracle" \
  > $out/tests.log 2>&1 || { tail -40 $out/tests.log; exit 1; }
tail -3 $out/tests.log
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $out/trace -o run -- python3 bench.py --cpu-baseline 0 --secondary 0 > $out/bench.log 2>&1 || { tail -20 $out/bench.log; exit 1; }
tr=$(ls $out/trace/*kernel_trace.csv | head -1)
python3 tools/replay_gaps.py $tr --skip 4 --count 20 > $out/replay_gaps.txt
python3 tools/step_sequence.py $tr --marker FusedAdam --index 10 > $out/step_sequence.txt || true
rm -f $tr
head -30 $out/replay_gaps.txt
