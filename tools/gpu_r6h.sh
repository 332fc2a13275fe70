#!/bin/bash
# round 6: fw3 with the stage interleaved into the MFMA stream (FW3_VARIANT 4; 5 = 4 + y stores by lane 0 only):
# bit-exactness of y against forms 0/1 under the variant library, then the standalone timings
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
out=gpurun_out/r6h
mkdir -p $out
HRL_LIB_PATH=tools/variants/libhrl_fw3_v4.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  "tests/test_bn_gpu.py::test_tile_shared_forward_matches_per_wave_conv" > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -2 $out/tests.log
timeout -k 10 120 python3 tools/fwd_bench.py --forms 2 >> $out/fwd.jsonl 2>> $out/fwd.err || { tail -20 $out/fwd.err; exit 1; }
for v in 4 5; do
  HRL_LIB_PATH=tools/variants/libhrl_fw3_v$v.so timeout -k 10 120 python3 tools/fwd_bench.py --forms 2 >> $out/fwd.jsonl 2>> $out/fwd.err || { tail -20 $out/fwd.err; exit 1; }
done
cat $out/fwd.jsonl
