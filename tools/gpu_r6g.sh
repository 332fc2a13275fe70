#!/bin/bash
# round 6: where the chain's forward ring conv (fw3) spends its time -- product forms 2 / 1 / 0, then the FW3_VARIANT
# builds (1 = y stores by lane 0 only, 2 = no MFMAs, 3 = both)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
out=gpurun_out/r6g
mkdir -p $out
timeout -k 10 120 python3 tools/fwd_bench.py --forms 2,1,0 >> $out/fwd.jsonl 2>> $out/fwd.err || { tail -20 $out/fwd.err; exit 1; }
for v in 1 2 3; do
  HRL_LIB_PATH=tools/variants/libhrl_fw3_v$v.so timeout -k 10 120 python3 tools/fwd_bench.py --forms 2 >> $out/fwd.jsonl 2>> $out/fwd.err || { tail -20 $out/fwd.err; exit 1; }
done
cat $out/fwd.jsonl
