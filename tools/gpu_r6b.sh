#!/bin/bash
# round 6: where the two-workgroup block backward's time goes -- product forms 2 / 1 per epilogue, then the
# BB4_VARIANT builds (1 = no loads after the first tile, 2 = no MFMA, 4 = no epilogue, 6 = neither)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
out=gpurun_out/r6b
mkdir -p $out
for e in 2 3 0; do
  timeout -k 10 120 python3 tools/block_bench.py --iters 50 --epi $e --forms 2,1 >> $out/bb.jsonl 2>> $out/bb.err || { tail -20 $out/bb.err; exit 1; }
done
for v in 1 2 4 6; do
  HRL_LIB_PATH=tools/variants/libhrl_bb4_v$v.so timeout -k 10 120 python3 tools/block_bench.py --iters 50 --epi 2 --forms 2 >> $out/bb.jsonl 2>> $out/bb.err || { tail -20 $out/bb.err; exit 1; }
done
cat $out/bb.jsonl
