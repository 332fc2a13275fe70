#!/bin/bash
# round 6: the LDS-staged ring forward's (fwd form 3) diagnostic variants (tools/fw5_variants.sh), standalone
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
out=gpurun_out/r6l
mkdir -p $out
timeout -k 10 120 python -u tools/fwd_bench.py --forms 2,3,2,3 --iters 100 > $out/fwd.log 2>&1 || { tail -20 $out/fwd.log; exit 1; }
for v in ${VARIANTS:-1 2}; do
  HRL_LIB_PATH=tools/variants/libhrl_fw5_v$v.so timeout -k 10 120 python -u tools/fwd_bench.py --forms 3,3 --iters 100 >> $out/fwd.log 2>&1 || { tail -20 $out/fwd.log; exit 1; }
done
timeout -k 10 120 python -u tools/fwd_bench.py --forms 2,3,2,3 --iters 100 >> $out/fwd.log 2>&1 || { tail -20 $out/fwd.log; exit 1; }
grep '^{' $out/fwd.log
