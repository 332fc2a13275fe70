#!/bin/bash
# round 6: PMC passes over the block backward, two-workgroup form 2 vs tile-shared form 1 (standalone, random data)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
out=gpurun_out/r6e
mkdir -p $out
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_COUNT GRBM_GUI_ACTIVE"
P2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VMEM SQ_INSTS_VALU SQ_INSTS_MFMA SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA"
P3="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_MISC"
for f in 2 1; do
  i=0
  for P in "$P1" "$P2" "$P3"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d $out/b${f}_p$i -o run -- python3 tools/conv_pmc.py bwd $f --iters 10 > $out/b${f}_p$i.log 2>&1 || { echo "pass $f $i failed"; tail -5 $out/b${f}_p$i.log; exit 1; }
    c=$(ls $out/b${f}_p$i/*counter_collection.csv | head -1)
    k=$([ "$f" = "2" ] && echo conv3x3_block_bwd4_kernel || echo conv3x3_block_bwd2_kernel)
    python3 tools/pmc_avg.py $c $k >> $out/summary.txt
    rm -f $c
  done
done
cat $out/summary.txt
