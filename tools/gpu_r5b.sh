#!/bin/bash
# round 5: PMC passes over the chain's ring forward (fwd form 2) and the tile-shared block backward (bwd form 1),
# standalone launches on random data (tools/conv_pmc.py): where a tile's cycles go
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
out=gpurun_out/r5b
mkdir -p $out
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_COUNT GRBM_GUI_ACTIVE"
P2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VMEM SQ_INSTS_VALU SQ_INSTS_MFMA SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA"
P3="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_MISC"
for which in "fwd 2" "bwd 1"; do
  tag=$(echo $which | tr ' ' '_')
  i=0
  for P in "$P1" "$P2" "$P3"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d $out/${tag}_p$i -o run -- python3 tools/conv_pmc.py $which --iters 10 > $out/${tag}_p$i.log 2>&1 || { echo "pass $tag $i failed"; tail -5 $out/${tag}_p$i.log; exit 1; }
    f=$(ls $out/${tag}_p$i/*counter_collection.csv | head -1)
    k=$([ "$tag" = "fwd_2" ] && echo conv3x3_fwd_dma_kernel || echo conv3x3_block_bwd2_kernel)
    python3 tools/pmc_avg.py $f $k >> $out/summary.txt
    rm -f $f
  done
done
cat $out/summary.txt
