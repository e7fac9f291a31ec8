#!/bin/bash
# Collect SQ counter passes for one short run (dev tool).  usage: tools/pmc.sh <tag> [cmd...]
# Each pass is a separate rocprofv3 --pmc run (no tracing domains combined with --pmc).
tag=$1; shift
cmd=${@:-python3 tools/time_c2.py --iters 1}
out=gpurun_out/pmc_$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
i=0
for pass in \
  "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_SALU SQ_INSTS_LDS" \
  "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES" \
  "SQ_INSTS_VMEM_RD SQ_INSTS_LDS_LOAD SQ_INSTS_LDS_STORE SQ_LDS_UNALIGNED_STALL SQ_INSTS_BRANCH SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE" \
  "SQ_WAIT_INST_LDS SQ_LDS_ADDR_CONFLICT SQ_LDS_DATA_FIFO_FULL SQ_INSTS_SMEM SQ_ACTIVE_INST_ANY SQ_INSTS_VALU_MFMA_F32 SQ_WAVES SQ_BUSY_CYCLES" ; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $pass --output-format csv -d $out/p$i -o pmc -- $cmd > $out/p$i.log 2>&1
  rc=$?
  echo "[pmc] pass $i rc=$rc"
  if [ $rc -ne 0 ]; then tail -20 $out/p$i.log; exit 99; fi
done
python3 tools/pmc_summary.py $out | tee $out/summary.txt
