#!/bin/bash
# f3 exported-spectrum k_o2: default one workgroup per item vs an item's batches split over
# workgroups of one XCD (diag build env knobs WST_O2X_SPLIT / WST_O2X_GROUP): time + L2 / wave PMC.
# usage (GPU box): tools/f3_split.sh <tag>     needs <pkg>/libwst_hip_diag.so (make EXTRA=-DWST_DIAG ...)
tag=$1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 99
o=gpurun_out/${tag}_f3split; mkdir -p $o
run() {  # name, env...
  name=$1; shift
  env "$@" AB_LIB=libwst_hip_diag.so WST_KM_GEOM=768,128,2 timeout -k 10 200 python3 tools/kernel_ms.py 1536 > $o/$name.time 2>&1 || { echo "$name time failed"; tail -5 $o/$name.time; exit 99; }
  echo "$name $(tail -1 $o/$name.time)"
  i=0
  for pass in "TCC_HIT_sum TCC_MISS_sum SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU" \
              "FETCH_SIZE SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_WAIT_INST_ANY"; do
    i=$((i+1))
    env "$@" AB_LIB=libwst_hip_diag.so timeout -s KILL 120 rocprofv3 --pmc $pass --output-format csv -d $o/${name}_p$i -o pmc -- python3 tools/time_c2.py --B 256 --C 3 --M 128 --J 2 --L 8 --iters 1 > $o/${name}_p$i.log 2>&1 || { echo "$name pmc $i failed"; tail -5 $o/${name}_p$i.log; exit 99; }
  done
  python3 tools/pmc_summary.py $o/${name}_p1 > $o/${name}_summary.txt
  python3 tools/pmc_summary.py $o/${name}_p2 >> $o/${name}_summary.txt
  grep -A12 "k_o2<17" $o/${name}_summary.txt | grep -E "==|TCC|WAVES|WAIT|FETCH|BUSY|VMEM|LDS_BANK" | head -24
}
run default WST_DUMMY=0
run split4g8 WST_O2X_SPLIT=4 WST_O2X_GROUP=8
run split2g8 WST_O2X_SPLIT=2 WST_O2X_GROUP=8
