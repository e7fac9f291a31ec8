#!/bin/bash
# c5 phase ablation of the order-2 kernels (diagnostic build) + c2 for reference
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 99
WST_KM_GEOM=256,256,6,12 timeout -k 10 500 python3 tools/ablate.py full no_o2_fold no_o2_ifft no_o2_lowpass no_order2_paths o2_only_load no_o2_fold_s2 no_o2_fold_box > gpurun_out/r05n_c5_ablate.txt 2>&1 || { tail -5 gpurun_out/r05n_c5_ablate.txt; exit 99; }
cat gpurun_out/r05n_c5_ablate.txt
