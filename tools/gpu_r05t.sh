#!/bin/bash
# Round-5 A/B: staged pass workgroup sizes (column passes 512 / 1024, row passes 512) vs 256
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 99
bash tools/ab_rep.sh r05t5 256,256,6,12 2 libwst_hip.so var_bc512.so var_bc1024.so var_br512.so || exit 99
