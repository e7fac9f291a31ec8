#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 99
bash tools/skip_ab.sh 768,128,2 0 8 16 64 2048 128 1 2 4 || exit 99
bash tools/skip_ab.sh 3072,64,4 0 8 16 64 || exit 99
