#!/bin/bash
# f3 (reference geometry 128^2 J=2): parity, kernel timing, LDS bank-conflict counters (dev)
tag=$1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 99
mkdir -p gpurun_out/$tag
tools/gpu_step.sh 600 gpurun_out/$tag/pytest.txt python3 -u -m pytest tests -m gpu -q -rs -x --timeout 120 --timeout-method thread || exit 99
tail -2 gpurun_out/$tag/pytest.txt
WST_KM_GEOM=768,128,2 timeout -k 10 200 python3 tools/kernel_ms.py 768 > gpurun_out/$tag/kms_f3.txt 2>&1 || exit 99
grep chunk gpurun_out/$tag/kms_f3.txt
timeout -k 10 200 python3 tools/kernel_ms.py 1536 > gpurun_out/$tag/kms_c2.txt 2>&1 || exit 99
grep chunk gpurun_out/$tag/kms_c2.txt
WST_KM_GEOM=768,128,2 timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY --output-format csv -d gpurun_out/$tag/pmc_f3 -o pmc -- python3 tools/kernel_ms.py 768 > gpurun_out/$tag/pmc_f3.log 2>&1 || exit 99
python3 tools/pmc_summary.py gpurun_out/$tag/pmc_f3 > gpurun_out/$tag/sq_f3.txt 2>&1
grep -E "==|LDS conflict" gpurun_out/$tag/sq_f3.txt | head -20
