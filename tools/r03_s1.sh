set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03s1
timeout -k 10 300 python3 tools/kernel_ms.py 3072 2048 1536 1024 768 512 > gpurun_out/r03s1/chunk_nt.txt 2>&1 && \
WST_LIB=var_nont.so timeout -k 10 300 python3 tools/kernel_ms.py 3072 2048 1536 1024 768 512 > gpurun_out/r03s1/chunk_nont.txt 2>&1
rc=$?
cat gpurun_out/r03s1/chunk_nt.txt gpurun_out/r03s1/chunk_nont.txt
exit $rc
