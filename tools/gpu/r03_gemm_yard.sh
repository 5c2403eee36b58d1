#!/bin/bash
# GEMM lab (256x256 vs 128x128 on the model shapes) + the hipBLASLt yardstick, same box.
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/yard; mkdir -p $O
timeout -k 10 200 tools/lab/gemm_lab 5 9,3,1,2,6 > $O/gemm_lab.txt 2>&1 && \
timeout -k 10 200 python -u tools/torch_gemm_ref.py > $O/torch_gemm.txt 2>&1
rc=$?; cat $O/gemm_lab.txt $O/torch_gemm.txt; exit $rc
