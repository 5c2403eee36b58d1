#!/bin/bash
# Fused FeedForward lab (tools/lab/ffn_lab): fused vs unfused FF on the model's shapes.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/ffn
timeout -k 10 150 tools/lab/ffn_lab ${1:-5} ${2:-1,2,4} > gpurun_out/ffn/lab.txt 2>&1
rc=$?; cat gpurun_out/ffn/lab.txt; exit $rc
