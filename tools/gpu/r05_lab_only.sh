#!/bin/bash
# attention lab timings only: tools/gpu/r05_lab_only.sh OUT SHAPES ARMS
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 240 tools/lab/attn_lab 5 "$2" "$3" > $O/lab.txt 2>&1; rc=$?
cat $O/lab.txt; exit $rc
