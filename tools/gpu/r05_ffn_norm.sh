#!/bin/bash
# Round-5 FF3 + BiasNorm epilogue A/B, same box: the previous kernel (tools/lab/ffn_lab_old*,
# built from the previous commit's zv_ffn.inc) against the tree's, normal and FFN_TIMING builds
# (epilogue clk per item), then optionally the GPU suite + bench (r05_val.sh).
#   tools/gpu/r05_ffn_norm.sh OUT [VAL=0|1]
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r05_ffn_norm}; mkdir -p $O
SH="6528x1920;13056x1920;26112x1920;52224x1920;78016x1920"
for b in ffn_lab_old ffn_lab; do
  echo "== $b"
  timeout -k 10 200 ./tools/lab/$b 5 8 "$SH" 0 "classic,pers" > $O/$b.txt 2>&1 || { echo "lab rc=$?"; tail -20 $O/$b.txt; exit 1; }
  cat $O/$b.txt
done
for b in ffn_lab_old_tim ffn_lab_tim; do
  echo "== $b"
  timeout -k 10 200 ./tools/lab/$b 2 8 "$SH" 0 "pers" > $O/$b.txt 2>&1 || { echo "lab rc=$?"; tail -20 $O/$b.txt; exit 1; }
  grep -E "timing|items" $O/$b.txt
done
[ "${2:-0}" = 1 ] || exit 0
bash tools/gpu/r05_val.sh "${1:-r05_ffn_norm}/val"
