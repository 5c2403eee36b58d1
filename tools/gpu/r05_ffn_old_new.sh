#!/bin/bash
# Same-box A/B of the fused FeedForward kernel and engine against the previous commit's build
# (tools/lab/ffn_lab_old, tools/lab/old/libzipvoice_hip.so, built from `git archive HEAD~N`).
#   tools/gpu/r05_ffn_old_new.sh OUT AB_ROUNDS "ENV_NEW..."
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r05_ffn_on}; mkdir -p $O
SH="6528x1536;13056x1536;26112x1536;52224x1536"
for b in ffn_lab_old ffn_lab; do
  echo "== $b"
  timeout -k 10 200 ./tools/lab/$b 5 1,8 "$SH" 0 "unfused,classic,pers" > $O/$b.txt 2>&1 || { echo "lab rc=$?"; tail -20 $O/$b.txt; exit 1; }
  grep -v "^M=" $O/$b.txt
done
[ "${2:-0}" -gt 0 ] || exit 0
bash tools/gpu/ab_env.sh "${1:-r05_ffn_on}/ab" "$2" "ZV_LIB_PATH=tools/lab/old/libzipvoice_hip.so" "${3:-ZV_FFN_SPLIT=0}"
