#!/bin/bash
# Fused FF weight-DMA issue slots (FFN_DMA_K0..3, lab builds tools/lab/ffn_lab_{d,e,m,f}: 1/17/33/49,
# 1/3/5/7, 1/9/17/25, 1/5/9/13), two rounds interleaved, plus the MX-fp8 adder probe.
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/ffn_dma; mkdir -p $O
timeout -k 10 60 tools/probe/mx8_align > $O/mx8_align.txt 2>&1 || { cat $O/mx8_align.txt; exit 1; }
for r in 1 2; do
  for v in d e m f; do
    echo "== $v round $r"
    timeout -k 10 150 tools/lab/ffn_lab_$v 5 1 > $O/lab_${v}_$r.txt 2>&1 || { tail -5 $O/lab_${v}_$r.txt; exit 1; }
    grep "M=" $O/lab_${v}_$r.txt | sed 's/|fused-unfused|.*unfused/unfused/'
  done
done
