# A/B: co-resident block stagger on the residual-linear GEMM (persistent grid and
# one tile per block), GEMM microbench, resid output mode.
set -o pipefail
OUT=gpurun_out/stagger; mkdir -p $OUT
SH="78016x512x1536;78016x512x512;78016x512x1920"
for st in 0 2 4 7; do
  ZV_GEMM_STAGGER=$st timeout -k 10 120 python -u tools/bench_gemm.py 0,100 2,4 "$SH" > $OUT/st$st.log 2>&1 || exit 1
done
