# A/B of GEMM tile policies on the same box: parity subset, per-shape forward
# profile per ZV_GEMM_TILE, GEMM microbench of tile variants.
set -o pipefail
mkdir -p gpurun_out/ab
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "decoder_forward or sample_c1" > gpurun_out/ab/pytest.log 2>&1 && \
for t in 0 1 2 3; do
  ZV_GEMM_TILE=$t timeout -k 10 200 python -u tools/profile_forward.py --report > gpurun_out/ab/forward_tile$t.txt 2>&1 || exit 1
done && \
timeout -k 10 300 python -u tools/bench_gemm.py 0,2,3,8 1,2 "78016x1536x512;78016x512x1536;78016x1024x512;78016x512x512;78016x512x48;39040x1920x512" > gpurun_out/ab/gemm_variants.txt 2>&1
