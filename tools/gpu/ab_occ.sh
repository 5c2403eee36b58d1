# Same-box A/B: baseline library (a) vs current build under GEMM occupancy policies.
set -o pipefail
mkdir -p gpurun_out/abocc
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "decoder_forward or sample_c1 or sample_batch" > gpurun_out/abocc/pytest.log 2>&1 && \
timeout -k 10 200 python -u -m pytest tests/test_gpu_fbank.py -x -v -s --timeout 120 --timeout-method thread > gpurun_out/abocc/pytest_fbank.log 2>&1 ; \
for r in 1 2; do
  ZV_LIB_PATH=$PWD/zipvoice_amd/libzipvoice_hip_a.so timeout -k 10 200 python -u tools/profile_forward.py --report --iters 3 > gpurun_out/abocc/fwd_a_$r.txt 2>&1 || exit 1
  timeout -k 10 200 python -u tools/profile_forward.py --report --iters 3 > gpurun_out/abocc/fwd_b1_$r.txt 2>&1 || exit 1
  ZV_GEMM_OCC_PLAIN=2 timeout -k 10 200 python -u tools/profile_forward.py --report --iters 3 > gpurun_out/abocc/fwd_b2_$r.txt 2>&1 || exit 1
  ZV_GEMM_OCC_FUSED=2 timeout -k 10 200 python -u tools/profile_forward.py --report --iters 3 > gpurun_out/abocc/fwd_b3_$r.txt 2>&1 || exit 1
done
