# Same-box A/B of two library builds (ZV_LIB_PATH): per-shape forward profiles
# and full-step wall time, alternating A, B, A, B.
set -o pipefail
mkdir -p gpurun_out/ablib
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "decoder_forward or sample_c1 or sample_batch" > gpurun_out/ablib/pytest.log 2>&1 && \
for r in 1 2; do
  for v in a b; do
    lib=zipvoice_amd/libzipvoice_hip.so; [ $v = a ] && lib=zipvoice_amd/libzipvoice_hip_a.so
    ZV_LIB_PATH=$PWD/$lib timeout -k 10 200 python -u tools/profile_forward.py --report --iters 3 > gpurun_out/ablib/forward_${v}_$r.txt 2>&1 || exit 1
  done
done
