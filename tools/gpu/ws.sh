# Wave-specialised residual GEMM: equivalence vs the plain kernel, same-box forward A/B (all residual linears on ws vs none).
set -o pipefail
OUT=gpurun_out/ws
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_resid_ws.py -x -v -s --timeout 120 --timeout-method thread > $OUT/pytest_ws.log 2>&1 && \
ZV_RESID_WS=2 timeout -k 10 200 python -u tools/profile_forward.py --report --iters 3 > $OUT/fwd_ws2.txt 2>&1 && \
ZV_RESID_WS=0 timeout -k 10 200 python -u tools/profile_forward.py --report --iters 3 > $OUT/fwd_ws0.txt 2>&1
