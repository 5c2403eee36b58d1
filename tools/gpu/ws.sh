# Wave-specialised residual GEMM (K <= 64 policy): all GPU tests, same-box bench A/B (default vs ZV_RESID_WS=0).
set -o pipefail
OUT=gpurun_out/ws
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v -s --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 && \
timeout -k 10 200 python -u tools/profile_forward.py --report --iters 3 > $OUT/fwd_ws1.txt 2>&1 && \
ZV_RESID_WS=0 timeout -k 10 200 python -u tools/profile_forward.py --report --iters 3 > $OUT/fwd_ws0.txt 2>&1 && \
timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-fp32-mode > $OUT/bench1.json 2> $OUT/bench1.err && \
ZV_RESID_WS=0 timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-fp32-mode > $OUT/bench0.json 2> $OUT/bench0.err && \
timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-fp32-mode > $OUT/bench1b.json 2> $OUT/bench1b.err
