# Pair-residual stream (bf16 mode): all GPU tests, same-box forward profiles
# pair vs fp32 stream, then the bench line.
set -o pipefail
mkdir -p gpurun_out/pair
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pair/pytest.log 2>&1 && \
timeout -k 10 200 python -u tools/profile_forward.py --report --iters 3 > gpurun_out/pair/fwd_pair.txt 2>&1 && \
ZV_PAIR_RESID=0 timeout -k 10 200 python -u tools/profile_forward.py --report --iters 3 > gpurun_out/pair/fwd_f32.txt 2>&1 && \
timeout -k 10 200 python -u tools/profile_forward.py --report --iters 3 > gpurun_out/pair/fwd_pair2.txt 2>&1 && \
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-fp32-mode > gpurun_out/pair/bench.json 2> gpurun_out/pair/bench.err
