#!/bin/bash
# Round-3 validation + GEMM yardstick: every GPU test, smoke, the bench line, the GEMM lab
# (256x256 vs 128x128 kernels on the model's shapes) and the hipBLASLt yardstick, same box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/val
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 && \
tail -3 $O/pytest_gpu.log && \
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && \
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err && \
timeout -k 10 200 tools/lab/gemm_lab 5 9,3,1,2,6 > $O/gemm_lab.txt 2>&1 && \
timeout -k 10 200 python -u tools/torch_gemm_ref.py > $O/torch_gemm.txt 2>&1
echo "exit $?"
