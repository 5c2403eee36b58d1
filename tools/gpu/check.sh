# Quick validation of the current tree: every GPU test, smoke, the default bench line.
set -o pipefail
OUT=gpurun_out/check
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 && \
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && \
timeout -k 10 400 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err
