#!/bin/bash
# Round-4 validation of the current tree: every GPU test, then smoke.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r04_final}; mkdir -p $O
echo "== pytest $(date +%T)"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { grep -E "FAIL|Error" $O/pytest_gpu.log | tail -20; tail -5 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
echo "== smoke $(date +%T)"
timeout -k 10 150 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
