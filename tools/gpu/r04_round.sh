#!/bin/bash
# Round 4 combined GPU session: FF ablations + lab, the changed GPU tests, bench A/B.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
bash tools/gpu/r04_x.sh ${1:-r04_round} || exit 1
O=gpurun_out/${1:-r04_round}
timeout -k 10 1200 python -u -m pytest tests/test_gpu_ffn.py tests/test_gpu_sa_tp.py tests/test_gpu_split_streams.py tests/test_gpu_fullsize.py tests/test_gpu_parity.py tests/test_gpu_host_sync.py -x -v --timeout 400 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; grep -E "PASS|FAIL|Error|error" $O/pytest.log | tail -30; exit 1; }
grep -E "PASS|FAIL|passed|failed" $O/pytest.log | tail -8
grep -E "mean=|vs oracle|max \|" $O/pytest.log | grep -i "fp16" | head -30
bash tools/gpu/ab_env.sh ${1:-r04_round}/ab 2 "-" "ZV_FFN_PERSIST=0" && BENCH_ARGS="--precision fp16" bash tools/gpu/ab_env.sh ${1:-r04_round}/ab16 2 "-" "ZV_MIXED_SA=0"
