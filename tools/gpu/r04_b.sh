#!/bin/bash
# Round 4 GPU session B: MFMA skeleton probe, FF ablations + variants + lab (r04_x.sh), the host-sync
# test, the fp16 numbers of the parity-hardening tests, bench A/B (persistent FF; SelfAttention
# weight split in the fp16 mode).
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r04_b}; mkdir -p $O
timeout -k 10 60 tools/probe/ffn_mfma_probe 256 400 > $O/probe.txt 2>&1 || { echo "probe rc=$?"; cat $O/probe.txt; exit 1; }
cat $O/probe.txt
bash tools/gpu/r04_x.sh ${1:-r04_b} || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_host_sync.py tests/test_gpu_ffn.py tests/test_gpu_sa_tp.py "tests/test_gpu_fullsize.py::test_velocity_full_size_fp16_fused_ff" "tests/test_gpu_fullsize.py::test_velocity_full_size_vs_oracle" -x -v -s --timeout 400 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; grep -E "PASS|FAIL|Error|error" $O/pytest.log | tail -30; exit 1; }
grep -E "passed|failed" $O/pytest.log | tail -3
grep -iE "split=|mean|vs oracle" $O/pytest.log | head -60
bash tools/gpu/ab_env.sh ${1:-r04_b}/ab 2 "-" "ZV_FFN_PERSIST=0" && BENCH_ARGS="--precision fp16" bash tools/gpu/ab_env.sh ${1:-r04_b}/ab16 2 "-" "ZV_MIXED_SA=0"
