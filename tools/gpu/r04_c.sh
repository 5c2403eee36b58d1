#!/bin/bash
# Round 4 GPU session C: skeleton probe (V8/V9: fragment ring, whole step), the FF phase timing of the
# new default (FFN_OUT_ASM + FFN_BIAS_ACC) and its ablations, old-vs-new lab, the FF / split / fused
# fp16 tests on the new kernel, bench.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r04_c}; mkdir -p $O
timeout -k 10 60 tools/probe/ffn_mfma_probe 256 400 > $O/probe.txt 2>&1 || { echo "probe rc=$?"; cat $O/probe.txt; exit 1; }
cat $O/probe.txt
for v in t x_noact x_now2 x_now12 x_noact_now12; do
  echo "== $v" >> $O/x.txt
  timeout -k 10 60 tools/lab/ffn_lab_$v 2 1,8 "78016x1536" 0 "pers,noDMA,noEpi" >> $O/x.txt 2>&1 || { echo "$v rc=$?"; tail -3 $O/x.txt; exit 1; }
done
cat $O/x.txt
for r in 1 2; do
  for v in ffn_lab_old ffn_lab; do
    echo "== $v round $r" >> $O/var.txt
    timeout -k 10 120 tools/lab/$v 3 1,2,8 "78016x1536;39008x1536;26005x1536" 0 "unfused,classic,pers,noEpi" >> $O/var.txt 2>&1 || { echo "$v rc=$?"; tail -5 $O/var.txt; exit 1; }
  done
done
cat $O/var.txt
timeout -k 10 900 python -u -m pytest tests/test_gpu_ffn.py tests/test_gpu_split_streams.py "tests/test_gpu_fullsize.py::test_velocity_full_size_fp16_fused_ff" "tests/test_gpu_fullsize.py::test_velocity_full_size_vs_oracle" tests/test_gpu_parity.py -x -v -s --timeout 400 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; grep -E "PASS|FAIL|Error|error" $O/pytest.log | tail -30; exit 1; }
grep -E "passed|failed" $O/pytest.log | tail -3
grep -iE "mean" $O/pytest.log | grep -iE "fp16|ZV_FFN|bf16\]" | head -40
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -5 $O/bench.err; exit 1; }
cat $O/bench.json
