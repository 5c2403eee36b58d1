#!/bin/bash
# Round 4 GPU session G: the transposed FF epilogue (FFN_EPI_T) vs the per-lane one, its prefetch
# depth; phase timing; the FF / split / parity tests on the new engine; bench.
#   builds: tools/lab/ffn_lab{,_noT -DFFN_EPI_T=0,_pt24 -DFFN_PT=24,_pt8 -DFFN_PT=8,_t -DFFN_TIMING=1,_t_noT}
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r04_g}; mkdir -p $O
for r in 1 2; do
  for v in ffn_lab_noT ffn_lab ffn_lab_pt24 ffn_lab_pt8; do
    echo "== $v round $r" >> $O/var.txt
    timeout -k 10 120 tools/lab/$v 3 1,2,4 "78016x1536;26005x1536;13002x1536" 0 "unfused,classic,pers" >> $O/var.txt 2>&1 || { echo "$v rc=$?"; tail -5 $O/var.txt; exit 1; }
  done
done
cat $O/var.txt
for v in t t_noT; do
  echo "== $v" >> $O/x.txt
  timeout -k 10 60 tools/lab/ffn_lab_$v 2 1 "78016x1536" 0 "pers" >> $O/x.txt 2>&1 || { echo "$v rc=$?"; tail -3 $O/x.txt; exit 1; }
done
cat $O/x.txt
timeout -k 10 900 python -u -m pytest tests/test_gpu_ffn.py tests/test_gpu_split_streams.py tests/test_gpu_parity.py "tests/test_gpu_fullsize.py::test_velocity_full_size_fp16_fused_ff" -x -q --timeout 400 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error|error" $O/pytest.log | tail -30; exit 1; }
tail -2 $O/pytest.log
bash tools/gpu/ab_env.sh ${1:-r04_g}/ab 2 "-"
