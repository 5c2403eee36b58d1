#!/bin/bash
# Round 4 GPU session L: the prologue chain overlapping the x loads' tail (FFN_XOVL) vs waiting for all
# of them (noxo), lab (bit-for-bit checks) + phase timing; FF / split / parity tests; bench.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r04_l}; mkdir -p $O
for r in 1 2; do
  for v in ffn_lab_noxo ffn_lab_xo; do
    echo "== $v round $r" >> $O/var.txt
    timeout -k 10 120 tools/lab/$v 3 1,4,8 "78016x1536;26005x1536" 0 "unfused,classic,pers,seg3" >> $O/var.txt 2>&1 || { echo "$v rc=$?"; tail -5 $O/var.txt; exit 1; }
  done
done
cat $O/var.txt
echo "== t_xo" >> $O/x.txt
timeout -k 10 60 tools/lab/ffn_lab_t_xo 2 1,8 "78016x1536" 0 "pers" >> $O/x.txt 2>&1 || { echo "t rc=$?"; tail -3 $O/x.txt; exit 1; }
cat $O/x.txt
timeout -k 10 900 python -u -m pytest tests/test_gpu_ffn.py tests/test_gpu_split_streams.py tests/test_gpu_parity.py "tests/test_gpu_fullsize.py::test_velocity_full_size_fp16_fused_ff" -x -q --timeout 400 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error|error" $O/pytest.log | tail -30; exit 1; }
tail -1 $O/pytest.log
bash tools/gpu/ab_env.sh ${1:-r04_l}/ab 2 "-"
