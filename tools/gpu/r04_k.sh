#!/bin/bash
# Round 4 GPU session K: FF3 + BiasNorm epilogue with its constants staged in LDS (FFN_NORM_LDS) vs
# loaded per group (nolds), lab + phase timing; FF / split / parity tests; bench A/B against an
# FFN_NORM_LDS=0 engine (python zipvoice_amd/csrc/build.py --out ab_libs/libzipvoice_hip_nolds.so -DFFN_NORM_LDS=0).
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r04_k}; mkdir -p $O
for r in 1 2; do
  for v in ffn_lab_nolds ffn_lab; do
    echo "== $v round $r" >> $O/var.txt
    timeout -k 10 120 tools/lab/$v 3 8 "78016x1536;26005x1536;13002x1536" 0 "classic,pers" >> $O/var.txt 2>&1 || { echo "$v rc=$?"; tail -5 $O/var.txt; exit 1; }
  done
done
cat $O/var.txt
for v in t t_nolds; do
  echo "== $v" >> $O/x.txt
  timeout -k 10 60 tools/lab/ffn_lab_$v 2 8 "78016x1536" 0 "pers" >> $O/x.txt 2>&1 || { echo "$v rc=$?"; tail -3 $O/x.txt; exit 1; }
done
cat $O/x.txt
timeout -k 10 900 python -u -m pytest tests/test_gpu_ffn.py tests/test_gpu_split_streams.py tests/test_gpu_parity.py "tests/test_gpu_fullsize.py::test_velocity_full_size_fp16_fused_ff" -x -q --timeout 400 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error|error" $O/pytest.log | tail -30; exit 1; }
tail -1 $O/pytest.log
bash tools/gpu/ab_env.sh ${1:-r04_k}/ab 2 "-" "ZV_LIB_PATH=ab_libs/libzipvoice_hip_nolds.so"
