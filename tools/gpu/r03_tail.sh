#!/bin/bash
# Fused FF tail (FFN_TAIL): lab old vs new (same results expected bit for bit), the FF GPU tests
# + parity / fullsize on the FFN_TAIL=1 library (ZV_LIB_PATH), then the C2 bench A/B (the default
# library vs the FFN_TAIL=1 one), interleaved.  Build first, on the CPU:
#   python zipvoice_amd/csrc/build.py --out zipvoice_amd/libzipvoice_hip_tail1.so -DFFN_TAIL=1
#   python zipvoice_amd/csrc/build.py --out zipvoice_amd/libzipvoice_hip_f16_tail1.so -DFFN_TAIL=1 -DZV_OPERAND_F16
#   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I zipvoice_amd/csrc tools/lab/ffn_lab.hip -DFFN_TAIL=1 -o tools/lab/ffn_lab
#   (and -DFFN_TAIL=0 -o tools/lab/ffn_lab_old)
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/tail; mkdir -p $O
T1=zipvoice_amd/libzipvoice_hip_tail1.so
for r in 1; do
  for v in ffn_lab_old ffn_lab; do
    echo "== $v round $r" >> $O/lab.txt
    timeout -k 10 150 tools/lab/$v 3 1,2,4 >> $O/lab.txt 2>&1 || { echo "lab $v rc=$?"; tail -20 $O/lab.txt; exit 1; }
  done
done
cat $O/lab.txt
ZV_LIB_PATH=$T1 ZV_LIB_F16_PATH=zipvoice_amd/libzipvoice_hip_f16_tail1.so timeout -k 10 600 python -u -m pytest tests/test_gpu_ffn.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -q \
  --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
bash tools/gpu/ab_env.sh tail/ab ${1:-2} "-" "ZV_LIB_PATH=$T1"
