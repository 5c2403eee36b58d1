#!/bin/bash
# round 2: where the 128x128 GEMM's cycles go (no-output mainloop vs residual epilogue):
# SQ instruction / wait / LDS counters per dispatch, two passes per configuration
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02gpmc
mkdir -p $O
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"
P2="SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_VALU SQ_ACTIVE_INST_MISC"
for cfg in "0 4 78016x512x1536" "100 2 78016x512x1536" "0 4 78016x1024x512" "0 1 78016x1024x512" "100 2 78016x512x512"; do
  set -- $cfg
  tag=v$1_m$2_$3
  for pass in 1 2; do
    if [ $pass = 1 ]; then C="$P1"; else C="$P2"; fi
    timeout -s KILL 90 rocprofv3 --pmc $C -f csv --kernel-include-regex zv_gemm_kernel -d $O/${tag}_p$pass -o run -- python3 tools/bench_gemm.py $1 $2 "$3" > $O/${tag}_p$pass.log 2>&1 || { echo "$tag pass $pass rc=$?"; exit 1; }
  done
done

# wave-tile variants (128x64 wave tiles: 7 = 256x128 BK64, 32 = BK32 2-stage, 33 = BK32 3-stage)
timeout -k 10 300 python -u tools/bench_gemm.py 0,7,32,33 4,1,2 "78016x512x1536;78016x1024x512;78016x1536x512;78016x512x512" > $O/variants.log 2>&1 || { echo "variants rc=$?"; exit 1; }
# the other BASELINE configurations
timeout -k 10 400 python -u tools/config_bench.py C3,C4,C5 2 > $O/configs.txt 2>&1 || { echo "configs rc=$?"; exit 1; }
timeout -k 10 400 python -u bench.py --config C3 --no-cpu-baseline --no-fp32-mode > $O/bench_c3.json 2> $O/bench_c3.err || { echo "c3 rc=$?"; exit 1; }
echo all-done
