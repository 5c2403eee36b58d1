#!/bin/bash
# round 2: SA Toeplitz register budget A/B (ZV_SA_TP 1 = 2-wave budget, 3 = 1-wave), parallel
# positional projection; parity subset; kernel trace of the default 3-stream bench for the
# concurrency analysis (tools/trace_overlap.py)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_sa_tp.py tests/test_gpu_parity.py tests/test_gpu_split_streams.py -v -s --timeout 300 --timeout-method thread > $O/r02_minw_test.log 2>&1 || { echo "tests failed rc=$?"; exit 1; }
for tp in 1 3 1 3; do
  ZV_SA_TP=$tp timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-fp32-mode --steps 4 > $O/r02_minw_$tp.json 2> $O/r02_minw_$tp.err || { echo "bench $tp rc=$?"; exit 1; }
  python -c "import json;d=json.load(open('$O/r02_minw_$tp.json'));k=d['roofline']['per_kernel_ms_per_step'];print('sa_tp=$tp', d['ms_per_step'], d['value'], 'sa ms/step', k.get('attn_sa_bf16'))" | tee -a $O/r02_minw_ab.txt
done
timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d $O/r02trace -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-fp32-mode > $O/r02trace.log 2>&1 || { echo "trace rc=$?"; exit 1; }
python3 tools/trace_overlap.py $(ls $O/r02trace/*kernel_trace.csv | head -1) > $O/r02_overlap.txt 2>&1
echo done
