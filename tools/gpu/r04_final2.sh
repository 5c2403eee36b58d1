#!/bin/bash
# Round-4 final tree: every GPU test + smoke, the bench line (reading profiles/r04_*_traffic.json),
# and the rocprofv3 kernel trace + stats of a short bench run (same engine build).
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r04_final2}; mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
step pytest
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { grep -E "FAIL|Error" $O/pytest_gpu.log | tail -20; tail -5 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
step smoke
timeout -k 10 150 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
step bench
timeout -k 10 500 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench.json'));r=d['roofline'];print(d['ms_per_step'],d['value'],r['kernel'],r['frac'],r['avg_launch_us'],r.get('traffic_over_algorithmic'));print({k:v['ms_per_step'] for k,v in d.items() if isinstance(v,dict) and 'ms_per_step' in v})"
step rocprof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/rp -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-fp32-mode > $O/rp_bench.log 2>&1 || { tail -5 $O/rp_bench.log; exit 1; }
S=$(ls $O/rp/*kernel_stats.csv | head -1); cp $S $O/kernel_stats.csv; rm -f $O/rp/*kernel_trace.csv
step done
