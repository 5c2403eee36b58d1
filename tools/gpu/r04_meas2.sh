#!/bin/bash
# Round-4 final tree, measurement only: the bench line and the rocprofv3 kernel trace + stats of a
# short bench run (same engine build, same box).
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r04_meas2}; mkdir -p $O
timeout -k 10 500 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench.json'));r=d['roofline'];print(d['ms_per_step'],d['value'],r['kernel'],r['frac'],r['avg_launch_us'],r.get('traffic_over_algorithmic'));print({k:v['ms_per_step'] for k,v in d.items() if isinstance(v,dict) and 'ms_per_step' in v})"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/rp -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-fp32-mode > $O/rp_bench.log 2>&1 || { tail -5 $O/rp_bench.log; exit 1; }
S=$(ls $O/rp/*kernel_stats.csv | head -1); cp $S $O/kernel_stats.csv; rm -f $O/rp/*kernel_trace.csv
echo done
