#!/bin/bash
# Other BASELINE configurations per GPU (tools/config_bench.py), the C3 bench line, single-
# sentence latency (tools/latency_c1.py) and the bf16 / fp16 per-kernel-family step profile.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/configs; mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
step configs
timeout -k 10 400 python -u tools/config_bench.py C3,C4,C5 3 > $O/configs_bf16.txt 2>&1 || { tail -5 $O/configs_bf16.txt; exit 1; }
timeout -k 10 200 python -u tools/config_bench.py C5 3 fp8 > $O/configs_fp8.txt 2>&1 || { tail -5 $O/configs_fp8.txt; exit 1; }
cat $O/configs_bf16.txt $O/configs_fp8.txt | grep -v "^$" | tail -8
step c3bench
timeout -k 10 400 python -u bench.py --config C3 --no-cpu-baseline --no-fp32-mode > $O/bench_c3.json 2> $O/bench_c3.err || { tail -5 $O/bench_c3.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_c3.json'));print(d['ms_per_step'],d['value'],d['unit'])"
step latency
timeout -k 10 200 python -u tools/latency_c1.py > $O/latency_c1.txt 2>&1 || { tail -5 $O/latency_c1.txt; exit 1; }
tail -4 $O/latency_c1.txt
step modes
timeout -k 10 400 python -u tools/mode_profile.py bf16,fp16 > $O/modes.txt 2>&1 || { tail -5 $O/modes.txt; exit 1; }
tail -30 $O/modes.txt
step done
