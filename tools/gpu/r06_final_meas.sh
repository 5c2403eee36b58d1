#!/bin/bash
# Round-6 measurement of the final tree: PMC traffic per roofline tag (FETCH_SIZE / WRITE_SIZE in
# separate passes over one guided forward + one text-encoder pass on the bench's 3-stream schedule;
# each tag's regex covers every tile instantiation the tag launches), the bench line (reads that
# traffic), a rocprofv3 kernel trace + stats of a short bench run.   tools/gpu/r06_final_meas.sh OUT
# (SKIP_PMC=1: keep the traffic files already in profiles/)
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r06_final}; mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
if [ -z "$SKIP_PMC" ]; then
step pmc
RX='zv_gemm_kernel|zv_ffn_kernel|zv_gemm256_kernel'
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -f csv --kernel-include-regex "$RX" -d $O/pmc_fetch -o run -- python3 tools/profile_forward.py --iters 1 --text > $O/pmc_fetch.log 2>&1 || { tail -5 $O/pmc_fetch.log; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -f csv --kernel-include-regex "$RX" -d $O/pmc_write -o run -- python3 tools/profile_forward.py --iters 1 --text > $O/pmc_write.log 2>&1 || { tail -5 $O/pmc_write.log; exit 1; }
timeout -k 10 150 python3 tools/profile_forward.py --iters 1 --text --alg-json $O/alg.json > $O/alg.log 2>&1 || { tail -5 $O/alg.log; exit 1; }
F=$(ls $O/pmc_fetch/*counter_collection.csv | head -1); W=$(ls $O/pmc_write/*counter_collection.csv | head -1)
# residual ROLEs: every tile form (128 x 128, 128 x 64 at 3 blocks per CU, 64 x 64 with the 4-deep ring)
R='zv_gemm_kernel<(128|64), (128|64), 2, 2, 1, 0, [0-9], [0-9], 64, 0, 0, 0'
# NAME|PROFILER_TAG(S)|SYMBOL_REGEX
for kv in "r06_gemm_resid_r1|gemm_bf16_resid|$R, 1, 1, 0>" \
          "r06_gemm_resid_r4|gemm_bf16_resid_rv|$R, 4, 1, 0>" \
          "r06_gemm_resid_r2|gemm_bf16_resid_byp|$R, 2, 1, 0>" \
          "r06_ffn|ffn_bf16|zv_ffn_kernel<(true|false), (true|false), true, 0, 0, (true|false)>" \
          "r06_ffn_norm|ffn_norm_bf16|zv_ffn_kernel<false, false, true, 0, 1, (true|false)>" \
          "r06_ffn_all|ffn_bf16+ffn_norm_bf16|zv_ffn_kernel<" \
          "r06_gemm_glu_dw|gemm_bf16_glu_dw|zv_gemm256_kernel<3, 3, 0, 0, 1, 1, (31|15|7)>"; do
  n=${kv%%|*}; rest=${kv#*|}; tag=${rest%%|*}; rx=${rest#*|}
  python3 tools/pmc_traffic.py "$F" "$W" "$rx" $O/${n}_traffic.json $O/alg.json "$tag" >> $O/pmc_traffic.log 2>&1
done
cut -c1-240 $O/pmc_traffic.log
rm -f $F $W
cp $O/r06_*_traffic.json profiles/
fi
step bench
timeout -k 10 500 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench.json'));r=d['roofline'];print(d['ms_per_step'],d['value'],r['kernel'],r['frac'],r['avg_launch_us'],r.get('traffic_over_algorithmic'));print({k:v['ms_per_step'] for k,v in d.items() if isinstance(v,dict) and 'ms_per_step' in v})"
step rocprof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/rp -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-fp32-mode > $O/rp_bench.log 2>&1 || { tail -5 $O/rp_bench.log; exit 1; }
S=$(ls $O/rp/*kernel_stats.csv | head -1); cp $S $O/kernel_stats.csv; rm -rf $O/rp
step done
