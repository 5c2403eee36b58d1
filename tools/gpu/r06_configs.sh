# round 6 final tree: every BASELINE config through bench.py on one GPU (C3 = the per-GPU share of
# north_star's 8-GPU config; C4; C5 in its default fp8 and in bf16)
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp
O=gpurun_out/r06_configs; mkdir -p $O; : > $O/configs.jsonl
for a in "--config C3" "--config C4" "--config C5" "--config C5 --precision bf16"; do
  timeout -k 10 400 python -u bench.py $a --steps 2 --warmup 2 --no-cpu-baseline --no-fp32-mode > $O/one.json 2> $O/one.err || { echo "rc=$? ($a)"; tail -5 $O/one.err; exit 1; }
  tail -1 $O/one.json >> $O/configs.jsonl
  python3 -c "import json; d=json.loads(open('$O/one.json').read().strip().splitlines()[-1]); print('$a', d['dtype'], d['ms_per_step'], d['value'], d['path_roofline']['frac'], d['roofline']['kernel'], d['roofline']['frac'])"
done
