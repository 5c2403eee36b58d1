# round 6: decoder row-block streams 3 (default) vs 4, and the FF persistent schedule off, on the
# final tree: the bench line's bf16 step and its fp16 / fp32 legs (same process, as the driver runs
# it), interleaved on one box
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp
O=gpurun_out/r06_streams_ab; mkdir -p $O
for r in 1 2; do
  for e in "-" "ZV_SPLIT_STREAMS=4" "ZV_SPLIT_STREAMS=4 ZV_FFN_PERSIST=0"; do
    envs=(); [ "$e" != "-" ] && read -r -a envs <<< "$e"
    n=$(echo "$e" | tr ' =' '__')
    timeout -k 10 400 env "${envs[@]}" python -u bench.py --no-cpu-baseline --steps 4 > $O/b_${n}_$r.json 2> $O/b_${n}_$r.err || { echo "bench rc=$? ($e)"; tail -5 $O/b_${n}_$r.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('$O/b_${n}_$r.json').read().strip().splitlines()[-1])
print('$e', 'run $r: bf16', d['ms_per_step'], 'fp16', d['fp16_parity_mode']['ms_per_step'], 'fp32', d['fp32_accurate_mode']['ms_per_step'])" | tee -a $O/ab.txt
  done
done
