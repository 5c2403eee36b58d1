#!/bin/bash
# Round-5 configuration table: C3 / C4 / C5 per-step times (tools/config_bench.py, 3 timed steps)
# and one rocprofv3 kernel summary each (1 timed step + the 2 warm-up steps), then the C4 summary
# of the round-4 tree (tools/lab/r04tree: `git archive f6e0fdd`, built in place) for the attention
# share before / after.   tools/gpu/r05_configs.sh OUT
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r05_configs}; mkdir -p $O
for c in C3 C4 C5; do
  if [ "${PROF_ONLY:-0}" != 1 ]; then
    timeout -k 10 300 python -u tools/config_bench.py $c 3 > $O/$c.json 2> $O/$c.err || { echo "$c rc=$?"; tail -5 $O/$c.err; exit 1; }
    cat $O/$c.json
  fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/prof_$c -o run -- python3 tools/config_bench.py $c 1 > $O/prof_$c.log 2>&1 \
    || { echo "prof $c rc=$?"; tail -5 $O/prof_$c.log; exit 1; }
  find $O/prof_$c -type f ! -name '*kernel_stats.csv' -delete   # (the traces exceed the copy-back cap)
done
if [ -d tools/lab/r04tree ]; then
  cd tools/lab/r04tree
  if [ "${PROF_ONLY:-0}" != 1 ]; then
    timeout -k 10 300 python -u tools/config_bench.py C4 3 > ../../../$O/C4_r04.json 2> ../../../$O/C4_r04.err || { echo "r04 C4 rc=$?"; exit 1; }
    cat ../../../$O/C4_r04.json
  fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d ../../../$O/prof_C4_r04 -o run -- python3 tools/config_bench.py C4 1 > ../../../$O/prof_C4_r04.log 2>&1 \
    || { echo "prof r04 C4 rc=$?"; exit 1; }
  find ../../../$O/prof_C4_r04 -type f ! -name '*kernel_stats.csv' -delete
fi
echo done
