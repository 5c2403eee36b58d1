#!/bin/bash
# round 2 (final tree): decoder row-block streams A/B (ZV_SPLIT_STREAMS)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/streams
mkdir -p $O
rm -f $O/ab.txt
run() {  # flag tag
  timeout -k 10 300 env ZV_SPLIT_STREAMS=$1 python -u bench.py --no-cpu-baseline --no-fp32-mode --steps 4 > $O/b_$1_$2.json 2> $O/b_$1_$2.err || { echo "bench rc=$?"; return 1; }
  python -c "import json;d=json.load(open('$O/b_$1_$2.json'));print('streams=$1', d['ms_per_step'])" | tee -a $O/ab.txt
}
run 3 a && run 4 a && run 2 a && run 3 b && run 4 b && run 2 b || exit 1
echo done
