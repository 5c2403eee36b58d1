#!/bin/bash
# Round-5 stream-count A/B (verdict item 5): decoder row blocks on 3 vs 4 streams, each mode in a
# process of its own (one engine, streams created on first use: the caller's + split - 1), so the
# 4-stream arm holds 4 streams against the 4 hardware queues.   tools/gpu/r05_streams_ab.sh OUT ROUNDS
cd "${GRAFT_REPO_ROOT:-.}"
O=${1:-r05_streams}; R=${2:-2}
for prec in fp16 bf16; do
  BENCH_ARGS="--precision $prec" bash tools/gpu/ab_env.sh "$O/$prec" "$R" "ZV_SPLIT_STREAMS=3" "ZV_SPLIT_STREAMS=4" || exit 1
done
