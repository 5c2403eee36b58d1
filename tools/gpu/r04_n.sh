#!/bin/bash
# Round 4 GPU session N: bench A/B of the fused-FeedForward row threshold (whole-batch rows of a
# stack): default 10000 (every stack fused) vs 20000 (the quarter-rate stack unfused) vs 40000 (the
# half- and quarter-rate stacks unfused); the per-stream launches there fill 40 % / 20 % of the CUs.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
bash tools/gpu/ab_env.sh ${1:-r04_n}/ab 2 "-" "ZV_FFN_MIN_ROWS=20000" "ZV_FFN_MIN_ROWS=40000"
