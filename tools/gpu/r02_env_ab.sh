#!/bin/bash
# round 2: launch-policy A/B under the 3-stream decoder (one tile per block vs persistent for
# the plain / fused-epilogue linears) and the C5 configuration with and without the split
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
run() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-fp32-mode --steps 4 > $O/r02_env_$tag.json 2> $O/r02_env_$tag.err || { echo "bench $tag rc=$?"; exit 1; }
  python -c "import json;d=json.load(open('$O/r02_env_$tag.json'));print('$tag', d['ms_per_step'], d['value'])" | tee -a $O/r02_env_ab.txt
}
run base ZV_X=0
run plain1 ZV_GEMM_GRIDX_PLAIN=-1
run fused1 ZV_GEMM_GRIDX_FUSED=-1
run both1 ZV_GEMM_GRIDX_PLAIN=-1 ZV_GEMM_GRIDX_FUSED=-1
run base2 ZV_X=0
for sp in 1 3; do
  ZV_SPLIT_STREAMS=$sp timeout -k 10 300 python -u tools/config_bench.py C4,C5 2 > $O/r02_env_cfg_$sp.txt 2>&1 || { echo "cfg rc=$?"; exit 1; }
  grep -v amdgpu $O/r02_env_cfg_$sp.txt | sed "s/^/split=$sp /" | tee -a $O/r02_env_ab.txt
done
