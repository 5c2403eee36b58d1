#!/bin/bash
# round 2 (final tree): GEMM launch-policy env A/B under the counted epilogues
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/policy
mkdir -p $O
rm -f $O/ab.txt
run() {  # tag envs...
  local tag=$1; shift
  timeout -k 10 300 env "$@" python -u bench.py --no-cpu-baseline --no-fp32-mode --steps 4 > $O/b_$tag.json 2> $O/b_$tag.err || { echo "bench rc=$?"; return 1; }
  python -c "import json;d=json.load(open('$O/b_$tag.json'));k=d['roofline']['per_kernel_ms_per_step'];print('$tag', d['ms_per_step'], 'resid', round(k.get('gemm_bf16_resid',0),1), 'gemm', round(k.get('gemm_bf16',0),1), 'glu', round(k.get('gemm_bf16_glu',0),1), 'na', round(k.get('gemm_bf16_na',0),1))" | tee -a $O/ab.txt
}
run base ZV_X=0 && run occp1 ZV_GEMM_OCC_PLAIN=1 && run occr1 ZV_GEMM_OCC_RESID=1 && run gxp0 ZV_GEMM_GRIDX_PLAIN=0 && run gxr0 ZV_GEMM_GRIDX_RESID=0 && run gxf0 ZV_GEMM_GRIDX_FUSED=0 && run base2 ZV_X=0 || exit 1
echo done
