# round 6 A/B: K-ring depth of the fp16 parity mode's weight-split value projection (gemm_wsplit_t):
# 2 stages (base), 3, 4 (one block per CU); same box, interleaved, tools/mode_profile.py fp16
O=gpurun_out/r06_wsplit_ab; mkdir -p $O
for i in 1 2; do
  for arm in base t3 t4; do
    if [ $arm = base ]; then unset ZV_LIB_F16_PATH; else export ZV_LIB_F16_PATH=$PWD/tools/lab/ab/libzipvoice_hip_f16_$arm.so; fi
    timeout -k 10 300 python -u tools/mode_profile.py fp16 > $O/$arm.$i.txt 2>&1 || { tail -5 $O/$arm.$i.txt; exit 1; }
    python3 -c "
import json
for l in open('$O/$arm.$i.txt'):
    if l.startswith('{'):
        d=json.loads(l)['fp16']; k=d['per_kernel_ms']
        print('$arm run $i: step', d['ms_per_step'], 'ms; gemm_wsplit_t', k.get('gemm_wsplit_t'), 'gemm_wsplit_n96', k.get('gemm_wsplit_n96'))"
  done
done
