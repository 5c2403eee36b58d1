# round 6 A/B: fp16 offsets from step 0 + the diagonal step (diag) vs step 0 alone (nodiag), same box,
# interleaved; tools/mode_profile.py fp16 (timed C2 step + serialized per-tag ms)
O=gpurun_out/r06_diag_ab; mkdir -p $O
for i in 1 2; do
  for arm in diag nodiag; do
    if [ $arm = nodiag ]; then export ZV_LIB_F16_PATH=$PWD/tools/lab/ab/libzipvoice_hip_f16_nodiag.so; else unset ZV_LIB_F16_PATH; fi
    timeout -k 10 300 python -u tools/mode_profile.py fp16 > $O/$arm.$i.txt 2>&1 || { tail -5 $O/$arm.$i.txt; exit 1; }
    python3 -c "
import json,sys
for l in open('$O/$arm.$i.txt'):
    if l.startswith('{'):
        d=json.loads(l)['fp16']; k=d['per_kernel_ms']
        print('$arm run $i: step', d['ms_per_step'], 'ms; attn_sa', k.get('attn_sa_bf16'), 'attn_na', k.get('attn_na_bf16'))"
  done
done
