# round 6 A/B: fragment preload in the weight-split (SPLIT 2) GEMM K step (fp16 parity mode's
# gemm_wsplit_t / gemm_wsplit_n96): base = the generic read -> MFMA loop; pre = preloaded fragments.
# Bitwise check (the fp16 parity + split-stream tests) on the new build, then interleaved timing.
O=gpurun_out/r06_pre2_ab; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_split_streams.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do
  for arm in base pre; do
    if [ $arm = pre ]; then unset ZV_LIB_F16_PATH; else export ZV_LIB_F16_PATH=$PWD/tools/lab/ab/libzipvoice_hip_f16_$arm.so; fi
    timeout -k 10 300 python -u tools/mode_profile.py fp16 > $O/$arm.$i.txt 2>&1 || { tail -5 $O/$arm.$i.txt; exit 1; }
    python3 -c "
import json
for l in open('$O/$arm.$i.txt'):
    if l.startswith('{'):
        d=json.loads(l)['fp16']; k=d['per_kernel_ms']
        print('$arm run $i: step', d['ms_per_step'], 'ms; gemm_wsplit_t', k.get('gemm_wsplit_t'), 'gemm_wsplit_n96', k.get('gemm_wsplit_n96'))"
  done
done
