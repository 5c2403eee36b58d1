# round 6: C4 (30 s dialogues, T = 3376) in the fp16 parity mode, offsets from step 0 alone (nodiag)
# vs step 0 + the diagonal step (diag, the tree); interleaved on one box; exact-path counts first
O=gpurun_out/r06_c4_fp16; mkdir -p $O
timeout -k 10 200 python -u tools/fallback_probe.py fp16 3376 > $O/probe_diag.txt 2>&1 || { tail -5 $O/probe_diag.txt; exit 1; }
ZV_LIB_F16_PATH=$PWD/tools/lab/ab/libzipvoice_hip_f16_nodiag.so timeout -k 10 200 python -u tools/fallback_probe.py fp16 3376 > $O/probe_nodiag.txt 2>&1 || { tail -5 $O/probe_nodiag.txt; exit 1; }
grep -h exact $O/probe_diag.txt | sed 's/^/diag   /'; grep -h exact $O/probe_nodiag.txt | sed 's/^/nodiag /'
for i in 1 2; do
  for arm in diag nodiag; do
    if [ $arm = nodiag ]; then export ZV_LIB_F16_PATH=$PWD/tools/lab/ab/libzipvoice_hip_f16_nodiag.so; else unset ZV_LIB_F16_PATH; fi
    timeout -k 10 400 python -u bench.py --config C4 --precision fp16 --steps 2 --warmup 1 --no-cpu-baseline --no-fp32-mode > $O/$arm.$i.json 2> $O/$arm.$i.err || { tail -5 $O/$arm.$i.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('$O/$arm.$i.json').read().strip().splitlines()[-1]); print('$arm run $i: C4 fp16', d['ms_per_step'], 'ms per step', d['value'], d['unit'])"
  done
done
