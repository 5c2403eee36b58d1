cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r05_fp32ab; mkdir -p $O
for r in 1 2; do
  for arm in r04 tree; do
    if [ $arm = r04 ]; then export ZV_LIB_PATH=tools/lab/r04tree/zipvoice_amd/libzipvoice_hip.so; else unset ZV_LIB_PATH; fi
    timeout -k 10 300 python -u bench.py --precision fp32 --steps 2 --warmup 2 --no-cpu-baseline > $O/$arm$r.json 2> $O/$arm$r.err || { echo "rc=$? $arm"; tail -5 $O/$arm$r.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/$arm$r.json'));print('$arm', d['ms_per_step'])"
  done
done
