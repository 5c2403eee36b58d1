# round 6: SQ counters of the NonlinAttention consumer (lab, 21 x 1219), 72-B padded V^T rows (old)
# vs 64-B XOR-swizzled rows (swz); one rocprofv3 --pmc pass each (8 SQ counters)
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp
O=gpurun_out/r06_na2_sq; mkdir -p $O
C="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAVES"
for arm in old swz; do
  B=tools/lab/attn2_time_bf16; [ $arm = old ] && B=tools/lab/ab/attn2_time_bf16_old
  timeout -s KILL 60 rocprofv3 --pmc $C -f csv --kernel-include-regex "zv_attn_na2" -d $O/$arm -o run -- $B 21 1219 3 > $O/$arm.log 2>&1 || { tail -5 $O/$arm.log; exit 1; }
  F=$(ls $O/$arm/*counter_collection.csv | head -1)
  python3 -c "
import csv,collections
s=collections.defaultdict(float); n=set()
for r in csv.DictReader(open('$F')):
    if 'na2_kernel<3, 8>' in r['Kernel_Name']: s[r['Counter_Name']]+=float(r['Counter_Value']); n.add(r['Dispatch_Id'])
print('$arm', 'dispatches', len(n), ' '.join(f'{k}={v/len(n):.4g}' for k,v in sorted(s.items())))
" | tee -a $O/summary.txt
  rm -rf $O/$arm
done
