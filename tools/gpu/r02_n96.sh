#!/bin/bash
# round 2: attention-score projection (N = 272) tiles on the counted plain epilogue (ZV_N96)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/n96b
mkdir -p $O
rm -f $O/ab.txt
cat > $O/t.py <<'PY'
import os, sys, numpy as np, torch
sys.path.insert(0, ".")
from zipvoice_amd.config import default_config
from zipvoice_amd.models import build_model
from zipvoice_amd.weights import synthetic_state_dict
rng = np.random.default_rng(3); B, T = 3, 333
f = lambda: torch.from_numpy(rng.standard_normal((B, T, 100), dtype=np.float32)).cuda()
x, tc, sc = f(), f(), f()
pm = torch.from_numpy(np.arange(T)[None] >= np.array([T, 250, 97])[:, None]).cuda()
cfg = default_config("zipvoice"); sd = synthetic_state_dict(cfg, 0)
outs = []
for flag in ("0", "1", "2"):
    os.environ["ZV_N96"] = flag
    m = build_model(cfg, precision="bf16"); m.load_state_dict(sd); m = m.cuda()
    outs.append(m.engine.velocity(0.4, 1.0, x, tc, sc, pm).cpu()); del m
for k in (1, 2):
    print(f"ZV_N96 0 vs {k} max |diff| =", (outs[0] - outs[k]).abs().max().item(), "equal", torch.equal(outs[0], outs[k]))
PY
timeout -k 10 200 python -u $O/t.py > $O/test.txt 2>&1 || { echo "test rc=$?"; exit 1; }
run() {  # flag tag
  timeout -k 10 300 env ZV_N96=$1 python -u bench.py --no-cpu-baseline --no-fp32-mode --steps 4 > $O/b_$1_$2.json 2> $O/b_$1_$2.err || { echo "bench rc=$?"; return 1; }
  python -c "import json;d=json.load(open('$O/b_$1_$2.json'));k=d['roofline']['per_kernel_ms_per_step'];print('n96=$1', d['ms_per_step'], 'n96', round(k.get('gemm_bf16_n96',0),1), 'gemm', round(k.get('gemm_bf16',0),1))" | tee -a $O/ab.txt
}
run 1 a && run 0 a && run 2 a && run 1 b && run 0 b || exit 1
echo done
