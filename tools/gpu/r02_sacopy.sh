#!/bin/bash
# round 2: copy-only SelfAttention out-projection on the counted epilogue (ROLE 5, ZV_SA_COPY)
# vs the wave-specialised kernel - bitwise test, bench A/B
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/sacopy
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
for flag in ("0", "1"):
    os.environ["ZV_SA_COPY"] = flag
    m = build_model(cfg, precision="bf16"); m.load_state_dict(sd); m = m.cuda()
    outs.append(m.engine.velocity(0.4, 1.0, x, tc, sc, pm).cpu()); del m
print("ZV_SA_COPY 0 vs 1 max |diff| =", (outs[0] - outs[1]).abs().max().item(), "equal", torch.equal(outs[0], outs[1]))
PY
timeout -k 10 200 python -u $O/t.py > $O/test.txt 2>&1 || { echo "test rc=$?"; exit 1; }
run() {  # flag tag
  timeout -k 10 300 env ZV_SA_COPY=$1 python -u bench.py --no-cpu-baseline --no-fp32-mode --steps 4 > $O/b_$1_$2.json 2> $O/b_$1_$2.err || { echo "bench rc=$?"; return 1; }
  python -c "import json;d=json.load(open('$O/b_$1_$2.json'));k=d['roofline']['per_kernel_ms_per_step'];print('sacopy=$1', d['ms_per_step'], 'ws', round(k.get('gemm_bf16_resid_ws',0),1), 'copy', round(k.get('gemm_bf16_resid_copy',0),1))" | tee -a $O/ab.txt
}
run 1 a && run 0 a && run 1 b && run 0 b || exit 1
echo done
