"""Which counted epilogue class changes the fp32-mode decoder output (ZV_RES_COUNTED bits:
1 residual, 2 plain, 4 NA, 8 GLU, 16 transposed)?  Runs each single class against none."""
import os
import subprocess
import sys

CODE = r'''
import numpy as np, torch, sys
sys.path.insert(0, ".")
from zipvoice_amd.config import default_config
from zipvoice_amd.models import build_model
from zipvoice_amd.weights import synthetic_state_dict
cfg = default_config("zipvoice"); sd = synthetic_state_dict(cfg, 0)
rng = np.random.default_rng(2); B, T = 3, 333
f = lambda: torch.from_numpy(rng.standard_normal((B, T, 100), dtype=np.float32)).cuda()
x, tc, sc = f(), f(), f()
pm = torch.from_numpy(np.arange(T)[None] >= np.array([T, 250, 97])[:, None]).cuda()
m = build_model(cfg, precision=sys.argv[1]); m.load_state_dict(sd); m = m.cuda()
np.save(sys.argv[2], m.engine.velocity(0.4, 1.0, x, tc, sc, pm).cpu().numpy())
'''
prec = sys.argv[1] if len(sys.argv) > 1 else "fp32"
import numpy as np
res = {}
for mask in (0, 1, 2, 4, 8, 16, 31):
    env = dict(os.environ, ZV_RES_COUNTED=str(32 + mask))
    out = f"gpurun_out/cb_{prec}_{mask}.npy"
    subprocess.run([sys.executable, "-c", CODE, prec, out], env=env, check=True, timeout=300)
    res[mask] = np.load(out)
    print(f"{prec} mask {mask:2d}: max |diff vs none| = {np.abs(res[mask] - res[0]).max():.3e}", flush=True)
