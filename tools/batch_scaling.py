#!/usr/bin/env python3
"""Wall time of one guided decoder evaluation (T=1219) per batch size: how the
per-utterance cost moves with the rows resident at once (L2 / Infinity-Cache
working set vs tile quantisation)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from zipvoice_amd.config import default_config  # noqa: E402
from zipvoice_amd.models import build_model  # noqa: E402
from zipvoice_amd.weights import synthetic_state_dict  # noqa: E402

T = int(os.environ.get("ZV_T", "1219"))
Bs = [int(b) for b in (sys.argv[1].split(",") if len(sys.argv) > 1 else ("4", "8", "16", "32"))]
cfg = default_config("zipvoice")
m = build_model(cfg, precision="bf16")
m.load_state_dict(synthetic_state_dict(cfg, 0))
m = m.to("cuda:0")
dev = torch.device("cuda:0")
rng = np.random.default_rng(0)
for B in Bs:
    x = torch.from_numpy(rng.standard_normal((B, T, 100), dtype=np.float32)).to(dev)
    tc = torch.from_numpy(rng.standard_normal((B, T, 100), dtype=np.float32)).to(dev)
    sc = torch.from_numpy(rng.standard_normal((B, T, 100), dtype=np.float32)).to(dev)
    pm = torch.zeros(B, T, dtype=torch.bool, device=dev)
    for _ in range(2):
        m.engine.velocity(0.3, 1.0, x, tc, sc, pm)
    torch.cuda.synchronize()
    n = max(3, 96 // B)
    t0 = time.perf_counter()
    for _ in range(n):
        m.engine.velocity(0.3, 1.0, x, tc, sc, pm)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / n
    print(f"B={B:3d} (CFG rows {2 * B:3d}) T={T}: {dt * 1e3:8.2f} ms per guided forward, "
          f"{dt * 1e3 / B:7.3f} ms per utterance", flush=True)
