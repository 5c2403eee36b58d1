"""Exact-path runs of the second-generation attention consumers (zv_attn_fallbacks) for one guided
velocity at the C2 / C4 shapes, per precision mode: how often the range check fires on the
synthetic weights (bf16: raw 2^s; fp16: per-query offsets from the first key step).

    python tools/fallback_probe.py [bf16,fp16] [T ...]     (ZV_PROBE_RAGGED=1: utterance lengths
                                                           0.6-1.0 T, the rest padded)"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from zipvoice_amd.config import default_config  # noqa: E402
from zipvoice_amd.models import build_model  # noqa: E402
from zipvoice_amd.weights import synthetic_state_dict  # noqa: E402

modes = (sys.argv[1] if len(sys.argv) > 1 else "bf16,fp16").split(",")
Ts = [int(t) for t in sys.argv[2:]] or [1219, 3376]
cfg = default_config("zipvoice")
sd = synthetic_state_dict(cfg, 0)
for mode in modes:
    m = build_model(cfg, precision=mode)
    m.load_state_dict(sd)
    m = m.to("cuda:0")
    for T in Ts:
        B = 8 if T < 2000 else 2
        rng = np.random.default_rng(T)
        x, tc, sc = (torch.from_numpy(rng.standard_normal((B, T, 100), dtype=np.float32)).to("cuda:0")
                     for _ in range(3))
        pm = None
        if os.environ.get("ZV_PROBE_RAGGED") == "1":
            lens = (T * rng.uniform(0.6, 1.0, B)).astype(int)
            lens[0] = T
            pm = torch.from_numpy(np.arange(T)[None, :] >= lens[:, None]).to("cuda:0")
        for t in (0.1, 0.5, 0.9):
            m.engine.attn_fallbacks(reset=True)
            m.engine.velocity(t, 1.0, x, tc, sc, pm)
            print(f"{mode} T={T} B={B} t={t}: exact-path runs (low, high, all) = "
                  f"{m.engine.attn_fallbacks(reset=True)}", flush=True)
    del m
    torch.cuda.empty_cache()
