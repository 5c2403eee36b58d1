#!/usr/bin/env python3
"""Single-sentence latency (the reference CLI's case: one sentence per call,
infer_zipvoice.py:568-577): ZipVoice sample() + vocoder for B=1, 3 s prompt,
~1.5 s generated (T=422 as config C1) and a 10 s sentence, N=16 steps."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from zipvoice_amd.config import default_config  # noqa: E402
from zipvoice_amd.models import build_model  # noqa: E402
from zipvoice_amd.vocoder import Vocos  # noqa: E402
from zipvoice_amd.weights import synthetic_state_dict  # noqa: E402

prec = sys.argv[1] if len(sys.argv) > 1 else "bf16"
cfg = default_config("zipvoice")
m = build_model(cfg, precision=prec)
m.load_state_dict(synthetic_state_dict(cfg, 0))
m = m.to("cuda:0")
voc = Vocos().load_synthetic(0).to("cuda:0")
rng = np.random.default_rng(0)
for S_t, T_g in ((20, 141), (134, 938)):
    toks = [[int(v) for v in rng.integers(1, 360, S_t)]]
    ptoks = [[int(v) for v in rng.integers(1, 360, 40)]]
    pf = torch.from_numpy((0.3 * rng.standard_normal((1, 281, 100)) - 0.5).astype(np.float32)).cuda()
    pl = torch.tensor([281], device="cuda")
    fl = torch.tensor([T_g], device="cuda")

    def step():
        gen, gl, _, _ = m.sample(tokens=toks, prompt_tokens=ptoks, prompt_features=pf,
                                 prompt_features_lens=pl, features_lens=fl, duration="real",
                                 num_step=16, guidance_scale=1.0, t_shift=0.5)
        return voc.decode_features(gen, gl)
    for _ in range(2):
        step()
    torch.cuda.synchronize()
    n = 10
    t0 = time.perf_counter()
    for _ in range(n):
        step()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / n
    print(f"[{prec}] B=1 T={281 + T_g} N=16: {dt * 1e3:.2f} ms per sentence "
          f"(RTF {dt / (T_g * 256 / 24000):.5f})", flush=True)
